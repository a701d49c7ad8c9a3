#!/bin/bash
# Kernel trace of the 64-prompt AR step: one replica of B prompts (default 32, half the set), AR only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/b64prof; mkdir -p $O; cd $R
B=${B:-32}
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --batch $B --replicas 1 --steps ${STEPS:-30}"
timeout -k 10 200 python3 bench.py $AR > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'], 'prefill', d['prefill_ms'])" $O/plain.log
cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $AR > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/prof_summary.py $f k_attn k_gemv > $O/summary.txt; head -60 $O/summary.txt
