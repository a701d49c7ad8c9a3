#!/bin/bash
# Quick loop: named GPU tests, then the 64-prompt AR line (2 replicas x 32).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quick2; mkdir -p $O; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --batch 64 --replicas 2 --steps ${STEPS:-100} $BENCH_EXTRA"
timeout -k 10 240 python3 bench.py $AR > $O/ar.log 2>&1 || { tail -5 $O/ar.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'], 'gemv_us', d['roofline']['avg_launch_us'])" $O/ar.log
