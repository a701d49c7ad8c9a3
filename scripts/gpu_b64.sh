#!/bin/bash
# The 64-prompt set on one GPU: AR-only lines at R replicas x 64/R prompts, then one AR + DAC line.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/b64; mkdir -p $O; cd $R
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --batch 64"
for r in ${REPS:-2 4 1}; do
  timeout -k 10 240 python3 bench.py $AR --steps ${STEPS:-100} --replicas $r > $O/ar_$r.log 2>&1 || { tail -5 $O/ar_$r.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('replicas', sys.argv[2], 'ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'], 'gemv_us', d['roofline']['avg_launch_us'], 'prefill', d['prefill_ms']['per_replica'])" $O/ar_$r.log $r
done
if [ -n "$DAC" ]; then
  timeout -k 10 300 python3 bench.py --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --batch 64 --steps 20 --replicas ${DACREP:-2} > $O/e2e.log 2>&1 || { tail -5 $O/e2e.log; exit 1; }
  tail -1 $O/e2e.log | cut -c1-700
fi
