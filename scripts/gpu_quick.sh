#!/bin/bash
# Quick loop: GEMV / Parler / Orpheus parity tests, then the AR-only bench line (2 replicas and 1).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quick; mkdir -p $O; cd $R
T="-x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gemv_gpu.py tests/test_parler_gpu.py tests/test_orpheus_gpu.py ${EXTRA_TESTS} $T > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --steps 200"
for r in 2 1; do
  timeout -k 10 200 python3 bench.py $AR --replicas $r > $O/ar_$r.log 2>&1 || { tail -5 $O/ar_$r.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('replicas', sys.argv[2], 'ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'], 'gemv_us', d['roofline']['avg_launch_us'])" $O/ar_$r.log $r
done
if [ -n "$ORPH" ]; then
  timeout -k 10 300 python3 bench.py --no-dac --kokoro-prompts 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --steps 20 --orpheus-steps 64 > $O/orph.log 2>&1 || { tail -5 $O/orph.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['orpheus'];print('orpheus ms', d['ms_per_step'], 'tok/s', d['tokens_per_s'], 'gemv_us', d['roofline']['avg_launch_us'])" $O/orph.log
fi
