#!/bin/bash
# Full GPU parity suite, then a short bench (all legs) for the per-leg numbers.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline > gpurun_out/sb.log 2>&1 || exit 1
tail -1 gpurun_out/sb.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ar_ms', d['ar_ms_per_step'], 'dac', d['dac_audio_sec_per_s'], 'kokoro', d['kokoro']['audio_sec_per_s'], 'orpheus_ms', d['orpheus']['ms_per_step'], 'dia_ms', d['dia']['ms_per_step'])"
