#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_orpheus_gpu.py tests/test_attn_gpu.py > gpurun_out/a128_tests.log 2>&1
rc=$?
tail -2 gpurun_out/a128_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/a128_orph.log 2>&1 || exit 1
tail -1 gpurun_out/a128_orph.log | cut -c1-200
bash scripts/gpu_orph_trace64.sh | grep -E "per step|attn"
