#!/bin/bash
# SwiGLU GEMV epilogue: Orpheus / matrix-core GEMV parity, Orpheus decode, kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemv_gpu.py -k "mfma" \
    tests/test_orpheus_gpu.py tests/test_ops_gpu.py > gpurun_out/sw_tests.log 2>&1
rc=$?
tail -3 gpurun_out/sw_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/grp_orph.log 2>&1 || exit 1
tail -1 gpurun_out/grp_orph.log | cut -c1-300
bash scripts/gpu_orph_trace.sh
