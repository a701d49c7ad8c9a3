#!/bin/bash
# Short-context attention with double-buffered V batches: attention / Parler / Orpheus / Dia parity,
# Orpheus decode, Orpheus kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attn_gpu.py tests/test_parler_gpu.py tests/test_orpheus_gpu.py \
    tests/test_dia_gpu.py tests/test_fusion_gpu.py > gpurun_out/as_tests.log 2>&1
rc=$?
tail -2 gpurun_out/as_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/as_orph.log 2>&1 || exit 1
tail -1 gpurun_out/as_orph.log | cut -c1-200
bash scripts/gpu_orph_trace.sh
