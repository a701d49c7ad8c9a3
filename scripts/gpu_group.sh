#!/bin/bash
# Look-ahead GEMV grouping (gate + up): full GPU suite, Orpheus decode, Orpheus kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/grp_orph.log 2>&1 || exit 1
tail -1 gpurun_out/grp_orph.log | cut -c1-300
bash scripts/gpu_orph_trace.sh
