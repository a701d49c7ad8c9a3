#!/bin/bash
# Re-entry check: full GPU parity suite, then the K-split GEMV study (scripts/gpu_ks.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ks.sh
