#!/bin/bash
# SNAC parity on the GPU + Orpheus decode-step kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_snac_gpu.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/t_snac.log 2>&1 || { tail -30 gpurun_out/t_snac.log; exit 1; }
grep -E "snac |passed|failed" gpurun_out/t_snac.log
bash scripts/gpu_orph_trace.sh
