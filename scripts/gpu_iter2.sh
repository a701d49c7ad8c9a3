#!/bin/bash
# Full GPU parity suite, then bench A/B lines from scripts/ab_args.txt (AR + DAC, no Kokoro, no CPU leg).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash scripts/gpu_ab.sh
