#!/bin/bash
# Residue-split GEMV with a deeper chunk pipeline: parity, phase study (Orpheus shapes), Orpheus decode.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orpheus_gpu.py tests/test_gemv_gpu.py > gpurun_out/oq_tests.log 2>&1
rc=$?
tail -1 gpurun_out/oq_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_orph_phase.sh || exit 1
timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/oq_orph.log 2>&1 || exit 1
tail -1 gpurun_out/oq_orph.log | cut -c1-200
