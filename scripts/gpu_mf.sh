#!/bin/bash
# Matrix-core Q4_K GEMV: parity tests, then the GEMV micro-benchmark (VALU lane layout vs tile layout)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gemv_gpu.py tests/test_orpheus_gpu.py tests/test_parler_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "mfma or orpheus" > gpurun_out/pytest_mf.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_mf.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_mf.log | head -20; exit $rc; }
S=orpheus_up,orpheus_down,orpheus_head,parler_fc1,parler_qkvo
timeout -k 10 200 python3 scripts/bench_gemv.py 20 1,8,16 0 $S > gpurun_out/gemv_valu.jsonl 2>&1 &&
timeout -k 10 200 python3 scripts/bench_gemv.py 20 1,8,16 1 $S > gpurun_out/gemv_tiled.jsonl 2>&1
rc=$?
cat gpurun_out/gemv_valu.jsonl gpurun_out/gemv_tiled.jsonl | cut -c1-200
exit $rc
