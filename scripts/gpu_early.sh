#!/bin/bash
# GEMV early-load change: parity, micro-benchmark, AR step time
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gemv_gpu.py tests/test_parler_gpu.py tests/test_fusion_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_early.log 2>&1 || { tail -20 gpurun_out/pytest_early.log; exit 1; }
tail -1 gpurun_out/pytest_early.log
timeout -k 10 120 python3 scripts/bench_gemv.py 30 1,4,8 0 parler_fc2,parler_qkvo,orpheus_down > gpurun_out/gemv_early.jsonl 2>&1 && cut -c1-160 gpurun_out/gemv_early.jsonl
for r in 1 2; do
timeout -k 10 200 python3 bench.py --steps 200 --warmup 3 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 --replicas $r > gpurun_out/early_ar_$r.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/early_ar_$r.log').read().strip().splitlines()[-1]); print('replicas $r ar_ms', d['ar_ms_per_step'], d['roofline']['avg_launch_us'])"
done
