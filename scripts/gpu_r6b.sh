#!/bin/bash
# Round 6: the step coalescer without VMM (executor-owned intermediates, per-member tables, ragged KV
# lengths) -- its tests first, then the whole GPU suite with the coalescer on by default, then the B=1 legs.
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_coalesce_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r6b_coal.log 2>&1
rc=$?; echo "coal rc $rc"; tail -15 gpurun_out/r6b_coal.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b_suite.log 2>&1
rc=$?; echo "suite rc $rc"; tail -3 gpurun_out/r6b_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline > gpurun_out/r6b_bench_b1.json 2> gpurun_out/r6b_bench_b1.err
rc=$?; echo "bench rc $rc"; tail -c 3000 gpurun_out/r6b_bench_b1.json; tail -5 gpurun_out/r6b_bench_b1.err
exit $rc
