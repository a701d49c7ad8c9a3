#!/bin/bash
# Round 6: coalescer v2 tests (with refusal diagnostics), ragged lock-step batches, the whole GPU suite,
# then the B=1 / prompt-pass bench legs.
cd $GRAFT_REPO_ROOT
TTS_HIP_COALESCE_DEBUG=1 timeout -k 10 400 python -u -m pytest tests/test_coalesce_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r6d_coal.log 2>&1
rc=$?; echo "coal rc $rc"; grep -m 10 "coalesce:" gpurun_out/r6d_coal.log; tail -15 gpurun_out/r6d_coal.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_parler_gpu.py -k ragged -x -v --timeout 200 --timeout-method thread > gpurun_out/r6d_ragged.log 2>&1
rc=$?; echo "ragged rc $rc"; tail -8 gpurun_out/r6d_ragged.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d_suite.log 2>&1
rc=$?; echo "suite rc $rc"; tail -3 gpurun_out/r6d_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --no-cpu-baseline > gpurun_out/r6d_bench_b1.json 2> gpurun_out/r6d_bench_b1.err
rc=$?; echo "bench rc $rc"; tail -c 4000 gpurun_out/r6d_bench_b1.json; tail -5 gpurun_out/r6d_bench_b1.err
exit $rc
