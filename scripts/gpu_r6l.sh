#!/bin/bash
# K-relay column-tile pairs on one XCD with L2-allocating weight loads (TTS_HIP_OPT_GEMM_KR_XCD = 1):
# parity, interleaved A/B against the grid order, then FETCH_SIZE / WRITE_SIZE of the XCD form.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gemv_gpu.py::test_q4_K_prefill_gemm_column_pairs" "tests/test_parler_gpu.py::test_many_prompt_step_in_kernel_operands" > gpurun_out/r6l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/ab_ar.py --blocks 5 --steps 12 base=GEMM_KR_XCD:0 xcd=GEMM_KR_XCD:1 > gpurun_out/r6l_ab.log 2>&1
rc=$?; cat gpurun_out/r6l_ab.log | grep variant; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-dac --graphs 0 --no-prefill --ctx 448 --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0 --sampled-steps 0 --prompt-pass 0 --gemm-kr-xcd 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc6x_fetch -o run --output-format csv -- $B > gpurun_out/pmc6x_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmc6x_write -o run --output-format csv -- $B > gpurun_out/pmc6x_write.log 2>&1
rc=$?; echo "pmc rc $rc"; tail -2 gpurun_out/pmc6x_fetch.log
rm -f gpurun_out/pmc6x_*/run_kernel_trace.csv
exit $rc
# the batched prompt pass's kernels: 1 warm + 4 traced passes of 32 ragged prompts, packet capture off
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_trace -o run --output-format csv -- python3 scripts/prompt_pass_probe.py 32 4 1 > gpurun_out/pp_trace.log 2>&1
rc=$?; echo "pp trace rc $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pp_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$f" k_gemv_q4K_kr k_attn k_bgemm > gpurun_out/pp_summary.txt; head -45 gpurun_out/pp_summary.txt
