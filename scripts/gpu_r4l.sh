#!/bin/bash
# two column tiles per K-relay workgroup: parity, then interleaved A/B on the 64-prompt step
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemv_gpu.py tests/test_parler_gpu.py -x -q -k "two_column or many_prompt" --timeout 400 --timeout-method thread > gpurun_out/ct2_test.log 2>&1 || { tail -30 gpurun_out/ct2_test.log; exit 1; }
tail -1 gpurun_out/ct2_test.log
timeout -k 10 300 python3 scripts/ab_ar.py --ctx 448 a=GEMM_KR_CT2:0 ct2=GEMM_KR_CT2:1 > gpurun_out/ab_ct2.log 2>&1 || { tail -5 gpurun_out/ab_ct2.log; exit 1; }
grep '^{' gpurun_out/ab_ct2.log | cut -c1-160
timeout -k 10 300 python3 scripts/ab_ar.py --ctx 448 all=FUSION:16383 noxattn=FUSION:14335 > gpurun_out/ab_xattn.log 2>&1 || { tail -5 gpurun_out/ab_xattn.log; exit 1; }
grep '^{' gpurun_out/ab_xattn.log | cut -c1-160
