#!/bin/bash
# K-relay column-pair / XCD variants (parity), the B=1 legs with host-time counters, interleaved A/B of the
# variants on the 64-prompt step, then the round-6 PMC passes (K-relay + attention at KV 448, Dia slab GEMV)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemv_gpu.py tests/test_parler_gpu.py -k "column_pairs or many_prompt" -x -q --timeout 200 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r6e_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6e_b1.json 2> gpurun_out/r6e_b1.err
rc=$?; echo "b1 rc $rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/r6e_b1.json').read().splitlines()[-1]);b=d['parler_b1']
for k,v in b.items(): print(k, v['ms_per_step'], v['ar_audio_sec_per_s'], json.dumps(v['coalescer']))"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_ar.py --blocks 5 --steps 12 base=GEMM_KR_XCD:1,GEMM_KR_CP:0 noxcd=GEMM_KR_XCD:0,GEMM_KR_CP:0 cp=GEMM_KR_XCD:1,GEMM_KR_CP:1 > gpurun_out/r6e_ab.log 2>&1
rc=$?; echo "ab rc $rc"; tail -4 gpurun_out/r6e_ab.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_r6.sh
