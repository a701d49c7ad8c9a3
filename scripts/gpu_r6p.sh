#!/bin/bash
# Coalesced read-back (co_readback): the coalescer tests, then the B = 1 legs (8 and 32 runners).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_coalesce_gpu.py tests/test_adapter_gpu.py > gpurun_out/r6p_tests.log 2>&1
rc=$?; grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/r6p_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6p_b1.json 2> gpurun_out/r6p_b1.err
rc=$?; echo "b1 rc $rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/r6p_b1.json').read().splitlines()[-1]);b=d['parler_b1']
for k,v in b.items(): print(k, v['ms_per_step'], v['ar_audio_sec_per_s'], json.dumps(v['coalescer']))"
exit $rc
