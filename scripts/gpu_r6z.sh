#!/bin/bash
# Coalescer with members' pre-plans: its tests, then the B = 1 legs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_coalesce_gpu.py tests/test_adapter_gpu.py > gpurun_out/r6z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6z_b1.json 2> gpurun_out/r6z_b1.err
rc=$?; echo "b1 rc $rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/r6z_b1.json').read().splitlines()[-1]);b=d['parler_b1']
for k,v in b.items(): print(k, v['ms_per_step'], v['ar_audio_sec_per_s'], json.dumps(v['coalescer']))"
exit $rc
