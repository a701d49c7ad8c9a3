#!/bin/bash
# Coalescer pre-fence: skip members whose stream has drained (default) vs fence every member
# (TTS_CO_FENCE_ALL=1), alternating processes; the coalescer tests first (ab_co_prefence_skip.log).
# ab_co_postfence_member_vs_leader.log came from a variant of this loop over a since-removed toggle
# (the post-fence in each member's thread vs the leader's).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_coalesce_gpu.py tests/test_adapter_gpu.py > gpurun_out/r6fe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6fe_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in skip all; do
    if [ $v = all ]; then export TTS_CO_FENCE_ALL=1; else unset TTS_CO_FENCE_ALL; fi
    timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
      --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6fe_${v}_$i.json 2> gpurun_out/r6fe_${v}_$i.err
    rc=$?; echo "$v $i rc $rc"; [ $rc -eq 0 ] || exit $rc
    python3 -c "
import json;d=json.loads(open('gpurun_out/r6fe_${v}_$i.json').read().splitlines()[-1]);b=d['parler_b1']
print('$v', ' '.join('%s %.3f exec %.0f' % (k, v['ms_per_step'], v['coalescer']['host_us_per_launch']['exec_us']) for k,v in b.items()))"
  done
done
