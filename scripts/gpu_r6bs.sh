#!/bin/bash
# Host waits on a blocking-sync event (TTS_HIP_BLOCKING_SYNC=1, the thread sleeps) vs the stream's own
# synchronize (polling), alternating processes: the B = 1 legs (8 and 32 runner threads), then the short
# headline line's AR leg.  (The toggle was removed after this comparison: profiles/r06/ab_blocking_sync.log.)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2 3; do
  for v in poll block; do
    if [ $v = block ]; then export TTS_HIP_BLOCKING_SYNC=1; else unset TTS_HIP_BLOCKING_SYNC; fi
    timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
      --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6bs_${v}_$i.json 2> gpurun_out/r6bs_${v}_$i.err
    rc=$?; echo "$v $i rc $rc"; [ $rc -eq 0 ] || exit $rc
    python3 -c "
import json;d=json.loads(open('gpurun_out/r6bs_${v}_$i.json').read().splitlines()[-1]);b=d['parler_b1']
print('$v', 'AR ms/step %.3f' % d['ms_per_step'], ' '.join('%s %.3f set %.0f' % (k, v['ms_per_step'], v['coalescer']['runner0_host_us_per_step']['set_inputs']) for k,v in b.items()))"
  done
done
