#!/bin/bash
# B=1 legs after the group-key fix, the round-6 kernel trace of the short bench, then the tracer
# repro (packet capture on, 80 steps) once with the async-signal-safe crash handler.
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --p8 0 \
  --sampled-steps 0 --prompt-pass 0 --no-cpu-baseline --no-prefill --b1-steps 60 > gpurun_out/r6f_b1.json 2> gpurun_out/r6f_b1.err
rc=$?; echo "b1 rc $rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/r6f_b1.json').read().splitlines()[-1]);b=d['parler_b1']
for k,v in b.items(): print(k, v['ms_per_step'], v['ar_audio_sec_per_s'], json.dumps(v['coalescer']))"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_trace_r6.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_tracer_repro.sh
