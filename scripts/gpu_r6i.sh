#!/bin/bash
# The driver's default bench line, untraced (the traced run faulted inside tts_parler_generate).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TTS_HIP_CRASH_HANDLER=1
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r6i_bench.json 2> gpurun_out/r6i_bench.err
rc=$?; echo "bench rc $rc"; tail -c 3000 gpurun_out/r6i_bench.err; tail -c 2500 gpurun_out/r6i_bench.json
exit $rc
