#!/bin/bash
# The rocprofv3 kernel tracer over HIP-graph replay with the runtime's packet capture ON (the default;
# round 3 saw the tracer fault here and traced with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).  One run, its whole
# log kept (gpurun_out/tracer/), the exit status printed; nothing runs on the GPU after it.
# TTS_HIP_CRASH_HANDLER=1: a fault prints its address, every frame as library + offset and the mappings
# around the address (tts_hip_install_crash_handler); the frames are symbolized here afterwards.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tracer; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export TTS_HIP_CRASH_HANDLER=1
STEPS=${TRACER_STEPS:-80}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/on -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 2 \
  --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0 --sampled-steps 0 --prompt-pass 0 \
  --no-cpu-baseline $TRACER_EXTRA > $O/on.log 2>&1
rc=$?
echo "tracer (packet capture on, $STEPS steps) rc $rc"
grep -A80 "tts_hip: signal" $O/on.log | grep -E "^  #" | while read -r n addr where sym; do
  lib=${where%+0x*}; off=${where##*+}
  [ -f "$lib" ] && echo "$n $where $sym -> $(/opt/rocm/lib/llvm/bin/llvm-symbolizer --obj="$lib" "$off" 2>/dev/null | head -2 | tr '\n' ' ')"
done > $O/frames.txt
grep -B2 -A40 "tts_hip: signal" $O/on.log | head -80
cat $O/frames.txt
exit 0
