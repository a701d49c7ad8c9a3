#!/bin/bash
# The kernel tracer over the driver's short bench line, packet capture OFF, crash handler on: the round-6 bench
# faulted under the tracer inside the generate()-shape leg (tts_parler_generate -> tts_hip_graph_launch).  One
# run; the handler's frames (library + offset) are symbolized here afterwards.  Nothing runs on the GPU after it.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tracer20; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export TTS_HIP_CRASH_HANDLER=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/run -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --b1-wide 0 --sampled-steps 0 $TRACER_EXTRA > $O/run.log 2>&1
rc=$?
echo "tracer bench20 (packet capture off) rc $rc"
grep -A80 "tts_hip: signal" $O/run.log | grep -E "^  #" | while read -r n addr where sym; do
  lib=${where%+0x*}; off=${where##*+}
  [ -f "$lib" ] && echo "$n $where $sym -> $(/opt/rocm/lib/llvm/bin/llvm-symbolizer --obj="$lib" "$off" 2>/dev/null | head -2 | tr '\n' ' ')"
done > $O/frames.txt
grep -B2 -A40 "tts_hip: signal" $O/run.log | head -80
cat $O/frames.txt
exit 0
