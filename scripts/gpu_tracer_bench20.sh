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
# keep what is judged: the stats, a per-kernel summary and the line; the per-dispatch CSV is too big to bring back
f=$(find $O/run -name "*kernel_trace.csv" | head -1)
if [ -n "$f" ]; then
  python3 $R/scripts/prof_summary.py "$f" k_gemv_q4K_kr k_attn_scores k_attn_pv_mp k_gemv_q8_0s > $O/summary.txt
  head -30 $O/summary.txt
  find $O/run -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
  rm -f "$f"
fi
grep '^{"metric"' $O/run.log > $O/line.json; tail -c 300 $O/line.json
exit 0
