#!/bin/bash
# The rocprofv3 kernel tracer over HIP-graph replay with the runtime's packet capture ON (the default;
# round 3 saw the tracer fault here and traced with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).  One short run,
# its whole log kept (gpurun_out/tracer/), the exit status printed; nothing runs on the GPU after it.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tracer; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# TRACER_FULL=1: the evidence run's command (every leg, 64 prompts, DAC, Orpheus, Dia)
if [ -n "$TRACER_FULL" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/full -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 \
    --no-cpu-baseline --orpheus-steps 16 --dia-steps 24 $TRACER_EXTRA > $O/full.log 2>&1
  rc=$?
  echo "tracer (packet capture on, full bench) rc $rc"
  tail -5 $O/full.log | cut -c1-400
  exit 0
fi
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/on -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 \
  --prompts 8 --replicas 2 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0 --no-cpu-baseline > $O/on.log 2>&1
rc=$?
echo "tracer (packet capture on) rc $rc"
tail -25 $O/on.log
exit 0
