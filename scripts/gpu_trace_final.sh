#!/bin/bash
# kernel trace + stats of the short bench on the final tree (graph packet capture off: DESIGN §6)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/trace_final; mkdir -p $O
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --orpheus-steps 16 --dia-steps 24 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | tail -1 | cut -c1-200
