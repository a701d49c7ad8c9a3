#!/bin/bash
# Round-3 start: smoke, short bench line, kernel-trace stats of the same short bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py --steps 200 --no-cpu-baseline > gpurun_out/r3/bench.log 2>&1 || { tail -5 gpurun_out/r3/*.log; exit 1; }
tail -1 gpurun_out/r3/bench.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --orpheus-steps 16 --dia-steps 16 > $R/gpurun_out/r3/prof.log 2>&1
