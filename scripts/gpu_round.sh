#!/bin/bash
# Round-end evidence: GPU parity suite, smoke, default bench (with CPU baseline), kernel-trace stats of a
# short bench, PMC HBM-traffic passes of the dominant kernels.  Every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench_full.log gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log
# graph replay under the kernel tracer needs the runtime's packet-capture path off (the tracer faults
# walking captured packets; kernel durations are unaffected)
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --orpheus-steps 16 --dia-steps 16 > $R/gpurun_out/prof.log 2>&1 || exit 1
cd $R
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 &&
bash scripts/gpu_pmc_orpheus.sh > gpurun_out/pmc_orpheus.log 2>&1
rc=$?
tail -1 gpurun_out/bench20.log | cut -c1-400
exit $rc
