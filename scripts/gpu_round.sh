#!/bin/bash
# Round-end evidence: GPU parity suite, smoke, default bench (with CPU baseline), kernel-trace stats of a
# short bench, PMC HBM-traffic passes of the dominant kernel.  Every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --orpheus-steps 16 --dia-steps 16 > $R/gpurun_out/prof.log 2>&1 || exit 1
cd $R
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 &&
bash scripts/gpu_pmc_orpheus.sh > gpurun_out/pmc_orpheus.log 2>&1
rc=$?
tail -1 gpurun_out/bench_full.log | cut -c1-400
exit $rc
