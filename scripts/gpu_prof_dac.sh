#!/bin/bash
# DAC-44k decode throughput and kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 scripts/bench_dac.py 50 861 > gpurun_out/dac_bench.jsonl 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profd -o run --output-format csv -- python3 scripts/bench_dac.py 50 > gpurun_out/profd.log 2>&1
rc=$?
cat gpurun_out/dac_bench.jsonl
exit $rc
