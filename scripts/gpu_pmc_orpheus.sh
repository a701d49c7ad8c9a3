#!/bin/bash
# HBM traffic of the K-relay matrix-core Q4_K GEMV on the Orpheus leg (8 prompts, M = 8): two separate
# counter passes, kernel trace + stats only.  The Parler leg is cut to one short step; the last
# 8 x 112 k_gemv_q4K_kr dispatches (28 layers x q/k/v, o, gate/up, down; the profiled decode steps) are kept.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 --kokoro-prompts 0 --dia-steps 0 --b1-replicas 0 --p8 0 --orpheus-steps 8"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmco_fetch -o run --output-format csv -- $B > gpurun_out/pmco_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmco_write -o run --output-format csv -- $B > gpurun_out/pmco_write.log 2>&1 &&
python3 scripts/pmc_gemv.py gpurun_out/pmco_fetch gpurun_out/pmco_write gpurun_out/pmc_gemv_q4k_kr_orpheus.json k_gemv_q4K_kr 896 \
  "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace --stats -- $B (last 896 k_gemv_q4K_kr dispatches, M = 8)"
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pmco_fetch.log
exit $rc
