#!/bin/bash
# HBM traffic of the Q4_K GEMV: two separate counter passes (FETCH_SIZE and WRITE_SIZE cannot share
# the TCC slots), kernel trace + stats only -- no sys/runtime trace domains with --pmc.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# --ctx 16: a 448-token prefill (56 column chunks per GEMV job) crashes the counter-collection
# tool inside its dispatch intercept; the GEMV's decode traffic does not depend on the KV length.
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1 &&
python3 scripts/pmc_gemv.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_gemv_q4k.json
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pmc_fetch.log
exit $rc
