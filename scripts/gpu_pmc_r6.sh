#!/bin/bash
# Round 6 evidence: HBM traffic of the headline K-relay GEMM and of the decode
# attention pair at KV 448 (the headline's KV length), and of Dia's slab Q8_0 GEMV; two separate
# counter passes each (FETCH_SIZE and WRITE_SIZE cannot share the TCC slots), kernel trace + stats only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-dac --graphs 0 --no-prefill --ctx 448 --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0 --sampled-steps 0 --prompt-pass 0"
D="python3 bench.py --steps 2 --warmup 1 --prompts 2 --replicas 1 --no-cpu-baseline --no-dac --graphs 0 --no-prefill --ctx 16 --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 16 --b1-replicas 0 --p8 0 --sampled-steps 0 --prompt-pass 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc6_fetch -o run --output-format csv -- $B > gpurun_out/pmc6_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmc6_write -o run --output-format csv -- $B > gpurun_out/pmc6_write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc6d_fetch -o run --output-format csv -- $D > gpurun_out/pmc6d_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/pmc6d_write -o run --output-format csv -- $D > gpurun_out/pmc6d_write.log 2>&1
rc=$?
echo "pmc rc $rc"; tail -3 gpurun_out/pmc6_fetch.log; tail -2 gpurun_out/pmc6d_fetch.log
exit $rc
