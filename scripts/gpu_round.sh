#!/bin/bash
# Round-end evidence: GPU parity suite, smoke, default bench (with CPU baseline), the driver's short
# bench, kernel-trace stats of a short bench, PMC HBM-traffic passes of the decode step's dominant
# kernels (the K-relay GEMM at 32 lock-step prompts per replica, the attention pair) and of the Orpheus
# leg's matrix-core GEMV.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python3 bench.py > $O/bench_full.log 2>&1 &&
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -5 $O/pytest_gpu.log $O/smoke.log $O/bench_full.log $O/bench20.log; exit 1; }
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
# graph replay under the kernel tracer needs the runtime's packet-capture path off
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --orpheus-steps 16 --dia-steps 24 > $O/prof.log 2>&1 || exit 1
cd $R
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
# PMC passes (one counter group each, kernel trace only): the 64-prompt decode step at a short KV (a
# 448-token prompt pass crashes the counter tool in its dispatch intercept; decode traffic per launch
# does not depend on the KV length for the GEMMs, the attention bytes scale with it)
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 --p8 0"
CMD="rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-dac --graphs 0 --ctx 16 (64 prompts, 2 replicas x 32; last profiled decode dispatches)"
cd /tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1 || exit 1
cd $R
N=$(python3 -c "import json;print([json.loads(l) for l in open('$O/pmc_fetch.log') if l.startswith('{')][-1]['roofline']['launches_sampled'])")
python3 scripts/pmc_gemv.py $O/pmc_fetch $O/pmc_write $O/pmc_gemv_q4k.json k_gemv_q4K_kr $N "$CMD" > /dev/null &&
python3 scripts/pmc_gemv.py $O/pmc_fetch $O/pmc_write $O/pmc_attn.json k_attn_ 240 "$CMD" > /dev/null || exit 1
bash scripts/gpu_pmc_orpheus.sh > $O/pmc_orpheus.log 2>&1
rc=$?
tail -1 $O/bench20.log | cut -c1-600
exit $rc
