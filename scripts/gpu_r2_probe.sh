#!/bin/bash
# round-2 first probe: DAC decode cost at short / long lengths, AR step kernel breakdown (B=8, 1 replica)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/bench_dac.py 20 861 > gpurun_out/dac_bench.jsonl 2>&1 || { cat gpurun_out/dac_bench.jsonl; exit 1; }
cat gpurun_out/dac_bench.jsonl
bash scripts/gpu_prof_ar.sh 8 448
