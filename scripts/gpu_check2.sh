#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash scripts/gpu_orph_quick.sh > gpurun_out/c2_orph.txt 2>&1 || { tail -5 gpurun_out/c2_orph.txt; exit 1; }
tail -1 gpurun_out/oq_tests.log; tail -1 gpurun_out/oq_orph.log | cut -c1-200
bash scripts/gpu_ar_quick.sh
