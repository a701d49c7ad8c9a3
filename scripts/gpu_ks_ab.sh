#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for ks in 256 0 256 0; do
  TTS_BENCH_KS=$ks timeout -k 10 200 python3 scripts/bench_orpheus.py 8 64 32 > gpurun_out/ksab_$ks.log 2>&1 || exit 1
  echo "ks $ks $(tail -1 gpurun_out/ksab_$ks.log | cut -c1-170)"
done
