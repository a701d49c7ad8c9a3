#!/bin/bash
# A/B bench variants in one box session: each line of args runs one bench
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
: > gpurun_out/ab.log
while IFS= read -r line; do
  [ -z "$line" ] && continue
  echo "== $line" >> gpurun_out/ab.log
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $line >> gpurun_out/ab.log 2>&1 || { echo "FAILED rc=$?" >> gpurun_out/ab.log; break; }
done < "${1:-scripts/ab_args.txt}"
cat gpurun_out/ab.log | cut -c1-400
