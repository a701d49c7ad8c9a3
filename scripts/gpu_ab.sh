#!/bin/bash
# interleaved A/B studies of the 64-prompt AR step (scripts/ab_ar.py); AB_RUNS: "args;args;..."
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/ab; mkdir -p $O
IFS=';' read -ra RUNS <<< "$AB_RUNS"
i=0
for r in "${RUNS[@]}"; do
  timeout -k 10 300 python3 scripts/ab_ar.py $r > $O/ab_$i.log 2>&1 || { tail -5 $O/ab_$i.log; exit 1; }
  echo "== $r"; grep '^{' $O/ab_$i.log | cut -c1-200
  i=$((i+1))
done
