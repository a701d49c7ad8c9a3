#!/bin/bash
# in-graph per-kernel durations of the Parler decode step (B=8, 1 replica), GEMV kernel A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for u in ${UVALS:-0 1}; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tr_u$u -o tr --output-format csv -- python3 $R/bench.py --steps 30 --warmup 2 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --batch 8 --replicas 1 --gemv-unique $u $EXTRA > $R/gpurun_out/tr_u$u.log 2>&1 || exit 1
f=$(find $R/gpurun_out/tr_u$u -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py $f 6 20 4608 > $R/gpurun_out/tr_u$u.txt
head -16 $R/gpurun_out/tr_u$u.txt
done
