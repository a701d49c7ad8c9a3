#!/bin/bash
# evidence run, then the 64-prompt option study (replicas, xattn fusion, eight-wave GEMM, DAC workers)
bash scripts/gpu_round.sh || exit 1
R=$GRAFT_REPO_ROOT; cd $R
OPTS="r2:--replicas 2|r2_nw8:--replicas 2 --gemm-kr-nw 8|r1:--replicas 1|r2_noxattn:--replicas 2 --fusion-mask 14335|r4:--replicas 4" STEPS=40 timeout -k 10 600 bash scripts/gpu_b64_opts.sh
