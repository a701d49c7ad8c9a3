#!/bin/bash
# Parler AR decode only: HIP runtime kernarg / graph-packet settings vs the step time.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
A="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --steps 200"
for env in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_USE_FGS_KERNARG=1" "ROC_USE_FGS_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "X=1"; do
  n=$(echo $env | tr -d '=_')
  env $env timeout -k 10 200 python3 bench.py $A > gpurun_out/r3/ka_$n.log 2>&1 || { echo "FAIL $env"; tail -3 gpurun_out/r3/ka_$n.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r3/ka_$n.log').read().strip().splitlines()[-1]);print('$env', d['ar_ms_per_step'], d['ar_audio_sec_per_s'], d['roofline']['avg_launch_us'])"
done
