#!/bin/bash
# Parler AR decode only: CU-mask placement probe, bench lines over replica / CU-partition settings,
# and a kernel trace of the 2-replica run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 60 ./scripts/bin/cumask_probe > gpurun_out/r3/cumask_probe.log 2>&1; cat gpurun_out/r3/cumask_probe.log
A="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --steps 200"
for cfg in "--replicas 1" "--replicas 2" "--replicas 2 --cu-partition 1" "--replicas 2 --cu-partition 2" "--replicas 4" "--replicas 4 --cu-partition 1" "--replicas 4 --cu-partition 2" "--replicas 8 --cu-partition 1"; do
  n=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python3 bench.py $A $cfg > gpurun_out/r3/pp_$n.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/r3/pp_$n.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r3/pp_$n.log').read().strip().splitlines()[-1]);print('$cfg', d['ar_ms_per_step'], d['ar_audio_sec_per_s'], d['roofline']['avg_launch_us'])"
done
