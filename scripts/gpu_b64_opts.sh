#!/bin/bash
# 64-prompt AR line (1 replica x 64) under bench option sets: OPTS="name1:--flag v|name2:..." 
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/b64opts; mkdir -p $O; cd $R
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --batch 64 --replicas ${REPL:-1} --steps ${STEPS:-40}"
IFS='|' read -ra SETS <<< "$OPTS"
for s in "${SETS[@]}"; do
  name=${s%%:*}; flags=${s#*:}
  timeout -k 10 240 python3 bench.py $AR $flags > $O/$name.log 2>&1 || { echo "$name failed"; tail -3 $O/$name.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'])" $O/$name.log $name
done
