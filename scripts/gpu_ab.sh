#!/bin/bash
# A/B of bench.py argument sets (one line each in $1, default scripts/ab_args.txt), AR decode only.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
f=${1:-scripts/ab_args.txt}
: > gpurun_out/ab.log
while read -r a; do
  [ -z "$a" ] && continue
  echo "== $a" >> gpurun_out/ab.log
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --kokoro-prompts 0 $a >> gpurun_out/ab.log 2>&1 || { echo "FAILED: $a"; exit 1; }
done < "$f"
python3 - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("=="): print(l.strip())
    elif l.startswith("{"):
        d=json.loads(l); print("  value", d["value"], "ar_ms", d.get("ar_ms_per_step"), "ar", d.get("ar_audio_sec_per_s"), "dac", d.get("dac_audio_sec_per_s"), "host", d.get("host_us_per_step"))
PY
