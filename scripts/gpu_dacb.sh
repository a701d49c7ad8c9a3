#!/bin/bash
# batched DAC decode: parity tests, then the 64-prompt short bench line with batching on / off
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dacb; mkdir -p $O; cd $R
[ -n "$NO_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_dac_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -1 $O/tests.log
# VARIANTS: "name:flags|name:flags|..."
IFS='|' read -ra VS <<< "${VARIANTS:-b8:--dac-batch 8|b8w4:--dac-batch 8 --dac-workers 4|b4:--dac-batch 4|b1:--dac-batch 1}"
[ -n "$NO_TESTS" ] || true
for v in "${VS[@]}"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python3 bench.py --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --p8 0 --steps ${STEPS:-20} $f > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'value', d['value'], 'ar', d['ar_audio_sec_per_s'], 'dac', d['dac_audio_sec_per_s'], d['config']['parallelism'])" $O/$n.log $n
done
