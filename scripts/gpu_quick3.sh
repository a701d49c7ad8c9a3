#!/bin/bash
# Quick loop: named GPU tests, then the 64-prompt AR line at several KV start lengths, pv_mp on / off.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quick3; mkdir -p $O; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for ctx in ${CTXS:-448 1200}; do
  for v in ${VARIANTS:-"mp1:--attn-pv-mp 1" "mp0:--attn-pv-mp 0"}; do
    n=${v%%:*}; f=${v#*:}
    AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --p8 0 --steps ${STEPS:-40} --ctx $ctx $f $BENCH_EXTRA"
    timeout -k 10 300 python3 bench.py $AR > $O/ar_${ctx}_$n.log 2>&1 || { tail -5 $O/ar_${ctx}_$n.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'ar_ms', d['ar_ms_per_step'], 'audio/s', d['ar_audio_sec_per_s'], 'attn', d['roofline'].get('attention'))" $O/ar_${ctx}_$n.log "ctx $ctx $n"
  done
done
