#!/bin/bash
# K-split matrix-core GEMV (k_gemv_q4K_ks): parity tests, in-chain timing vs the other Q4_K kernels,
# Parler AR decode with every Q4_K matrix tiled vs the default layout.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemv_gpu.py -k "mfma" \
    tests/test_parler_gpu.py::test_full_parler_mini_q4k_tokens_mfma > gpurun_out/ks_tests.log 2>&1
rc=$?
tail -3 gpurun_out/ks_tests.log
[ $rc -ne 0 ] && exit $rc
GEMV_PHASE_TILED=1 timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/ks_phase.jsonl 2>&1 &&
GEMV_PHASE_TILED=1 GEMV_KS=0 timeout -k 10 120 scripts/bin/gemv_phase > gpurun_out/mf_phase.jsonl 2>&1 || exit 1
python3 - <<'EOF'
import json
for f in ("gpurun_out/ks_phase.jsonl", "gpurun_out/mf_phase.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1][:2], d["shape"], "chain", d["chain_us"], "event", d["event_us"])
EOF
for tb in 1 4194304; do
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-dac --kokoro-prompts 0 --orpheus-steps 0 \
    --dia-steps 0 --tile-bytes $tb "$@" > gpurun_out/ks_bench_$tb.log 2>&1 || exit 1
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ks_bench_$tb.log').read().strip().splitlines()[-1])
print('tile_bytes $tb', 'ar_ms_per_step', d['ar_ms_per_step'], 'ar', d['ar_audio_sec_per_s'], 'gemv', d['roofline'])"
done
