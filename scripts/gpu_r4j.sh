#!/bin/bash
# attention parity, then the Dia leg alone (its 1024-position cross-attention has 32 rows)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r4j
timeout -k 10 300 python -u -m pytest tests/test_attn_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/tests.log 2>&1 || { tail -20 gpurun_out/r4j/tests.log; exit 1; }
tail -1 gpurun_out/r4j/tests.log
timeout -k 10 300 python3 bench.py --steps 5 --no-dac --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --b1-replicas 0 --p8 0 > gpurun_out/r4j/dia.log 2>&1 || { tail -5 gpurun_out/r4j/dia.log; exit 1; }
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['dia'];print('dia ms/step', d['ms_per_step'], 'audio/s', d['audio_sec_per_s'])" gpurun_out/r4j/dia.log
