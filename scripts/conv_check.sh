#!/bin/bash
# Conv-kernel change check: conv / DAC / Kokoro / audio GPU parity, one 20-frame DAC decode, the
# driver's short line with the Kokoro leg, and the conv kernels' register use under the tracer.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_dac_gpu.py tests/test_kokoro_model_gpu.py tests/test_audio_gpu.py > gpurun_out/t_conv.log 2>&1 && tail -1 gpurun_out/t_conv.log &&
timeout -k 10 120 python3 scripts/dac_host_probe.py 20 > gpurun_out/dp.log 2>&1 && grep frames gpurun_out/dp.log &&
timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --kokoro-prompts 8 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 > gpurun_out/bs.log 2>&1 &&
tail -1 gpurun_out/bs.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('short line', d['value'], 'AR ms', d['ar_ms_per_step'], 'DAC', d['dac_audio_sec_per_s'], 'kokoro', d['kokoro']['audio_sec_per_s'])" &&
bash scripts/dac1_trace.sh 20 > /dev/null && python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/study/profd1/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps = [i for i in range(1, len(rows)) if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 300000]
d = rows[gaps[-1]:]
agg = collections.Counter(); vg = {}
for r in d:
    n = r["Kernel_Name"].split("(")[0]
    agg[n.split("<")[0][-24:]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "conv" in n: vg[n[-40:]] = (r["VGPR_Count"], r["Scratch_Size"])
print("one decode, device us by kernel:", {k: round(v, 1) for k, v in agg.most_common(6)})
print("VGPRs:", vg)
PY
