#!/bin/bash
# The measurement studies behind DESIGN.md §7b, one case per study (run on the GPU box through gpurun:
#   gpurun -- scripts/gpu_study.sh <study> [args]).  Every GPU step has its own time limit and the
# steps are chained with &&; results go to gpurun_out/study/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/study
mkdir -p "$O"
cd "$R"
AR="--no-dac --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --steps 200"
T="-x -v --timeout 300 --timeout-method thread"
ar_line() {  # bench.py AR-only line: ms/step, audio-s/s, average GEMV launch, prefill ms per replica
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['ar_ms_per_step'], d['ar_audio_sec_per_s'], d['roofline']['avg_launch_us'], d.get('prefill_ms', {}).get('per_replica'))" "$1" "$2"
}
case "$1" in
  ar)          # Parler AR decode only, bench.py options appended (e.g. --replicas 1)
    shift
    timeout -k 10 200 python3 bench.py $AR "$@" > "$O/ar.log" 2>&1 && ar_line "$O/ar.log" "ar $*" ;;
  replicas)    # runner replicas per GPU (8 prompts)
    for r in 1 2 4 8; do
      timeout -k 10 200 python3 bench.py $AR --replicas $r > "$O/rep_$r.log" 2>&1 && ar_line "$O/rep_$r.log" "replicas $r" || exit 1
    done ;;
  cu_partition)  # replicas on disjoint CU masks (TTS_HIP_OPT_CU_PARTITION) + the mask placement probe
    timeout -k 10 60 ./scripts/bin/cumask_probe > "$O/cumask_probe.log" 2>&1 || exit 1
    for cfg in "--replicas 2" "--replicas 2 --cu-partition 1" "--replicas 2 --cu-partition 2" "--replicas 4" \
               "--replicas 4 --cu-partition 1" "--replicas 4 --cu-partition 2" "--replicas 8 --cu-partition 1"; do
      n=$(echo $cfg | tr -d ' -')
      timeout -k 10 200 python3 bench.py $AR $cfg > "$O/cp_$n.log" 2>&1 && ar_line "$O/cp_$n.log" "$cfg" || exit 1
    done ;;
  kernarg)     # HIP runtime kernarg / graph-packet settings
    for env in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_USE_FGS_KERNARG=1" "ROC_USE_FGS_KERNARG=0" \
               "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
      n=$(echo $env | tr -d '=_')
      env $env timeout -k 10 200 python3 bench.py $AR > "$O/ka_$n.log" 2>&1 && ar_line "$O/ka_$n.log" "$env" || exit 1
    done ;;
  gemv_phase)  # in-kernel phase timestamps of the Parler (or, with ORPHEUS=1, Orpheus) GEMV launches
    E=""; [ -n "$ORPHEUS" ] && E="GEMV_PHASE_ORPHEUS=1 GEMV_PHASE_TILED=1"
    env $E timeout -k 10 120 scripts/bin/gemv_phase > "$O/phase_warm.jsonl" 2>&1 &&
    env $E GEMV_PHASE_COLD=1 timeout -k 10 120 scripts/bin/gemv_phase > "$O/phase_cold.jsonl" 2>&1 && grep '^{' "$O"/phase_*.jsonl ;;
  attn)        # attention parity + micro-benchmark under the kernel trace
    timeout -k 10 300 python -u -m pytest tests/test_attn_gpu.py $T > "$O/pytest_attn.log" 2>&1 &&
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/profa" -o run --output-format csv -- python3 "$R/scripts/bench_attn.py" 30 > "$O/bench_attn.log" 2>&1) &&
    grep '^{' "$O/bench_attn.log" ;;
  dac)         # DAC-44k decode per frame count (default 20 50 861) and its kernel trace at 200 frames
    shift; F="${@:-20 50 861}"
    timeout -k 10 300 python3 scripts/bench_dac.py $F > "$O/dac_bench.jsonl" 2>&1 &&
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/profd" -o run --output-format csv -- python3 "$R/scripts/bench_dac.py" 200 > "$O/profd.log" 2>&1) &&
    cat "$O/dac_bench.jsonl" ;;
  dac_short)   # the driver's short line (20 frames): DAC workers x conv split
    for w in 8 4 2; do for sp in 1 0; do
      timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 \
          --dac-workers $w --dac-conv-split $sp > "$O/ds_${w}_$sp.log" 2>&1 &&
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('workers $w split $sp', d['value'], d['ar_ms_per_step'], d['dac_audio_sec_per_s'])" "$O/ds_${w}_$sp.log" || exit 1
    done; done ;;
  conv_split)  # split-conv workgroup target: one 20-frame DAC decode, then the driver's short line
    timeout -k 10 200 python3 scripts/dac_host_probe.py 20 1,768,1024,1536,2048 > "$O/conv_split_dac1.jsonl" 2>&1 && cat "$O/conv_split_dac1.jsonl" &&
    for sp in ${@:2}; do
      timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --kokoro-prompts 0 --orpheus-steps 0 --dia-steps 0 --b1-replicas 0 \
          --dac-conv-split $sp > "$O/cs_$sp.log" 2>&1 &&
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('split $sp', d['value'], d['ar_ms_per_step'], d['dac_audio_sec_per_s'])" "$O/cs_$sp.log" || exit 1
    done ;;
  ar_trace)    # kernel trace of the AR-only bench (one replica of 8 prompts unless options say otherwise) + per-step breakdown
    shift
    (cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/proft" -o run --output-format csv -- python3 "$R/bench.py" $AR --steps 60 "$@" > "$O/ar_trace.log" 2>&1) &&
    f=$(find "$O/proft" -name "*kernel_trace.csv" | sort | tail -1) && python3 scripts/step_breakdown.py "$f" 5 30 > "$O/ar_breakdown.txt" && cat "$O/ar_breakdown.txt" | cut -c1-150 ;;
  orph_trace)  # kernel trace of the Orpheus leg + per-step breakdown (markers: the wide-vocabulary greedy step)
    shift
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/profo" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-dac --kokoro-prompts 0 --dia-steps 0 --no-cpu-baseline --b1-replicas 0 --orpheus-steps 40 "$@" > "$O/orph_trace.log" 2>&1) &&
    f=$(find "$O/profo" -name "*kernel_trace.csv" | sort | tail -1) && python3 scripts/step_breakdown.py "$f" 10 25 - k_greedy_step_wide > "$O/orph_breakdown.txt" && cut -c1-150 "$O/orph_breakdown.txt" ;;
  attn_opts)   # split-attention geometry (scores positions per workgroup x P.V dims per workgroup), AR-only
    for cfg in "--attn-ks 2 --attn-pv8 0" "--attn-ks 1 --attn-pv8 0" "--attn-ks 2 --attn-pv8 1" "--attn-ks 1 --attn-pv8 1" "--attn-ks 4 --attn-pv8 0" "--attn-ks 2 --attn-pv8 0"; do
      n=$(echo $cfg | tr -d ' -')
      timeout -k 10 200 python3 bench.py $AR $cfg > "$O/at_$n.log" 2>&1 && ar_line "$O/at_$n.log" "$cfg" || exit 1
    done ;;
  dia)         # Dia leg only (100 CFG steps), one bench run per option set, e.g. dia "--gemv-q80-pro 0" "--gemv-q80-pro 1"
    shift
    for cfg in "$@"; do
      n=$(echo $cfg | tr -d ' -')
      timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --no-cpu-baseline --b1-replicas 0 --dia-steps 100 $cfg > "$O/dia_$n.log" 2>&1 &&
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['dia'];print(sys.argv[2], d['ms_per_step'], d['encoder_step_ms'])" "$O/dia_$n.log" "$cfg" || exit 1
    done ;;
  dac20_trace)  # kernel trace of the driver's short line (AR + DAC of 20 frames), AR/DAC legs only
    shift
    (cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/profd20" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --kokoro-prompts 0 --orpheus-steps 0 --no-cpu-baseline --b1-replicas 0 --dia-steps 0 "$@" > "$O/dac20_trace.log" 2>&1) &&
    tail -1 "$O/dac20_trace.log" | cut -c1-300 ;;
  dia_trace)   # kernel trace of the Dia leg + per-step breakdown (markers: the greedy step)
    shift
    (cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/profdia" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-dac --kokoro-prompts 0 --orpheus-steps 0 --no-cpu-baseline --b1-replicas 0 --dia-steps 40 "$@" > "$O/dia_trace.log" 2>&1) &&
    f=$(find "$O/profdia" -name "*kernel_trace.csv" | sort | tail -1) && python3 scripts/step_breakdown.py "$f" 3 25 - k_greedy_step > "$O/dia_breakdown.txt" && cut -c1-150 "$O/dia_breakdown.txt" ;;
  tests)       # selected GPU test files, e.g. scripts/gpu_study.sh tests tests/test_dia_gpu.py
    shift
    timeout -k 10 900 python -u -m pytest "$@" $T > "$O/tests.log" 2>&1; rc=$?; tail -3 "$O/tests.log"; exit $rc ;;
  sync)        # grid barrier inside a persistent kernel vs a dependent kernel boundary
    hipcc --offload-arch=gfx950 -O3 scripts/microbench_sync.hip -o build/microbench_sync && timeout -k 10 120 build/microbench_sync > "$O/sync.jsonl" 2>&1 && cat "$O/sync.jsonl" ;;
  mfma_f64)    # the f64 MFMA ceiling
    hipcc --offload-arch=gfx950 -O3 scripts/mfma_f64_peak.hip -o build/mfma_f64_peak && timeout -k 10 120 build/mfma_f64_peak > "$O/mfma_f64.log" 2>&1 && cat "$O/mfma_f64.log" ;;
  *)
    echo "usage: $0 {ar|ar_trace|orph_trace|dia|dia_trace|dac20_trace|replicas|cu_partition|kernarg|gemv_phase|attn|dac|dac_short|tests|sync|mfma_f64} [args]"; exit 2 ;;
esac
