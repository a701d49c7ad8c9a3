#!/bin/bash
# MFMA evidence for the codec convolutions (k_conv1d_f64, k_convt_f64_lds): one DAC-44k decode of 200
# latent frames (f64 accumulation, the default) under the kernel trace, then SQ counter passes of the
# same command (each pass its own run, counters checked against `rocprofv3 -L` first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/pmc_conv
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/scripts/bench_dac.py 200 --default-only"
timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- $CMD > "$O/trace.log" 2>&1 || exit 1
P1="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
n=1
for P in "$P1" "$P2"; do
  ok=1
  for c in $P; do grep -q "\b$c\b" "$O/counters.txt" || { echo "counter $c not listed; pass $n skipped"; ok=0; }; done
  if [ $ok = 1 ]; then
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d "$O/pmc$n" -o run --output-format csv -- $CMD > "$O/pmc$n.log" 2>&1 || { echo "pmc pass $n failed"; exit 1; }
  fi
  n=$((n + 1))
done
echo done
