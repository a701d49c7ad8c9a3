#!/bin/bash
# PMC counters of the GEMV variants in the phase micro-benchmark (build/gemv_phase), one pass per
# counter group (SQ block: up to 8 counters per pass, no trace domains besides the kernel trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmc_ph1 -o run --output-format csv -- ./build/gemv_phase > gpurun_out/pmc_ph1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/pmc_ph2 -o run --output-format csv -- ./build/gemv_phase > gpurun_out/pmc_ph2.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pmc_ph1.log
exit $rc
