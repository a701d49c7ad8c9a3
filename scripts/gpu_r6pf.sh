#!/bin/bash
# Phase timeline of the prefill GEMM (scripts/gemv_phase.hip, GEMV_PHASE_PREFILL): warm and cold caches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
GEMV_PHASE_PREFILL=1 timeout -k 10 120 scripts/_bin/gemv_phase > gpurun_out/pf_phase.jsonl 2>&1
rc=$?; cat gpurun_out/pf_phase.jsonl; [ $rc -eq 0 ] || exit $rc
GEMV_PHASE_PREFILL=1 GEMV_PHASE_COLD=1 timeout -k 10 120 scripts/_bin/gemv_phase > gpurun_out/pf_phase_cold.jsonl 2>&1
rc=$?; cat gpurun_out/pf_phase_cold.jsonl; exit $rc
