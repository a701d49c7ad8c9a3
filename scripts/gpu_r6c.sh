#!/bin/bash
# the coalescer's tests alone, with refusal diagnostics (TTS_HIP_COALESCE_DEBUG=1)
cd $GRAFT_REPO_ROOT
TTS_HIP_COALESCE_DEBUG=1 timeout -k 10 400 python -u -m pytest tests/test_coalesce_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r6c_coal.log 2>&1
rc=$?; echo "coal rc $rc"; grep -m 20 "coalesce:" gpurun_out/r6c_coal.log; tail -25 gpurun_out/r6c_coal.log
exit $rc
