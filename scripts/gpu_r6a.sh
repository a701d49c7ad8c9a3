set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6a_suite.log 2>&1
rc=$?; echo "suite rc $rc"; tail -3 gpurun_out/r6a_suite.log
[ $rc -eq 0 ] || exit $rc
TTS_HIP_COALESCE_TESTS=1 timeout -k 10 400 python -u -m pytest tests/test_coalesce_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r6a_coal.log 2>&1
rc=$?; echo "coal rc $rc"; tail -15 gpurun_out/r6a_coal.log
[ $rc -eq 0 ] || exit $rc
TTS_HIP_COALESCE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6a_suite_vmm.log 2>&1
rc=$?; echo "suite-vmm rc $rc"; tail -3 gpurun_out/r6a_suite_vmm.log
exit $rc
