# BA solve GPU tests + the FD/geometry tests that share fd_obs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-ba}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/pytest_$TAG.log | tail -30
exit $rc
