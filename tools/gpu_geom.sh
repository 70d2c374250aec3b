# Geometry GPU tests + DLT A/B timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-geom}
timeout -k 10 300 python -u -m pytest tests/test_gpu_geometry.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/pytest_$TAG.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_dlt.py > gpurun_out/dlt_$TAG.txt 2>&1 || { tail -20 gpurun_out/dlt_$TAG.txt; exit 1; }
cat gpurun_out/dlt_$TAG.txt
