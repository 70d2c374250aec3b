# TSDF branch-free lane predicates A/B (tools/gpu_ab_lib.sh vs ab/lib_prev.so); DLT Jacobi test
# without the square root: geometry parity + DLT kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_geometry.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_geom_r3u.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_geom_r3u.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_dlt_probe.sh 2>&1 | grep "probe 0"
bash tools/gpu_ab_lib.sh
