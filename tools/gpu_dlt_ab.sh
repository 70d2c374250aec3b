# DLT A/B of two library builds (ab/lib_prev.so vs in-tree): geometry GPU tests on the
# new build, then tools/bench_dlt.py alternating builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_geometry.py tests/test_gpu_ba.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/dlt_tests.log 2>&1 || { tail -20 gpurun_out/dlt_tests.log; exit 1; }
tail -1 gpurun_out/dlt_tests.log
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 200 python tools/bench_dlt.py 2>&1 | grep "^DLT" | sed "s/^/$v /" || exit 1
done
cp ab/lib_new.so $L
