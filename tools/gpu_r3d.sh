# BA solve: GPU parity tests (default variant), then the layout / thread-count variants timed
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r3d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for v in 0 1 2 3 0 1; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
cat gpurun_out/ba_variants_$TAG.txt | grep variant
