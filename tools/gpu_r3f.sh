# BA fused-pass kernel: parity tests with it forced, then timing of the variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r3f}
SFMHIP_BA_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_$TAG.log; grep -E "^E |assert" gpurun_out/pytest_ba_$TAG.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for v in 4 1 4; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
grep variant gpurun_out/ba_variants_$TAG.txt
