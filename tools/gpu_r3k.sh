# Adam allocation-history microbenchmark; BA solve variants 1/2 parity and timing of 0-3, 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3k}
for m in sep churn hold rev sep churn; do
  timeout -k 10 120 tools/adam_layout_micro $m >> gpurun_out/adam_micro_$TAG.txt 2>&1 || { tail -5 gpurun_out/adam_micro_$TAG.txt; exit 1; }
done
cat gpurun_out/adam_micro_$TAG.txt
for v in 1 2; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_v${v}_$TAG.log 2>&1
  rc=$?; tail -1 gpurun_out/pytest_ba_v${v}_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
for v in 0 1 2 3 5 0 1 2 3 5; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
grep variant gpurun_out/ba_variants_$TAG.txt
