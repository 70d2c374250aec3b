# Round-3 session b (first box run of the re-created container): -m gpu suite + smoke,
# bench line, the --gpus 2 launcher rehearsal, the Adam placement probe, and the BA
# solve variants (parity with the fused kernel forced, then timing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r3g}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
head -c 600 gpurun_out/bench_$TAG.json; echo
SFMHIP_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --n-img 48 --dist-backend gloo --no-cpu-baseline --skip-secondary > gpurun_out/bench_gpus2_$TAG.json 2> gpurun_out/bench_gpus2_$TAG.err || { echo "gpus2 rehearsal failed"; tail -20 gpurun_out/bench_gpus2_$TAG.err; exit 1; }
cat gpurun_out/bench_gpus2_$TAG.json
for m in fresh after trim copy; do
  timeout -k 10 300 python tools/adam_probe.py $m >> gpurun_out/adam_probe_$TAG.txt 2>&1 || { echo "adam probe $m failed"; tail -5 gpurun_out/adam_probe_$TAG.txt; exit 1; }
done
cat gpurun_out/adam_probe_$TAG.txt
for v in 4 5; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_v${v}_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_ba_v${v}_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
for v in 0 4 5 1 0 4 5; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
grep variant gpurun_out/ba_variants_$TAG.txt
