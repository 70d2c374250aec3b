# BA record prefetch variants (4: 512 threads + prefetch, 5: 256 + prefetch) parity + timing;
# slab kernel-trace breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3q}
for v in 4 5; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py tests/test_gpu_sfm.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_v${v}_$TAG.log 2>&1
  rc=$?; echo "v$v: $(tail -1 gpurun_out/pytest_ba_v${v}_$TAG.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
for v in 2 4 5 1 2 4 5 1; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
grep variant gpurun_out/ba_variants_$TAG.txt
bash tools/gpu_slab_ktrace.sh
