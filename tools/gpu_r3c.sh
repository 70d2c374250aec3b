# TSDF batch variants A/B (kernel trace, C5) + N=8 slab timing per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider -k "tsdf_culling_is_exact or c5_full" --timeout 300 --timeout-method thread > gpurun_out/pytest_tsdf_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_tsdf_$TAG.log; tail -2 gpurun_out/pytest_tsdf_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
CONFIGS="BATCH=0;BATCH=1;BATCH=2;BATCH=0;BATCH=2" bash tools/gpu_tsdf_ktrace.sh > gpurun_out/tsdf_ab_$TAG.txt 2>&1 || { cat gpurun_out/tsdf_ab_$TAG.txt; exit 1; }
cat gpurun_out/tsdf_ab_$TAG.txt
for b in 0 2; do
SFMHIP_TSDF_BATCH=$b timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_b${b}_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_b${b}_$TAG.txt; exit 1; }
grep "equal" gpurun_out/slabs_b${b}_$TAG.txt
done
