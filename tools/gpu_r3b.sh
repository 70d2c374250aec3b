# Round-3 session b: TSDF batched gathers — TSDF parity tests, kernel-trace A/B (BATCH 0/1) on C5,
# N=8 slab timing with and without batching.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_voxel.py tests/test_gpu_train.py -q -p no:cacheprovider -k "tsdf or sdf_mode" --timeout 300 --timeout-method thread > gpurun_out/pytest_tsdf_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_tsdf_$TAG.log; tail -3 gpurun_out/pytest_tsdf_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
CONFIGS="BATCH=0;BATCH=1;BATCH=0;BATCH=1" bash tools/gpu_tsdf_ktrace.sh > gpurun_out/tsdf_ab_$TAG.txt 2>&1 || { cat gpurun_out/tsdf_ab_$TAG.txt; exit 1; }
cat gpurun_out/tsdf_ab_$TAG.txt
SFMHIP_TSDF_BATCH=0 timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_b0_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_b0_$TAG.txt; exit 1; }
SFMHIP_TSDF_BATCH=1 timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_b1_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_b1_$TAG.txt; exit 1; }
tail -6 gpurun_out/slabs_b0_$TAG.txt gpurun_out/slabs_b1_$TAG.txt
