set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_voxel.log 2>&1 || { echo "voxel tests failed"; tail -40 gpurun_out/pytest_voxel.log; exit 1; }
tail -1 gpurun_out/pytest_voxel.log
timeout -k 10 300 python tools/tsdf_cull_stats.py > gpurun_out/cull_stats.log 2>&1 || { echo "stats failed"; tail -20 gpurun_out/cull_stats.log; exit 1; }
cat gpurun_out/cull_stats.log
timeout -k 10 300 python tools/bench_tsdf_variants.py "FREE=1;CHUNK=32;CHUNK=64;CHUNK=128;CULLSUB=4;CHUNK=64,CULLSUB=4;CHUNK=128,CULLSUB=4;FREE=0,CHUNK=32" > gpurun_out/ab_free.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_free.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_free.log
bash tools/gpu_tsdf_prof.sh
