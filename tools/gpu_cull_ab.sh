set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_voxel.log 2>&1 || { echo "voxel tests failed"; tail -30 gpurun_out/pytest_voxel.log; exit 1; }
tail -1 gpurun_out/pytest_voxel.log
timeout -k 10 300 python tools/tsdf_cull_stats.py 2>&1 | grep -v amdgpu
timeout -k 10 300 python tools/bench_tsdf_variants.py "FREE=1;REFINE=0" 2>&1 | grep -v amdgpu
bash tools/gpu_tsdf_prof.sh
