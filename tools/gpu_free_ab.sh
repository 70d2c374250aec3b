set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_voxel.log 2>&1 || { echo "voxel tests failed"; tail -40 gpurun_out/pytest_voxel.log; exit 1; }
tail -1 gpurun_out/pytest_voxel.log
timeout -k 10 300 python tools/bench_tsdf_variants.py "${AB:-FREE=1;VOXTEST=0;SBZ=4;SBX=2,SBY=2;IL=0;SBX=4,SBY=4,SBZ=2;CHUNK=64}" > gpurun_out/ab_free.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_free.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_free.log
