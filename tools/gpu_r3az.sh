# wave-uniform ray / unit indices in render, render_train and the vq kernels: GPU tests on the new
# build, then render and vq timing new vs ab/lib_prev.so alternating (identical outputs required)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_voxel.py tests/test_gpu_train.py tests/test_gpu_match.py -k "render or train or vq or sdf or plenoxel" -p no:cacheprovider > gpurun_out/pytest_r3az.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r3az.log; grep -E "^E  |FAILED" gpurun_out/pytest_r3az.log | head -5; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  { timeout -k 10 120 python tools/bench_render_train.py && timeout -k 10 120 python tools/bench_vq.py 6; } 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done | tee gpurun_out/uniform_ab_r3az.txt
cp ab/lib_new.so $L
