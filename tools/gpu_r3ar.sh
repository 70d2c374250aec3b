# DDA walk without short-circuit branches, one wave per count workgroup: voxel tests on the new build,
# then the V1 call new vs ab/lib_prev.so alternating (identical output required)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_voxel.py -k "traversal" -p no:cacheprovider > gpurun_out/pytest_dda_r3ar.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_dda_r3ar.log; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 120 python tools/bench_dda.py 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done | tee gpurun_out/dda_ab_r3ar.txt
cp ab/lib_new.so $L
