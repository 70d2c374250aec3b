# BA: wave-uniform index in the block reductions: geometry / BA GPU tests on the new build, then bit checksums and
# timings of the FD Jacobian and BA solve, new vs ab/lib_prev.so alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_geometry.py tests/test_gpu_ba.py tests/test_gpu_sfm.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_fd_r3ba.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_fd_r3ba.log; grep -E "^E  " gpurun_out/pytest_fd_r3ba.log | head -3; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 300 python tools/ab_fd_bits.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done
cp ab/lib_new.so $L
