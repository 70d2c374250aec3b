# essential RANSAC: scoring out of line (A/B, reverted): GPU tests on the new build, then timing and
# output checksums new vs ab/lib_prev.so alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "essential or ransac or verif or pose or pnp" -p no:cacheprovider > gpurun_out/pytest_pnp_r3bd.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_pnp_r3bd.log; grep -E "^E  |FAILED" gpurun_out/pytest_pnp_r3bd.log | head -5; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 120 python tools/ab_verify.py 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done | tee gpurun_out/pnp_ab_r3bd.txt
cp ab/lib_new.so $L
