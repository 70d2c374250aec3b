# PnP: phase profile (tool-only build ab/lib_pprof.so), then the fused-Jacobi builds (ab/lib_fj.so, ab/lib_fj2.so):
# PnP GPU tests, timing + output checksums vs ab/lib_base.so alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp ab/lib_pprof.so $L
timeout -k 10 120 python tools/prof_pnp.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pnp_prof_r3bi.txt || exit 1
cp ab/lib_g8s.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "pnp or PnP or incremental or register" -p no:cacheprovider > gpurun_out/pytest_pnp_r3bi.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_pnp_r3bi.log; grep -E "^E  |FAILED" gpurun_out/pytest_pnp_r3bi.log | head -5; [ $rc -eq 0 ] || exit 1
for v in g8s g8 fj2 g8s g8 fj2; do
  cp ab/lib_$v.so $L
  timeout -k 10 120 python tools/ab_pnp.py 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || exit 1
done | tee gpurun_out/pnp_ab_r3bi.txt
