# PnP workgroup timeline (tool-only build ab/lib_pprof.so), then the product build back
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_keep.so
cp ab/lib_pprof.so $L
timeout -k 10 120 python tools/prof_pnp.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pnp_prof_r3bj.txt
rc=$?
cp ab/lib_keep.so $L
exit $rc
