# essential RANSAC phase profile (tool-only build ab/lib_rprof.so), then the product build back
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
cp ab/lib_rprof.so $L
timeout -k 10 120 python tools/prof_ransac.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ransac_prof_r3aq.txt
rc=$?
cp ab/lib_new.so $L
exit $rc
