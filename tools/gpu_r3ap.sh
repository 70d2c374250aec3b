# vq f16s: exact pass with coalesced codeword rows; vq/bow/sfm GPU tests on the new
# build, then the vq call new vs ab/lib_prev.so (the committed f16s kernel), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_bow.py tests/test_gpu_sfm.py -k "vq or bow or kmeans or sfm or golden" -p no:cacheprovider > gpurun_out/pytest_vq_r3ap.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_vq_r3ap.log; grep -E "^E  |FAILED" gpurun_out/pytest_vq_r3ap.log | head -5; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 120 python tools/bench_vq.py 6,0 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done | tee gpurun_out/vq_ab_r3ap.txt
cp ab/lib_new.so $L
