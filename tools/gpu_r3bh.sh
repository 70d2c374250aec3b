# DDA one-walk (capped) form: traversal GPU tests, then the V1 call new vs ab/lib_prev.so alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_voxel.py tests/test_abi.py -k "traversal or abi or export" -p no:cacheprovider > gpurun_out/pytest_dda_r3bh.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_dda_r3bh.log; grep -E "^E  |FAILED" gpurun_out/pytest_dda_r3bh.log | head -5; [ $rc -eq 0 ] || exit 1
for v in new two new two; do
  if [ $v = two ]; then export SFMHIP_DDA_CAP=0; else unset SFMHIP_DDA_CAP; fi
  timeout -k 10 120 python tools/bench_dda.py 2>&1 | grep -v "amdgpu.ids" | sed "s/^/$v /" || exit 1
done | tee gpurun_out/dda_ab_r3bh.txt
