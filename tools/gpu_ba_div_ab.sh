set -o pipefail
L=3d_reconstruction_amd/libsfmhip.so
mkdir -p gpurun_out
cp abl/lib_new.so $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_geometry.py tests/test_gpu_sfm.py > gpurun_out/ba_div_t.log 2>&1 || { tail -30 gpurun_out/ba_div_t.log; exit 1; }
tail -1 gpurun_out/ba_div_t.log
for rep in 1 2 3; do
  for v in base new; do
    cp abl/lib_$v.so $L
    echo -n "$v "; timeout -k 10 120 python tools/ab_ba.py 0 2>/dev/null | tail -1 || exit 1
  done
done
