# A/B of two builds of libsfmhip.so on one box (ab/lib_prev.so vs the in-tree build):
# the TSDF GPU tests on the new build, then kernel-trace sums of the C5 call and the
# N-way slab timing, alternating builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -x -q -k "tsdf" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  CONFIGS="EASY=1" bash tools/gpu_tsdf_ktrace.sh | sed "s/^/$v /" || exit 1
done
for v in new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 300 python tools/bench_tsdf_slabs.py > gpurun_out/ab_slabs_$v.txt 2>&1 || { tail -5 gpurun_out/ab_slabs_$v.txt; exit 1; }
  grep "N=8\|whole" gpurun_out/ab_slabs_$v.txt | cut -c1-100 | sed "s/^/$v /"
done
cp ab/lib_new.so $L
