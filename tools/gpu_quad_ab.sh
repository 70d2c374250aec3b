# TSDF thin-slab quad variant: parity (TSDF GPU tests with latency mode + quad forced,
# then the default suite's TSDF tests), then N-way slab timing quad off / on / off / on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
SFMHIP_TSDF_LATENCY=1 SFMHIP_TSDF_QUAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -x -q -k "tsdf" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/quad_tests.log 2>&1 || { tail -30 gpurun_out/quad_tests.log; exit 1; }
tail -1 gpurun_out/quad_tests.log
for q in 0 1 0 1; do
  SFMHIP_TSDF_QUAD=$q timeout -k 10 300 python tools/bench_tsdf_slabs.py > gpurun_out/quad_slabs_$q.txt 2>&1 || { tail -5 gpurun_out/quad_slabs_$q.txt; exit 1; }
  grep "^N=\|whole" gpurun_out/quad_slabs_$q.txt | cut -c1-60 | sed "s/^/quad=$q /"
  grep "^N=8 planned" gpurun_out/quad_slabs_$q.txt | grep -o "ms \[.*" | sed "s/^/quad=$q N=8 /"
done
