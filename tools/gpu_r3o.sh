# TSDF fusion wave priority A/B (SFMHIP_TSDF_PRIO 1/0): parity with it on, kernel-trace sums on C5,
# N = 8 slabs (equal + feedback-balanced) with and without
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3o}
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider -k tsdf --timeout 120 --timeout-method thread > gpurun_out/pytest_tsdf_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_tsdf_$TAG.log; [ $rc -eq 0 ] || exit 1
CONFIGS="PRIO=1;PRIO=0;PRIO=1;PRIO=0" bash tools/gpu_tsdf_ktrace.sh > gpurun_out/tsdf_prio_$TAG.txt 2>&1 || { cat gpurun_out/tsdf_prio_$TAG.txt; exit 1; }
cat gpurun_out/tsdf_prio_$TAG.txt
for pr in 1 0; do
  SFMHIP_TSDF_PRIO=$pr timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_p${pr}_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_p${pr}_$TAG.txt; exit 1; }
  echo "PRIO=$pr"; grep "N=8\|whole" gpurun_out/slabs_p${pr}_$TAG.txt | cut -c1-150
done
TAG=r3 bash tools/gpu_traffic_r2.sh > gpurun_out/traffic_r3.log 2>&1 || { tail -20 gpurun_out/traffic_r3.log; exit 1; }
tail -3 gpurun_out/traffic_r3.log
