# TSDF fusion with three frames in flight: latency mode (SFMHIP_TSDF_PIPE=2 vs 1) and whole grid
# (SFMHIP_TSDF_RING=1 vs 0): parity with each forced, C5 kernel-trace A/B, N = 8 slabs, timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3s}
for E in SFMHIP_TSDF_PIPE=2 SFMHIP_TSDF_RING=1; do
  env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py tests/test_dist.py -q -p no:cacheprovider -k "tsdf or table or slab" --timeout 120 --timeout-method thread > gpurun_out/pytest_tsdf_${E}_$TAG.log 2>&1
  rc=$?; echo "$E: $(tail -1 gpurun_out/pytest_tsdf_${E}_$TAG.log)"; grep -E "^E  " gpurun_out/pytest_tsdf_${E}_$TAG.log | head -3; [ $rc -eq 0 ] || exit 1
done
CONFIGS="RING=1;RING=0;RING=1;RING=0" bash tools/gpu_tsdf_ktrace.sh > gpurun_out/tsdf_ring_$TAG.txt 2>&1 || { cat gpurun_out/tsdf_ring_$TAG.txt; exit 1; }
cat gpurun_out/tsdf_ring_$TAG.txt
for pm in 2 1; do
  SFMHIP_TSDF_PIPE=$pm timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_pipe${pm}_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_pipe${pm}_$TAG.txt; exit 1; }
  echo "PIPE=$pm"; grep "N=8\|whole" gpurun_out/slabs_pipe${pm}_$TAG.txt | cut -c1-160
done
SFMHIP_TSDF_PIPE=2 SFMHIP_TSDF_RING=1 timeout -k 10 300 python tools/tsdf_wave_prof.py > gpurun_out/tsdf_wave_prof_ring.txt 2>&1 || { tail -5 gpurun_out/tsdf_wave_prof_ring.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tsdf_wave_prof_ring.txt | grep -v "last-ending" | head -30
