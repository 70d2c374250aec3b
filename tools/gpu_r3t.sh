# Latency-mode fusion with LDS camera records + three frames in flight (SFMHIP_TSDF_PIPE=2) vs 1:
# parity with 2 forced, N = 8 slabs, per-wave timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3t}
SFMHIP_TSDF_PIPE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py tests/test_dist.py -q -p no:cacheprovider -k "tsdf or table or slab" --timeout 120 --timeout-method thread > gpurun_out/pytest_tsdf_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_tsdf_$TAG.log; grep -E "^E  " gpurun_out/pytest_tsdf_$TAG.log | head -3; [ $rc -eq 0 ] || exit 1
for pm in 2 1; do
  SFMHIP_TSDF_PIPE=$pm timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_pipe${pm}_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_pipe${pm}_$TAG.txt; exit 1; }
  echo "PIPE=$pm"; grep "N=8" gpurun_out/slabs_pipe${pm}_$TAG.txt | cut -c1-100
done
SFMHIP_TSDF_PIPE=2 timeout -k 10 300 python tools/tsdf_wave_prof.py > gpurun_out/tsdf_wave_prof_ldsrec.txt 2>&1 || { tail -5 gpurun_out/tsdf_wave_prof_ldsrec.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tsdf_wave_prof_ldsrec.txt | grep -v "last-ending\|^whole" | head -20
