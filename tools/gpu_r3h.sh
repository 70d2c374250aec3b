# TSDF batched gathers re-measured (the r3b results were lost with the container): TSDF parity
# with BATCH=1 (default in this build) and BATCH=2, kernel-trace A/B on C5, N=8 slabs; then the
# Adam clock-ramp probe modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3h}
for b in 1 2; do
  SFMHIP_TSDF_BATCH=$b timeout -k 10 400 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider -k "tsdf" --timeout 300 --timeout-method thread > gpurun_out/pytest_tsdf_b${b}_$TAG.log 2>&1
  rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_tsdf_b${b}_$TAG.log; tail -2 gpurun_out/pytest_tsdf_b${b}_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
CONFIGS="BATCH=0;BATCH=1;BATCH=2;BATCH=0;BATCH=1;BATCH=2" bash tools/gpu_tsdf_ktrace.sh > gpurun_out/tsdf_ab_$TAG.txt 2>&1 || { cat gpurun_out/tsdf_ab_$TAG.txt; exit 1; }
cat gpurun_out/tsdf_ab_$TAG.txt
for b in 0 1 2; do
  SFMHIP_TSDF_BATCH=$b timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_b${b}_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_b${b}_$TAG.txt; exit 1; }
  echo "BATCH=$b"; tail -4 gpurun_out/slabs_b${b}_$TAG.txt
done
for m in fresh warm sleep iters; do
  timeout -k 10 300 python tools/adam_probe.py $m >> gpurun_out/adam_probe_$TAG.txt 2>&1 || { echo "adam probe $m failed"; tail -5 gpurun_out/adam_probe_$TAG.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/adam_probe_$TAG.txt
for v in 5 4; do
  timeout -k 10 120 python tools/ba_phase_prof.py $v >> gpurun_out/ba_phase_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_phase_$TAG.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ba_phase_$TAG.txt
