# Render device ordering v2 (two-level histogram) parity + timing; TSDF w_runs hoist A/B
# (ab/lib_prev.so = the previous voxel.hip); Adam layout microbenchmark in fresh processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_voxel_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_voxel_$TAG.log; grep -E "^E " gpurun_out/pytest_voxel_$TAG.log | head -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_render_order.py > gpurun_out/render_order_$TAG.txt 2>&1 || { tail -5 gpurun_out/render_order_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/render_order_$TAG.txt
for m in sep one all sep one; do
  timeout -k 10 120 tools/adam_layout_micro $m >> gpurun_out/adam_micro_$TAG.txt 2>&1 || { tail -5 gpurun_out/adam_micro_$TAG.txt; exit 1; }
done
cat gpurun_out/adam_micro_$TAG.txt
bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/tsdf_hoist_ab_$TAG.txt
