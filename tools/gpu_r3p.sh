# Render chunk-major launches: parity (render tests), timing vs one launch, PMC traffic of the
# chunked launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider -k render --timeout 120 --timeout-method thread > gpurun_out/pytest_render_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_render_$TAG.log; grep -E "^E  " gpurun_out/pytest_render_$TAG.log | head -3; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_render_order.py > gpurun_out/render_order_$TAG.txt 2>&1 || { tail -5 gpurun_out/render_order_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/render_order_$TAG.txt | head -8
REPS=2 bash tools/pmc.sh render_$TAG "render_kernel" tools/run_render_once.py > /dev/null || exit 1
python tools/pmc_summary.py gpurun_out/pmc_render_$TAG > gpurun_out/pmc_render_$TAG.txt 2>&1
grep -E "==|HBM|L2 hit|VALU-active" gpurun_out/pmc_render_$TAG.txt
