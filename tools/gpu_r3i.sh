# Adam buffer-layout probe, render ray order (host keys + the device sort), render parity,
# MFMA ceilings incl. d = 128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider -k "render" --timeout 120 --timeout-method thread > gpurun_out/pytest_render_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_render_$TAG.log; grep -E "^E " gpurun_out/pytest_render_$TAG.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python tools/bench_render_order.py > gpurun_out/render_order_$TAG.txt 2>&1 || { tail -5 gpurun_out/render_order_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/render_order_$TAG.txt
timeout -k 10 300 python tools/adam_layout_probe.py > gpurun_out/adam_layout_$TAG.txt 2>&1 || { tail -5 gpurun_out/adam_layout_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/adam_layout_$TAG.txt
timeout -k 10 120 tools/mfma_peak 2000 1 > gpurun_out/mfma_peak_$TAG.txt 2>&1 || { tail -5 gpurun_out/mfma_peak_$TAG.txt; exit 1; }
cat gpurun_out/mfma_peak_$TAG.txt
