# vq default switched to the f16-split filter
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_bow.py tests/test_gpu_sfm.py -k "vq or bow or kmeans or sfm or golden" > gpurun_out/pytest_vq_r3ac.log 2>&1 || { tail -30 gpurun_out/pytest_vq_r3ac.log; exit 1; }
tail -2 gpurun_out/pytest_vq_r3ac.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_voxel.py -k "render" > gpurun_out/pytest_render_r3ac.log 2>&1 || { tail -30 gpurun_out/pytest_render_r3ac.log; exit 1; }
tail -2 gpurun_out/pytest_render_r3ac.log
timeout -k 10 120 python tools/bench_vq.py 6,0,6,0 > gpurun_out/vq_ab_r3ac.txt 2>&1 || { cat gpurun_out/vq_ab_r3ac.txt; exit 1; }
cat gpurun_out/vq_ab_r3ac.txt
