# vq default switched to the f16-split filter: match / bow / sfm GPU tests, then vq A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_bow.py tests/test_gpu_sfm.py > gpurun_out/pytest_vq_r3ab.log 2>&1 || { tail -30 gpurun_out/pytest_vq_r3ab.log; exit 1; }
tail -3 gpurun_out/pytest_vq_r3ab.log
timeout -k 10 120 python tools/bench_vq.py 6,0,6,0 > gpurun_out/vq_ab_r3ab.txt 2>&1 || { cat gpurun_out/vq_ab_r3ab.txt; exit 1; }
cat gpurun_out/vq_ab_r3ab.txt
