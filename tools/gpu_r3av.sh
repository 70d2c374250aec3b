# per-stream scratch cache: the full -m gpu suite, then host enqueue vs GPU time of the BA-obs calls
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3av.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_r3av.log; grep -E "^FAILED|^E  " gpurun_out/pytest_gpu_r3av.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/ba_host_overhead.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ba_host_r3av.txt
