# host enqueue cost vs GPU time of the BA-obs step calls
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/ba_host_overhead.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ba_host_r3au.txt
