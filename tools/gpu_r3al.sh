# vq f16s streaming probes: 64-B row pieces (shipped) vs 1 KB contiguous loads, with / without the MFMA pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_vq.py 6,6:8,6:9,6:10,6,6:8,6:9,6:10 2>&1 | grep -v "amdgpu.ids\|codes agree" | tee gpurun_out/vq_probe_r3al.txt
