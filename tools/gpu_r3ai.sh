# C2 shape: the default match kernel on float-mode vs SIFT-mode operands (same code and shape)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for data in float sift float sift; do
  DATA=$data N_IMG=64 DIM=128 MKPT=2048 timeout -k 10 120 python tools/bench_match_variants.py 0 2>&1 | grep -v amdgpu.ids | sed "s/^/$data /" || exit 1
done | tee gpurun_out/match_c2_data_r3ai.txt
