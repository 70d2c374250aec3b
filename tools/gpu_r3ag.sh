# C2 shape (64 x 2048 x 128): every match kernel variant, interleaved, identical outputs required
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
N_IMG=64 DIM=128 MKPT=2048 timeout -k 10 300 python tools/bench_match_variants.py 0,1,2,3,4,5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/match_variants_c2_r3ag.txt
