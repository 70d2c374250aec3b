# Probes: TSDF slab balance (equal vs planned) and exact-float / C2 matcher cost.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-probe}
timeout -k 10 300 python -u tools/bench_tsdf_slabs.py 2 4 8 > gpurun_out/slabs_$TAG.txt 2>&1 || { tail -20 gpurun_out/slabs_$TAG.txt; exit 1; }
cat gpurun_out/slabs_$TAG.txt
timeout -k 10 300 python -u tools/bench_match_exact.py 4096 > gpurun_out/exact_$TAG.txt 2>&1 || { tail -20 gpurun_out/exact_$TAG.txt; exit 1; }
cat gpurun_out/exact_$TAG.txt
