# Round-2 closing session: -m gpu suite + smoke (gpu_r2a.sh), bench + rocprof stats
# (gpu_bench_prof.sh), the N-way slab timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r2f}
TAG=$TAG bash tools/gpu_r2a.sh || exit 1
NO_REHEARSE=1 TAG=$TAG bash tools/gpu_bench_prof.sh || exit 1
timeout -k 10 300 python tools/bench_tsdf_slabs.py > gpurun_out/slabs_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_$TAG.txt; exit 1; }
grep "N=\|whole" gpurun_out/slabs_$TAG.txt | cut -c1-120
