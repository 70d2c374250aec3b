# Bench line + rocprofv3 kernel-trace stats of the same bench, then the N>1
# path rehearsals (one-rank C-ABI RCCL comm; 2-rank gloo on one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
find gpurun_out/prof_$TAG -type f ! -name "*stats*" -delete
[ -n "$NO_REHEARSE" ] && exit 0
timeout -k 10 300 python bench.py --rehearse-overlap --steps 3 --warmup 1 --skip-secondary --no-cpu-baseline > gpurun_out/bench_overlap_$TAG.json 2> gpurun_out/bench_overlap_$TAG.err || { echo "overlap rehearsal failed"; tail -20 gpurun_out/bench_overlap_$TAG.err; exit 1; }
cat gpurun_out/bench_overlap_$TAG.json
SFMHIP_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --n-img 48 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench_rehearsal_$TAG.json 2> gpurun_out/bench_rehearsal_$TAG.err || { echo "rehearsal failed"; tail -20 gpurun_out/bench_rehearsal_$TAG.err; exit 1; }
cat gpurun_out/bench_rehearsal_$TAG.json
du -sh gpurun_out
