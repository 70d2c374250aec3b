# Full GPU session: parity tests, bench line, rocprofv3 kernel-trace stats of
# the bench, PMC traffic passes for the match + TSDF kernels, and a 2-rank
# rehearsal of the distributed bench path (gloo, both ranks on device 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
find gpurun_out/prof_$TAG -type f ! -name "*stats*" -delete
bash tools/pmc.sh match_$TAG match_kernel tools/run_match_once.py || exit 1
bash tools/pmc.sh tsdf_$TAG "tsdf_kernel|tsdf_cull|depth_blockmax" tools/run_tsdf_once.py || exit 1
SFMHIP_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --n-img 48 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench_rehearsal_$TAG.json 2> gpurun_out/bench_rehearsal_$TAG.err || { echo "rehearsal failed"; tail -20 gpurun_out/bench_rehearsal_$TAG.err; exit 1; }
cat gpurun_out/bench_rehearsal_$TAG.json
du -sh gpurun_out
