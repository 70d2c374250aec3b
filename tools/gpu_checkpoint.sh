# Round-3 checkpoint: -m gpu suite + smoke, bench line, rocprof kernel stats of the bench, the
# --gpus 2 rehearsal incl. the TSDF feedback balancing, N = 8 slab balancing on one GPU, BA timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3x}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED|^E  " gpurun_out/pytest_gpu_$TAG.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
head -c 400 gpurun_out/bench_$TAG.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
find gpurun_out/prof_$TAG -type f ! -name "*kernel_stats*" -delete
SFMHIP_BENCH_SAME_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --n-img 48 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench_gpus2_$TAG.json 2> gpurun_out/bench_gpus2_$TAG.err || { echo "gpus2 rehearsal failed"; tail -20 gpurun_out/bench_gpus2_$TAG.err; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_gpus2_$TAG.json').read()); print('gpus2', d['n_gpus'], round(d['value']), [(s['metric'], s['config'].get('slabs')) for s in d.get('secondary', [])][:1])"
timeout -k 10 300 python tools/bench_tsdf_slabs.py 8 > gpurun_out/slabs_$TAG.txt 2>&1 || { tail -5 gpurun_out/slabs_$TAG.txt; exit 1; }
grep "N=8\|whole" gpurun_out/slabs_$TAG.txt | cut -c1-160
