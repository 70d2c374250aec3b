# Parameterised GPU session (one gpurun call): TAG names the outputs under gpurun_out/.
#   TESTS="tests/test_gpu_x.py ..."  pytest targets (default: every -m gpu test); TESTS=none skips
#   SMOKE=1    __graft_entry__.smoke()
#   BENCH=1    python bench.py (default steps) -> gpurun_out/bench_$TAG.json
#   BENCH_ARGS extra bench.py arguments
#   PROF=1     rocprofv3 --kernel-trace --stats of a short bench -> gpurun_out/prof_$TAG
#   EXTRA="cmd"  one more command (own time limit 300 s)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s}
if [ "${TESTS:-all}" != none ]; then
  T=${TESTS:-tests}
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pytest_$TAG.log | head -80; exit 1; }
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 bash -c "$EXTRA" > gpurun_out/extra_$TAG.log 2>&1 || { tail -30 gpurun_out/extra_$TAG.log; exit 1; }
  tail -40 gpurun_out/extra_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 700 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  python tools/bench_summary.py gpurun_out/bench_$TAG.json
fi
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
  find gpurun_out/prof_$TAG -type f ! -name "*stats*" -delete
fi
du -sh gpurun_out
