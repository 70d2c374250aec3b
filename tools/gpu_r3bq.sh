# refine grid 8192 as the default: TSDF / voxel GPU tests, smoke, bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_voxel.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_voxel_r3bq.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_voxel_r3bq.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3bq.log 2>&1 || { tail -20 gpurun_out/smoke_r3bq.log; exit 1; }
tail -1 gpurun_out/smoke_r3bq.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r3bq.json 2> gpurun_out/bench_r3bq.err || { tail -20 gpurun_out/bench_r3bq.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_r3bq.json').read()); print(round(d['value']), d['ms_per_step'])
for s in d['secondary'][:2]: print(s['metric'], s['value'], s.get('ms_per_step'))"
