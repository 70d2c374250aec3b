# BA solve: 512-thread (variant 2, default) vs 1024-thread field-major (variant 4, 4 waves/SIMD with spills),
# alternated; BA/geometry tests under variant 4; bench line with the DDA / exact-float rooflines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 2 4 2 4; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_v4_ab_r3bl.txt 2>&1 || exit 1
done
cat gpurun_out/ba_v4_ab_r3bl.txt
SFMHIP_BA_VARIANT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_v4_r3bl.log 2>&1
echo "ba v4 tests rc=$?"; tail -2 gpurun_out/pytest_ba_v4_r3bl.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_r3bl.json 2> gpurun_out/bench_r3bl.err || { tail -20 gpurun_out/bench_r3bl.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_r3bl.json').read())
for s in d['secondary']:
    if s['metric'].startswith(('voxel_trav','exact')): print(s['metric'], json.dumps(s['roofline'])[:300])"
