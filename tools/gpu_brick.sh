# Brick pre-pass A/B: TSDF GPU tests, interleaved C5 timing with the pre-pass on/off,
# kernel-trace stats of both, the N-way slab timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-brick}
timeout -k 10 600 python -u -m pytest tests/test_gpu_voxel.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -2
timeout -k 10 300 python tools/bench_tsdf_variants.py "BRICK=1;BRICK=0;BRICK=1,REFINE=0" > gpurun_out/variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/variants_$TAG.txt; exit 1; }
cat gpurun_out/variants_$TAG.txt
for B in 1 0; do
  SFMHIP_TSDF_BRICK=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof_$TAG$B -o run -- python tools/run_tsdf_once.py > gpurun_out/tprof_$TAG$B.log 2>&1 || { echo "prof $B failed"; tail -5 gpurun_out/tprof_$TAG$B.log; exit 1; }
  find gpurun_out/tprof_$TAG$B -type f ! -name "*stats*" -delete
  python - "gpurun_out/tprof_$TAG$B" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sfmhip" in r["Name"]:
        print(sys.argv[1][-7:], r["Name"].split("(")[0][-34:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
[ -n "$SLABS" ] && timeout -k 10 300 python tools/bench_tsdf_slabs.py > gpurun_out/slabs_$TAG.txt 2>&1 && cat gpurun_out/slabs_$TAG.txt
exit 0
