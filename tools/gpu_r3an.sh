# kernel-trace averages of the vq call (filter + exact pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vq_r3an -o run -- python tools/bench_vq.py 6,6:4,6:1 > gpurun_out/prof_vq_r3an.log 2>&1 || { tail -20 gpurun_out/prof_vq_r3an.log; exit 1; }
grep -v amdgpu.ids gpurun_out/prof_vq_r3an.log | head -5
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_vq_r3an/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "vq_" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
find gpurun_out/prof_vq_r3an -type f ! -name "*kernel_stats*" -delete
