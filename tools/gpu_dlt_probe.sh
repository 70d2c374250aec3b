# DLT list pass: where its time goes (rocprofv3 kernel-trace averages of dlt_normal / dlt_list
# under the timing probes: 0 = real, 1 = loads + stores only, 2 = QR3 without the dlt_point fallback)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for pr in 0 1 2 0; do
  env SFMHIP_DLT_LISTPROBE=$pr timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dltp$pr -o run -- python tools/bench_dlt.py > gpurun_out/dltp$pr.log 2>&1 || { echo "probe $pr failed"; tail -5 gpurun_out/dltp$pr.log; exit 1; }
  find gpurun_out/dltp$pr -type f ! -name "*kernel_stats*" -delete
  python - "gpurun_out/dltp$pr" "$pr" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = [f"{r['Name'].split('(')[0][-20:]}={float(r['AverageNs'])/1e3:.1f}us x{r['Calls']}" for r in csv.DictReader(open(f)) if "dlt" in r["Name"]]
print("probe", sys.argv[2], " ".join(rows))
PY
done
