# Kernel-trace stats of the C5 TSDF integration with the free-space path on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for FR in 1 4; do
  SFMHIP_TSDF_FREE=$FR timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof_free$FR -o run -- python tools/run_tsdf_once.py > gpurun_out/tprof_free$FR.log 2>&1 || { echo "prof $FR failed"; tail -5 gpurun_out/tprof_free$FR.log; exit 1; }
  find gpurun_out/tprof_free$FR -type f ! -name "*stats*" -delete
  python - "$FR" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/tprof_free{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sfmhip" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 2e6, 3), "ms/integration")
PY
done
