# Kernel-trace breakdown of one N = 8 slab call (rank 2: a heavy centre slab, rank 6: a light one)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 2 6; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/slabkt$r -o run -- python tools/run_tsdf_slab.py 8 $r 10 > gpurun_out/slabkt$r.log 2>&1 || { echo "slab $r failed"; tail -5 gpurun_out/slabkt$r.log; exit 1; }
  find gpurun_out/slabkt$r -type f ! -name "*kernel_stats*" -delete
  python - "gpurun_out/slabkt$r" "$r" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
rows = []
for r in csv.DictReader(open(f)):
    if "sfmhip" in r["Name"]:
        a = float(r["AverageNs"]) / 1e3
        tot += a
        rows.append(f"{r['Name'].split('(')[0][-24:]}={a:.1f}")
print("slab", sys.argv[2], f"sum {tot:.1f} us |", " ".join(rows))
PY
done
