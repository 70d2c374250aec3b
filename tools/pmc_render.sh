# Render kernel HBM traffic (FETCH_SIZE) and kernel time, rays in bench order and direction-sorted.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_render
for SO in 0 1; do
  SORT=$SO timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex render --output-format csv -d gpurun_out/pmc_render/s$SO -o p -- python tools/run_render_once.py > gpurun_out/pmc_render/log$SO.txt 2>&1 || { tail -5 gpurun_out/pmc_render/log$SO.txt; exit 1; }
  python - "$SO" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/pmc_render/s{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
acc = {}
dur = []
for r in csv.DictReader(open(f)):
    acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
m = {k: sum(v) / len(v) for k, v in acc.items()}
print("sort", sys.argv[1], "FETCH x2 GB %.3f" % (2 * m["FETCH_SIZE"] * 1024 / 1e9), "dur ms %.3f" % (sum(dur) / len(dur)))
PY
done
