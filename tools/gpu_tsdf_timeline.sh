# Kernel-trace timeline of the last C5 TSDF call for each SFMHIP_AB form in FORMS (default
# "1 0"): every sfmhip kernel's start offset and duration (tools/trace_summary.py), so the
# overlap of the side-stream block pass with the culling / fusion shows directly.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for ab in ${FORMS:-1 0}; do
  SFMHIP_AB=$ab REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl$ab -o run -- python tools/run_tsdf_once.py > gpurun_out/tl$ab.log 2>&1 || { echo "trace $ab failed"; tail -5 gpurun_out/tl$ab.log; exit 1; }
  f=$(find gpurun_out/tl$ab -name "*kernel_trace.csv" | head -1)
  n=$(python - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sfmhip" in r["Kernel_Name"]]
last = max(i for i, r in enumerate(rows) if "tsdf_setup_kernel" in r["Kernel_Name"])
print(len(rows) - last)
PY
)
  echo "== SFMHIP_AB=$ab (last call, $n kernels)"
  python tools/trace_summary.py "$f" "sfmhip" "$n" gpurun_out/timeline_ab$ab.txt > /dev/null
  python - gpurun_out/timeline_ab$ab.txt <<'PY'
import re, sys
rows = [ln for ln in open(sys.argv[1])]
end = 0.0
for ln in rows:
    m = re.search(r"start\s+([\d.]+) us\s+dur\s+([\d.]+)", ln)
    s, d = float(m.group(1)), float(m.group(2))
    end = max(end, s + d)
    print(ln.rstrip())
print(f"call span {end:.1f} us")
PY
  find gpurun_out/tl$ab -type f -delete
done
