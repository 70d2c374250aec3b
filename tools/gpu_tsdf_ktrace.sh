# Kernel-trace A/B of TSDF env knobs on C5: CONFIGS="A=1,B=0;A=0" (SFMHIP_TSDF_ prefix added).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
IFS=';' read -ra CF <<< "$CONFIGS"
for c in "${CF[@]}"; do
  i=$((i+1))
  ENVS=""
  IFS=',' read -ra KV <<< "$c"
  for kv in "${KV[@]}"; do ENVS="$ENVS SFMHIP_TSDF_$kv"; done
  env $ENVS REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt$i -o run -- python tools/run_tsdf_once.py > gpurun_out/kt$i.log 2>&1 || { echo "prof $c failed"; tail -5 gpurun_out/kt$i.log; exit 1; }
  find gpurun_out/kt$i -type f ! -name "*stats*" -delete
  python - "gpurun_out/kt$i" "$c" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
rows = []
for r in csv.DictReader(open(f)):
    if "sfmhip" in r["Name"]:
        a = float(r["AverageNs"]) / 1e3
        tot += a
        rows.append(f"{r['Name'].split('(')[0][-26:]}={a:.1f}")
print(sys.argv[2], f"sum {tot:.1f} us |", " ".join(rows))
PY
done
