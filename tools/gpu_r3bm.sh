# TSDF: what frame chunking costs the fusion (potential of overlapping chunk k+1's block pass with
# chunk k's fusion tail): whole-call A/B of CHUNK 512 / 129 / 86, then a kernel trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_tsdf_variants.py "CHUNK=512;CHUNK=129;CHUNK=86" > gpurun_out/tsdf_chunk_ab_r3bm.txt 2>&1 || { cat gpurun_out/tsdf_chunk_ab_r3bm.txt; exit 1; }
cat gpurun_out/tsdf_chunk_ab_r3bm.txt
for c in 512 129; do
  SFMHIP_TSDF_CHUNK=$c REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_chunk$c -o run -- python tools/run_tsdf_once.py > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import csv, glob
for c in (512, 129):
    f = glob.glob(f"gpurun_out/kt_chunk{c}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "sfmhip" in r["Kernel_Name"]]
    n = len(t) // 3
    last = t[-n:]
    t0 = last[0][1]
    print(f"CHUNK={c}: last call, {n} kernels")
    for name, s, e in last:
        print(f"  {name:40s} start {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:8.1f} us")
PY
rm -rf gpurun_out/kt_chunk*
timeout -k 10 200 python tools/bench_tsdf_overlap.py 32 64 96 129 > gpurun_out/tsdf_overlap_ab_r3bm.txt 2>&1 || { cat gpurun_out/tsdf_overlap_ab_r3bm.txt; exit 1; }
cat gpurun_out/tsdf_overlap_ab_r3bm.txt
