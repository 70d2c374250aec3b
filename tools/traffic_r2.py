"""Derive profiles/<round>/traffic.json (HBM bytes per step of the dominant kernels)
from a tools/gpu_traffic_r2.sh run, and copy the PMC summaries next to it.
usage: python tools/traffic_r2.py <tag> [round dir, default r2]"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r2"
rnd = sys.argv[2] if len(sys.argv) > 2 else "r2"
src, dst = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
old = os.path.join(dst, "traffic.json")
traffic = json.load(open(old)) if os.path.exists(old) else {}   # kinds without a run here keep their entry
for kind in ("match", "match_int8", "tsdf", "render", "ba", "vq"):
    if not glob.glob(os.path.join(src, f"pmc_{kind}_{tag}", "p*")):
        continue
    per = {}
    for f in glob.glob(os.path.join(src, f"pmc_{kind}_{tag}", "p*", "p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            per.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    avg = {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in per.items()}
    rd = sum(2 * c.get("FETCH_SIZE", 0.0) * 1024 for c in avg.values())
    wr = sum(c.get("WRITE_SIZE", 0.0) * 1024 for c in avg.values())
    traffic[kind] = {"bytes_per_step": rd + wr, "read_bytes_per_step": rd, "write_bytes_per_step": wr,
                     "per_kernel_bytes": {k: 2 * c.get("FETCH_SIZE", 0.0) * 1024 + c.get("WRITE_SIZE", 0.0) * 1024
                                          for k, c in avg.items()},
                     "kernels": sorted(avg)}
    s = os.path.join(src, f"pmc_{kind}_{tag}.txt")
    if os.path.exists(s):
        shutil.copy(s, os.path.join(dst, f"pmc_{kind}.txt"))
traffic["source_" + tag] = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/gpu_traffic_r2.sh, tag {tag}); "
                     "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half the bytes of wide streaming "
                     "reads); per dispatch: the C3 all-pairs match launch (tools/run_match_once.py), one C5 TSDF call "
                     "= every pre-pass + the fusion (tools/run_tsdf_once.py), one V2+V4 render launch "
                     "(tools/run_render_once.py), one BA solve launch (tools/run_ba_once.py), one vq call "
                     "(tools/run_vq_once.py): whichever ran under this tag")
json.dump(traffic, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
print(json.dumps({k: (v["bytes_per_step"] / 1e9 if isinstance(v, dict) else v) for k, v in traffic.items()}, indent=1))
