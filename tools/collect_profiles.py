"""Copy one GPU round's outputs (tools/gpu_round.sh TAG=<tag>) from gpurun_out/
into profiles/r1/ and derive profiles/r1/traffic.json from the PMC passes.
usage: python tools/collect_profiles.py <tag>"""
import csv
import glob
import json
import math
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src, dst = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles", "r1")
os.makedirs(os.path.join(dst, "pmc_raw"), exist_ok=True)
copies = {f"bench_{tag}.json": "bench.json", f"prof_{tag}/run_kernel_stats.csv": "bench_kernel_stats.csv",
          f"bench_rehearsal_{tag}.json": "bench_rehearsal_2rank_gloo.json", f"pytest_gpu_{tag}.log": "pytest_gpu.log"}
for a, b in copies.items():
    shutil.copy(os.path.join(src, a), os.path.join(dst, b))


def per_dispatch(kind):
    """{kernel: {counter: average per dispatch}} over the pass CSVs"""
    out = {}
    for i, f in enumerate(sorted(glob.glob(os.path.join(src, f"pmc_{kind}_{tag}", "p*", "p_counter_collection.csv")))):
        shutil.copy(f, os.path.join(dst, "pmc_raw", f"{kind}_pass{i + 1}.csv"))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            out.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    summ = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
                           os.path.join(src, f"pmc_{kind}_{tag}")], capture_output=True, text=True).stdout
    open(os.path.join(dst, f"pmc_{kind}_kernel.txt"), "w").write(summ)
    return {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in out.items()}


traffic = {}
for kind, nd in (("match", 1), ("tsdf", 1)):
    kern = per_dispatch(kind)
    rd = sum(2 * c["FETCH_SIZE"] * 1024 * nd for c in kern.values())
    wr = sum(c["WRITE_SIZE"] * 1024 * nd for c in kern.values())
    traffic[kind] = {"bytes_per_step": rd + wr, "read_bytes_per_step": rd, "write_bytes_per_step": wr,
                     "dispatches_per_step": nd, "kernels": sorted(kern)}
traffic["source"] = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/pmc.sh, GPU round {tag}, "
                     "profiles/r1/pmc_raw); FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half the bytes "
                     "of wide streaming reads); workloads: C3 all-pairs match launch (tools/run_match_once.py), C5 "
                     "full 257-frame fusion, one launch of each pre-pass and of the fusion kernel (tools/run_tsdf_once.py)")
json.dump(traffic, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
print(json.dumps(traffic, indent=1))
