"""Summarise a rocprofv3 kernel-trace CSV: for the last N dispatches matching a regex, their
start offsets and durations (us) relative to the first of them.  Writes a small text file so the
raw CSV can be deleted on the GPU box.  python tools/trace_summary.py <csv> <regex> <n> <out>"""
import csv
import re
import sys

path, rx, n, out = sys.argv[1], re.compile(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
rows = [r for r in csv.DictReader(open(path)) if rx.search(r["Kernel_Name"])]
rows = rows[-n:]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
with open(out, "w") as f:
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        f.write(f"{r['Kernel_Name'][:48]:48s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  "
                f"grid {r.get('Grid_Size_X', r.get('Grid_Size', ''))} wg {r.get('Workgroup_Size_X', r.get('Workgroup_Size', ''))}\n")
print(open(out).read())
