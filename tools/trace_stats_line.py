"""One line per rocprofv3 kernel_stats.csv: the sfmhip kernels' average durations (us) and their sum."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
rows = []
for r in csv.DictReader(open(f)):
    if "sfmhip" in r["Name"]:
        a = float(r["AverageNs"]) / 1e3
        tot += a
        rows.append(f"{r['Name'].split('(')[0].replace('sfmhip::', '')[-28:]}={a:.1f}")
print(sys.argv[2] if len(sys.argv) > 2 else "", f"sum {tot:.1f} us |", " ".join(rows))
