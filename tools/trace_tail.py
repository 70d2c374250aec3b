"""Print the last N kernels of a rocprofv3 kernel trace with durations and the
gaps between them: python tools/trace_tail.py <trace.csv> [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'][:48]:48s} dur {(e - s) / 1e3:8.1f} us  gap {gap:7.1f} us  "
          f"grid {r.get('Grid_Size_X', '')} wg {r.get('Workgroup_Size_X', '')} lds {r.get('LDS_Block_Size', r.get('Lds_Size', ''))} "
          f"vgpr {r.get('VGPR_Count', r.get('Arch_VGPR_Count', ''))}")
    prev = e
