"""Summarise tools/pmc.sh output: per-kernel average of every counter plus the
derived numbers used in DESIGN.md (clock, HBM bytes with the gfx950 FETCH_SIZE
x2 correction, VALU utilisation, L2 hit rate)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for f in glob.glob(f"{root}/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-60:]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k, c in vals.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    dt = sum(durs[k]) / len(durs[k])
    print(f"== {k}  (profiled duration ~{dt * 1e3:.2f} ms)")
    for n in sorted(avg):
        print(f"   {n:32s} {avg[n]:.4g}")
    if "GRBM_GUI_ACTIVE" in avg:
        clk = avg["GRBM_GUI_ACTIVE"] / 8 / dt
        print(f"   clock ~ {clk / 1e9:.2f} GHz (GRBM_GUI_ACTIVE/8/duration)")
    if "FETCH_SIZE" in avg:
        print(f"   HBM read  ~ {2 * avg['FETCH_SIZE'] * 1024 / 1e9:.3f} GB (FETCH_SIZE x2, gfx950 correction)")
    if "WRITE_SIZE" in avg:
        print(f"   HBM write ~ {avg['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
    if "TCC_HIT_sum" in avg:
        print(f"   L2 hit    ~ {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):.1%}")
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        print(f"   VALU-active / wave-cycles {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.1%}, "
              + (f"wait_any {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.1%}, " if "SQ_WAIT_ANY" in avg else "")
              + (f"wait_inst {avg['SQ_WAIT_INST_ANY'] / avg['SQ_WAVE_CYCLES']:.1%}" if "SQ_WAIT_INST_ANY" in avg else ""))
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8 * 256   # CU-cycles (8 XCDs x 32 CUs)
        for n in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TD_TC_STALL_sum",
                  "TCP_PENDING_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"):
            if n in avg:
                print(f"   {n[:-4]} per CU-cycle {avg[n] / cyc:.1%}")
        if "SQ_INSTS_VALU" in avg:   # a wave64 VALU op holds its SIMD 4 cycles (4 SIMDs per CU)
            print(f"   VALU issue per SIMD-cycle ~ {avg['SQ_INSTS_VALU'] * 4 / (cyc * 4):.1%} (x4 cycles per op)")
