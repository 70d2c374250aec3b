"""Print a compact summary of a bench.py JSON line (headline + every secondary line)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"headline {d['value']:.0f} {d['unit']} {d['ms_per_step']:.2f} ms frac {d['roofline']['frac']:.3f}"
      f" | tsdf {d.get('tsdf_value', 0):.0f} {d.get('tsdf_unit', '')} {d.get('tsdf_ms_per_step', 0):.3f} ms")
for s in d.get("secondary", []):
    r = s.get("roofline") or {}
    extra = ""
    if "unchanged_sfm_py" in s:
        u = s["unchanged_sfm_py"]
        extra = (f" | sfm.py unchanged {u['s_per_pair'] * 1e3:.1f} ms/pair (residual {u['s_in_residual'] * 1e3:.1f}, "
                 f"{u['us_per_residual_call']:.0f} us/call; cpu {u.get('cpu_s_per_pair', 0) * 1e3:.1f})")
    print(f"  {s['metric'][:40]:40s} {s['value']:.4g} {s['unit']:18s} {s.get('ms_per_step', 0) or 0:.4f} ms "
          f"frac {r.get('frac', 0) or 0:.3f} {r.get('kernel', '')}{extra}")
