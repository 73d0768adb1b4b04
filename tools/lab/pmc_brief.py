#!/usr/bin/env python3
"""One-line PMC digest per profile summary (lab tool).
usage: pmc_brief.py <summary.json> ..."""
import json
import sys

for f in sys.argv[1:]:
    s = json.load(open(f))
    p = s["pmc_per_launch_avg"]
    w = p["SQ_WAVE_CYCLES"]
    ns = float(s.get("kernel_avg_ns") or s["kernel_stats"][0]["AverageNs"])
    clk = p.get("GRBM_GUI_ACTIVE", 0) / 8 / (ns * 1e-9) / 1e9
    print(f, f"{ns / 1e6:.3f} ms vgpr {s.get('vgpr')} clk {clk:.2f} GHz")
    print("  per wave:", {k[3:]: round(v / p["SQ_WAVES"]) for k, v in p.items() if k.startswith("SQ_") and k != "SQ_WAVES"})
    print(f"  wait_any {p['SQ_WAIT_ANY'] / w:.2f} wait_inst {p['SQ_WAIT_INST_ANY'] / w:.2f} "
          f"active {p['SQ_ACTIVE_INST_ANY'] / w:.2f} lds_conflict/lds_active {p['SQ_LDS_BANK_CONFLICT'] / max(1, p.get('SQ_LDS_IDX_ACTIVE', 0)):.2f}")
