"""The second roofline of a profiled kernel: VALU issue.

A kernel that does not stream at HBM speed is bound by the vector ALU's issue
rate when its instruction stream, issued back to back, already takes as long
as the kernel.  This module turns a profile summary (tools/summarize_profile.py:
the dynamic SQ_INSTS_VALU per launch, the static VALU mix of the exact kernel
from the shipped library, optionally GRBM_GUI_ACTIVE / SQ_LDS_IDX_ACTIVE for
the clock held and the LDS-array busy share) and the measured
per-instruction issue rates (tools/lab/valu_rates.hip on MI355X,
profiles/r6_valu_rates.json) into:

  issue_floor_ms  = SQ_INSTS_VALU x (sum_i f_i c_i) / (SIMDs x clock)
                    f_i = static share of mnemonic i in the kernel,
                    c_i = 256 / rate_i  cycles per wave64 instruction per SIMD
                    (rate_i in lane-ops per CU per clock, 4 SIMDs per CU);
  frac            = issue_floor_ms / kernel_ms   (1.0 = the VALU issued
                    every cycle of the kernel on every SIMD);
  achieved        = SQ_INSTS_VALU / (CUs x clock x kernel time), wave
                    instructions per CU-cycle, against peak 2.0 (full-rate
                    instructions) and 1.0 (half-rate: 32-bit multiplies,
                    v_mad_u64_u32, three-operand and carry forms, 64-bit ops).

The rates were measured at the clock the chip held and normalised to the
nominal 2.4 GHz, and the floor uses the same nominal clock, so the DVFS of
the microbenchmark is folded into the costs.  Static shares stand in for the
dynamic ones (loops run their bodies several times, cold slow paths not at
all); `unmeasured_share` is the static share of mnemonics the table lacks,
priced at the full rate (2 cycles).
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RATES = os.path.join(ROOT, "profiles", "r6_valu_rates.json")
N_CU = 256
SIMDS_PER_CU = 4
CLOCK_GHZ = 2.4
FULL_RATE_CYC = 2.0  # wave64 on a 32-lane SIMD


def parse_rates_text(txt):
    """valu_rates output -> {mnemonic: lane-ops per CU per clock}.  A row
    timing two instructions (`a+b`) gives b's rate when a's is known."""
    rows = {}
    for line in txt.splitlines():
        m = re.match(r"^(\S+)\s+[\d.]+ ms\s+[\d.]+ Tlane-ops/s\s+([\d.]+) lane-ops/CU/clk", line)
        if m:
            rows[m.group(1)] = float(m.group(2))
    rates = {}
    for name, r in rows.items():
        if "+" in name or "(" in name:
            continue
        rates[name] = r
    # v_cndmask_b32: the row reading an SGPR mask (the form the kernels use);
    # the VCC-reading row of the first table measured 12.5 (a loop that reads
    # a VCC no instruction writes: not the kernels' pattern) and is not used
    rates.pop("v_cndmask_b32", None)
    if "v_cndmask_b32(sgpr)" in rows:
        rates["v_cndmask_b32"] = rows["v_cndmask_b32(sgpr)"]
    return rates


def load_rates(path=RATES):
    try:
        return json.load(open(path))["rates"]
    except (OSError, ValueError, KeyError):
        return None


def issue_cycles(mnemonic, rates):
    """(cycles per wave64 instruction per SIMD, measured?)"""
    r = rates.get(mnemonic)
    if r:
        return 256.0 / r, True
    return FULL_RATE_CYC, False


def valu_roofline(summary, rates, kernel_ms=None, n_cu=N_CU, clock_ghz=CLOCK_GHZ):
    """VALU-issue roofline record of one profile summary, or None without
    SQ_INSTS_VALU / a static mix / rates.  kernel_ms: the time to price
    against (default the profile's own kernel-trace average)."""
    pmc = summary.get("pmc_per_launch_avg", {})
    mix = summary.get("valu_static_mix")
    insts = pmc.get("SQ_INSTS_VALU")
    prof_ms = summary.get("kernel_trace_full_batch", {}).get("avg_ns", 0) / 1e6 or None
    if not insts or not mix or not rates or not prof_ms:
        return None
    total = sum(mix.values())
    cyc = 0.0
    unmeasured = 0
    for mn, cnt in mix.items():
        c, ok = issue_cycles(mn, rates)
        cyc += cnt * c
        if not ok:
            unmeasured += cnt
    cyc_per_inst = cyc / total
    simds = n_cu * SIMDS_PER_CU
    floor_ms = insts * cyc_per_inst / simds / (clock_ghz * 1e9) * 1e3
    out = {
        "bound": "valu",
        "unit": "fraction of VALU issue cycles",
        "issue_floor_ms": floor_ms,
        "cycles_per_valu_inst": cyc_per_inst,
        "valu_insts_per_launch": insts,
        "profile_kernel_ms": prof_ms,
        "frac_profile": floor_ms / prof_ms,
        "achieved_inst_per_cu_cycle_profile": insts / (n_cu * clock_ghz * 1e9 * prof_ms * 1e-3),
        "peak_inst_per_cu_cycle": {"full_rate": SIMDS_PER_CU / FULL_RATE_CYC, "half_rate": SIMDS_PER_CU / 4.0,
                                   "this_mix": SIMDS_PER_CU / cyc_per_inst},
        "unmeasured_share": unmeasured / total,
        "clock_ghz": clock_ghz,
        "mix_source": "static VALU mix of the exact kernel in the loaded library (tools/isa_mix.py)",
        "rates_source": "profiles/r6_valu_rates.json (tools/lab/valu_rates.hip)",
    }
    if kernel_ms:
        out["kernel_ms"] = kernel_ms
        out["frac"] = floor_ms / kernel_ms
        out["achieved_inst_per_cu_cycle"] = insts / (n_cu * clock_ghz * 1e9 * kernel_ms * 1e-3)
    for k in ("effective_clock_ghz", "valu_insts_per_cu_cycle_measured", "lds_busy_frac"):
        if summary.get(k) is not None:
            out[k] = summary[k]
    # The clock the kernel held (GRBM_GUI_ACTIVE / 8 over its duration) is
    # below 2.4 GHz for the multiply-dense kernels (1.9-2.2 GHz): the same
    # issue cycles take longer there, so the floor at the held clock is the
    # bound the kernel can actually reach.
    clk = summary.get("effective_clock_ghz")
    if clk:
        held = floor_ms * clock_ghz / clk
        out["issue_floor_ms_at_held_clock"] = held
        out["frac_profile_at_held_clock"] = held / prof_ms
        if kernel_ms:
            out["frac_at_held_clock"] = held / kernel_ms
    return out


def hbm_frac_profile(summary, algorithmic_bytes, peak_gbs=8000.0):
    """The HBM roofline fraction priced on the profile's own kernel time (the
    bench's `frac` uses the HIP-event time of its run)."""
    prof_ms = summary.get("kernel_trace_full_batch", {}).get("avg_ns", 0) / 1e6
    if not prof_ms:
        return None
    return algorithmic_bytes / (prof_ms * 1e-3) / 1e9 / peak_gbs


if __name__ == "__main__":
    import sys

    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r6a", "valu_rates.txt")
    rates = parse_rates_text(open(src).read())
    json.dump({"source": os.path.relpath(src, ROOT), "unit": "lane-ops per CU per nominal 2.4 GHz clock",
               "rates": rates}, open(RATES, "w"), indent=1)
    for k, v in sorted(rates.items(), key=lambda kv: -kv[1]):
        print(f"{k:24s} {v:7.1f}  {256.0 / v:5.2f} cycles per wave64 instruction per SIMD")
