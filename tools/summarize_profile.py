#!/usr/bin/env python3
"""Summarize a rocprofv3 run of tools/gpu_evidence.sh into profiles/<tag>/.

Per kernel of interest: average duration (kernel trace stats), and per
launch the PMC counters.  HBM traffic per launch follows
/opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, are in KiB, and on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so
    traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Only launches of the full benchmark batch are used (the bench's 2-row parity
spot check is excluded by grid size).

usage: summarize_profile.py gpurun_out/prof_<tag> profiles/<tag> [--kernel-substr fwd_mul]
       [--workload kernel,n,batch,q[,mode]] [--build-id ID]

The summary records the exact demangled name of the profiled kernel (the
full-batch launches matching the substring) and the build id of the library
the run loaded (fhe_build_id()); bench.py uses a summary only when both match
the kernel it launches and the library it runs.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    ksub = sys.argv[sys.argv.index("--kernel-substr") + 1] if "--kernel-substr" in sys.argv else "fwd_mul"
    os.makedirs(dst, exist_ok=True)
    import datetime

    out = {"source": src, "kernel_substr": ksub,
           "generated": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")}
    if "--build-id" in sys.argv:
        out["build_id"] = sys.argv[sys.argv.index("--build-id") + 1]
    if "--workload" in sys.argv:
        parts = sys.argv[sys.argv.index("--workload") + 1].split(",")
        k, n, b, q = parts[:4]
        out["workload"] = {"kernel": k, "n": int(n), "batch": int(b), "q": int(q)}
        if len(parts) > 4:
            out["workload"]["mode"] = parts[4]
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        rows = list(csv.DictReader(open(stats[0])))
        out["kernel_stats"] = [
            {k: (r[k][:160] if k == "Name" else r[k]) for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
            for r in rows[:8]
        ]
        # the kernel this summary is about (kernel_stats is sorted by total
        # time, so its first row can be another kernel of the same run)
        mine = [r for r in rows if ksub in r["Name"]]
        if mine:
            top = max(mine, key=lambda r: float(r["TotalDurationNs"]) if "TotalDurationNs" in r else float(r["AverageNs"]))
            out["kernel_stats_name"] = top["Name"][:160]
            out["kernel_avg_ns"] = float(top["AverageNs"])
    per_counter = defaultdict(list)
    full_names = set()
    for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
        acc = defaultdict(float)
        names, grid, meta = {}, {}, {}
        for r in csv.DictReader(open(f)):
            if ksub not in r["Kernel_Name"]:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
            meta[r["Dispatch_Id"]] = (r.get("VGPR_Count"), r.get("LDS_Block_Size"))
        if not acc:
            continue
        gmax = max(grid.values())
        for d, g in grid.items():
            if g == gmax:
                full_names.add(names[d])
                out["vgpr"], out["lds_bytes"] = meta[d]
        for (d, c), v in acc.items():
            if grid[d] == gmax:
                per_counter[c].append(v)
    if len(full_names) == 1:
        out["kernel_name"] = next(iter(full_names))
        # per-dispatch durations of that exact kernel at the full grid, from
        # the kernel trace (kernel_stats averages every launch of the name)
        for tf in glob.glob(os.path.join(src, "trace", "*kernel_trace.csv")):
            durs, gmax = [], 0
            rows = [r for r in csv.DictReader(open(tf)) if r["Kernel_Name"] == out["kernel_name"]]
            for r in rows:
                gmax = max(gmax, int(r["Grid_Size_X"]))
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if int(r["Grid_Size_X"]) == gmax]
            if durs:
                out["kernel_trace_full_batch"] = {"dispatches": len(durs), "avg_ns": sum(durs) / len(durs),
                                                  "min_ns": min(durs), "max_ns": max(durs)}
    elif full_names:  # several kernels match: ambiguous, bench.py will not use it
        out["kernel_names"] = sorted(full_names)
    pmc = {c: sum(v) / len(v) for c, v in per_counter.items()}
    out["pmc_per_launch_avg"] = pmc
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        out["hbm_traffic_bytes_per_launch"] = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
        out["traffic_note"] = "(2*FETCH_SIZE + WRITE_SIZE) KiB; gfx950 FETCH_SIZE counts half of wide streaming reads"
    if "SQ_WAVE_CYCLES" in pmc:
        w = pmc["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in pmc:
                out[c + "_frac_of_wave_cycles"] = pmc[c] / w
    if "SQ_WAVES" in pmc and "SQ_INSTS_VALU" in pmc:
        out["valu_insts_per_wave"] = pmc["SQ_INSTS_VALU"] / pmc["SQ_WAVES"]
    # VALU-issue roofline inputs (tools/valu_roofline.py): the static VALU
    # mix of this exact kernel in the library the run loaded, and the
    # measured busy fraction where SQ_ACTIVE_INST_VALU was collected
    if out.get("kernel_name"):
        try:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            import isa_mix

            mix = isa_mix.valu_mix(out["kernel_name"])
            if mix is not None:
                out["valu_static_mix"] = dict(mix.most_common())
        except Exception as e:  # llvm tools missing: the roofline stays null
            out["valu_static_mix_error"] = str(e)[:200]
    if "GRBM_GUI_ACTIVE" in pmc:
        # GRBM_GUI_ACTIVE: GPU-busy cycles summed over the 8 XCDs
        # (MI355X_MICROARCH.md DVFS note): the clock the kernel ran at, and the
        # VALU instructions per CU per real cycle.  (SQ_ACTIVE_INST_VALU counts
        # one per VALU instruction on gfx950 -- equal to SQ_INSTS_VALU on every
        # microbenchmark kernel of profiles/r6b -- so it is no busy-cycle count.)
        cyc = pmc["GRBM_GUI_ACTIVE"] / 8
        kt = out.get("kernel_trace_full_batch", {}).get("avg_ns")
        if kt:
            out["effective_clock_ghz"] = cyc / kt
        if "SQ_INSTS_VALU" in pmc:
            out["valu_insts_per_cu_cycle_measured"] = pmc["SQ_INSTS_VALU"] / (256 * cyc)
        if "SQ_LDS_IDX_ACTIVE" in pmc:
            # LDS-array busy cycles summed over the 256 CUs
            out["lds_busy_frac"] = pmc["SQ_LDS_IDX_ACTIVE"] / (256 * cyc)
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
