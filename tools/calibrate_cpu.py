#!/usr/bin/env python3
"""CPU-baseline calibration.

The bench's cpu_baseline is oracle/ref_cpu.c, the operation-for-operation
restatement of the reference's NTTProcessor::forward_ntt
(cpp/src/ntt_processor.cpp:262-311) and PolynomialRing::multiply
(cpp/src/polynomial_ring.cpp:421-447).  The reference itself cannot be built
here (cpp/include/modular_arithmetic.h includes <arm_neon.h>), but SURVEY.md
section 6 recorded the compiled reference's single-thread timings on this same
container class (8-core Xeon, g++ -O3) when the survey was written.  This
script times the restatement at the same configs, one thread, and writes the
ratio port / reference per config to profiles/r6_cpu_calibration.json, which
bench.py carries into cpu_baseline.calibration.

usage: python3 tools/calibrate_cpu.py [--reps R] [--out PATH]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

P27 = 132120577
P62 = 4611686018326724609
# SURVEY.md section 6 / BASELINE.md section 2 ([verified] compiled reference,
# 1 thread, microseconds per call)
REFERENCE_US = {
    ("forward_ntt", P27): {1024: 136.0, 4096: 599.0, 16384: 2843.0},
    ("multiply", P27): {1024: 427.0, 4096: 1816.0, 16384: 8603.0},
    ("forward_ntt", P62): {1024: 121.0, 4096: 596.0, 16384: 2896.0},
    ("multiply", P62): {1024: 372.0, 4096: 1820.0, 16384: 8650.0},
}


def host():
    model = "unknown"
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    return {"cpu_model": model, "nproc": os.cpu_count()}


def time_op(fn, reps):
    """(min, median) microseconds per call; the minimum is the ratio's basis
    (deterministic code: noise only adds time)."""
    fn()  # warm-up (tables, caches)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return min(ts), statistics.median(ts)


def calibrate(reps=15):
    import oracle

    rows = []
    for (op, q), ref in REFERENCE_US.items():
        for n, ref_us in ref.items():
            t = oracle.NTT(n, q)
            a = oracle.splitmix_fill(1, q, n).reshape(1, n)
            b = oracle.splitmix_fill(2, q, n).reshape(1, n)
            fn = (lambda: t.forward(a)) if op == "forward_ntt" else (lambda: t.polymul(a, b))
            us, med = time_op(fn, reps if n < 16384 else max(9, reps // 3))
            rows.append({"op": op, "q": q, "n": n, "port_us": us, "port_us_median": med, "reference_us": ref_us,
                         "ratio": us / ref_us})
    ratios = [r["ratio"] for r in rows]
    return {
        "what": "oracle/ref_cpu.c (restated NTTProcessor::forward_ntt, PolynomialRing::multiply), one thread, "
                "minimum over repeated single-polynomial calls, vs the compiled reference timed on this container class "
                "(SURVEY.md section 6)",
        "host": host(),
        "rows": rows,
        "ratio_min": min(ratios), "ratio_max": max(ratios), "ratio_median": statistics.median(ratios),
        "within_10pct": all(0.9 <= r <= 1.1 for r in ratios),
        "generated": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=41)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6_cpu_calibration.json"))
    a = ap.parse_args()
    res = calibrate(a.reps)
    json.dump(res, open(a.out, "w"), indent=1)
    for r in res["rows"]:
        print(f"{r['op']:12s} q={r['q']:<20d} N={r['n']:<6d} port {r['port_us']:9.1f} us  "
              f"reference {r['reference_us']:8.1f} us  ratio {r['ratio']:.3f}")
    print(f"ratio median {res['ratio_median']:.3f} [{res['ratio_min']:.3f}, {res['ratio_max']:.3f}]; "
          f"within +-10%: {res['within_10pct']}")


if __name__ == "__main__":
    main()
