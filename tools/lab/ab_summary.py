#!/usr/bin/env python3
"""Aggregate 'AB tag op q ms chk' lines: median/min per (op, q, tag), checksum agreement."""
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
chk = defaultdict(set)
for line in open(sys.argv[1]):
    if not line.startswith("AB "):
        continue
    _, tag, op, q, ms, c = line.split()
    rows[(op, q, tag)].append(float(ms))
    chk[(op, q)].add(c)
n, B = 16384, 65536
for (op, q, tag), ts in sorted(rows.items()):
    med = statistics.median(ts)
    print(f"{op:8s} q={q:<30s} {tag:8s} median {med:8.3f} ms  min {min(ts):8.3f}  n={len(ts)}  "
          f"{B / med * 1e3 / 1e6:7.3f} M/s  {24 * n * B / (med * 1e-3) / 1e9:7.1f} GB/s")
for k, v in chk.items():
    if len(v) != 1:
        print("CHECKSUM MISMATCH", k, v)
