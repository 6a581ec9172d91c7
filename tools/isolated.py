#!/usr/bin/env python3
"""Per-kernel average duration over launches that overlapped no other kernel
(the bench's one-frame-at-a-time segment), from a rocprofv3 kernel trace csv.

    python tools/isolated.py gpurun_out/prof3/kt/kt_kernel_trace.csv"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>(]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][:50]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
iso = collections.defaultdict(list)
max_end = -1
for i, (s, e, k) in enumerate(ev):
    nxt = ev[i + 1][0] if i + 1 < len(ev) else 1 << 62
    if s >= max_end and e <= nxt:
        iso[k].append(e - s)
    max_end = max(max_end, e)
tot = 0.0
print(f"{'kernel':<34}{'isolated':>9}{'avg_us':>10}")
for k, v in sorted(iso.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    print(f"{k:<34}{len(v):>9}{sum(v) / len(v) / 1e3:>10.2f}")
