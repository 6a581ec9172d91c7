#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter over the launches of the LATEST process
in each rocprofv3 --pmc output directory (tools/profile.sh layout).

    python tools/pmc_agg.py [gpurun_out/prof] [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
sub = sys.argv[2] if len(sys.argv) > 2 else "k_blend"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    last = max(int(r["Process_Id"]) for r in rows if r["Process_Id"].isdigit())
    for r in rows:
        if int(r["Process_Id"]) != last or sub not in r["Kernel_Name"]:
            continue
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k[:90])
    for c, v in sorted(d.items()):
        print(f"  {c:26s} launches={len(v):4d} mean={sum(v) / len(v):.5g}")
