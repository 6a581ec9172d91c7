#!/usr/bin/env python3
"""Per-launch-position breakdown of kernels that run several times per frame (e.g. the
depth sort's downsweeps): kernel-trace durations and PMC values grouped by the launch's
index inside its frame (frame boundaries = k_preprocess launches).

    python tools/pass_split.py gpurun_out/profg [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
sub = sys.argv[2] if len(sys.argv) > 2 else "k_radix_downsweep"


def positions(rows, key_name, key_val):
    """yield (position-in-frame, row) for rows whose kernel matches sub."""
    pos = None
    for r in rows:
        name = r["Kernel_Name"]
        if "k_preprocess" in name:
            pos = collections.Counter()
        if sub in name and pos is not None:
            yield pos[sub], r
            pos[sub] += 1


kt = list(csv.DictReader(open(os.path.join(root, "kt", "kt_kernel_trace.csv"))))
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = collections.defaultdict(list)
for p, r in positions(kt, None, None):
    dur[p].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{sub}: kernel-trace duration by launch position in the frame (us)")
for p in sorted(dur):
    v = sorted(dur[p])
    print(f"  pos {p}: n={len(v):4d} median={v[len(v) // 2]:8.2f} mean={sum(v) / len(v):8.2f}")
for f in sorted(glob.glob(os.path.join(root, "pmc_*", "pmc_counter_collection.csv"))):
    rows = list(csv.DictReader(open(f)))
    last = max(int(r["Process_Id"]) for r in rows)
    rows = [r for r in rows if int(r["Process_Id"]) == last]
    # one row per (dispatch, counter): group rows of a dispatch
    byd = collections.OrderedDict()
    for r in rows:
        byd.setdefault(int(r["Dispatch_Id"]), []).append(r)
    disp = [v[0] | {"_c": {x["Counter_Name"]: float(x["Counter_Value"]) for x in v}} for v in byd.values()]
    disp.sort(key=lambda r: int(r["Dispatch_Id"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p, r in positions(disp, None, None):
        for c, v in r["_c"].items():
            acc[p][c].append(v)
    for p in sorted(acc):
        print(f"  {os.path.basename(os.path.dirname(f))} pos {p}: " +
              " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(acc[p].items())))
