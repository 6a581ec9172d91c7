#!/usr/bin/env python3
"""Concurrency of the pipelined region from a rocprofv3 kernel trace.

    python tools/overlap.py gpurun_out/prof/kt

Finds the longest run of dispatches whose blend launches overlap (frames in
flight, gsr_render_path) and reports, over that window: wall time per frame,
busy time per kernel family (sum of durations / frames), the fraction of the
window with at least one blend running, and what ran concurrently with blends.
"""
import csv
import glob
import os
import re
import sys


def fam(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"])))
    rows.sort()
    blends = [r for r in rows if r[2].startswith("k_blend_w")]
    # overlapping blend pairs mark the pipelined segment
    ov = [i for i in range(1, len(blends)) if blends[i][0] < blends[i - 1][1]]
    if not ov:
        print("no overlapping blends")
        return
    # longest contiguous stretch of overlapping blends
    best, cur = (ov[0], ov[0]), (ov[0], ov[0])
    for a, b in zip(ov, ov[1:]):
        cur = (cur[0], b) if b == a + 1 else (b, b)
        if cur[1] - cur[0] > best[1] - best[0]:
            best = cur
    t0, t1 = blends[best[0] - 1][0], blends[best[1]][1]
    frames = best[1] - best[0] + 2
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    busy = {}
    for s, e, k in win:
        busy[k] = busy.get(k, 0) + (e - s)
    # union of blend intervals
    ivs = sorted((s, e) for s, e, k in win if k.startswith("k_blend_w"))
    un, cs, ce = 0, None, None
    for s, e in ivs:
        if cs is None or s > ce:
            if cs is not None:
                un += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    un += ce - cs
    wall = t1 - t0
    print(f"pipelined window: {frames} frames, {wall / 1e3:.1f} us, {wall / frames / 1e3:.1f} us/frame")
    print(f"at least one blend running: {100 * un / wall:.1f} % of the window")
    print(f"{'kernel':<28}{'us/frame (sum of durations)':>30}")
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"{k:<28}{v / frames / 1e3:>30.1f}")
    # per-frame gap: time with no blend running, attributed to the kernels running then
    gaps = {}
    prev = t0
    for s, e in ivs:
        pass


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/kt")
