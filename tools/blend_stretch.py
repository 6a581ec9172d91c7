#!/usr/bin/env python3
"""Why a blend runs longer with frames in flight (round-3 verdict, item 7).

    python tools/blend_stretch.py <dir with a rocprofv3 *kernel_trace.csv> [--lanes 4]

From the kernel trace of a bench run with frames in flight, takes every blend launch
(k_blend_w, any template) and, for each, the time other kernels ran concurrently with
it, split by kernel family.  Reports:
  * the blend's duration: one frame at a time (launches no other kernel overlapped)
    against in flight;
  * per family, the mean overlap per blend and the share of blends it overlapped;
  * a least-squares attribution of the stretch: duration = d0 + sum_k c_k * overlap_k,
    so c_k is the blend time lost per microsecond of family k running beside it and
    c_k * mean overlap_k the stretch that family accounts for.
"""
import argparse
import csv
import glob
import os
import re

import numpy as np


def family(name):
    m = re.search(r"(k_\w+)", name)
    if m:
        return m.group(1)
    return name.split("(")[0].strip()[:40]


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for r in csv.DictReader(open(f[0])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--min-blend-us", type=float, default=100.0,
                    help="ignore blend launches shorter than this (tiny diagnostic images)")
    a = ap.parse_args()
    rows = load(a.trace_dir)
    starts = np.array([r[0] for r in rows], dtype=np.int64)
    ends = np.array([r[1] for r in rows], dtype=np.int64)
    longest = int((ends - starts).max())
    blends = [i for i, r in enumerate(rows) if r[2] == "k_blend_w" and "true" not in r[3].split(",")[0]
              and (r[1] - r[0]) >= a.min_blend_us * 1e3]
    fams = sorted({r[2] for r in rows if r[2] != "k_blend_w"})
    fi = {k: j for j, k in enumerate(fams)}
    dur = np.zeros(len(blends))
    ov = np.zeros((len(blends), len(fams)))
    for bi, i in enumerate(blends):
        s, e = rows[i][0], rows[i][1]
        dur[bi] = (e - s) / 1e3
        lo = np.searchsorted(starts, s - longest)
        hi = np.searchsorted(starts, e)
        for j in range(lo, hi):
            if j == i:
                continue
            o = min(e, rows[j][1]) - max(s, rows[j][0])
            if o > 0 and rows[j][2] != "k_blend_w":
                ov[bi, fi[rows[j][2]]] += o / 1e3
    alone = ov.sum(axis=1) == 0
    print(f"blend launches: {len(blends)} ({int(alone.sum())} with no other kernel beside them)")
    if alone.any():
        print(f"  alone:     mean {dur[alone].mean():.1f} us, median {np.median(dur[alone]):.1f} us")
    if (~alone).any():
        print(f"  in flight: mean {dur[~alone].mean():.1f} us, median {np.median(dur[~alone]):.1f} us")
    base = float(np.median(dur[alone])) if alone.sum() >= 5 else float(dur.min())
    sel = ~alone
    if sel.sum() < len(fams) + 2:
        return
    X = np.concatenate([np.ones((int(sel.sum()), 1)), ov[sel]], axis=1)
    coef, *_ = np.linalg.lstsq(X, dur[sel], rcond=None)
    stretch = dur[sel].mean() - base
    print(f"\nstretch in flight: {stretch:.1f} us per blend over the one-at-a-time median {base:.1f} us")
    print(f"least squares: d0 = {coef[0]:.1f} us\n")
    print(f"{'family beside the blend':<28}{'blends overlapped':>18}{'mean overlap us':>17}{'c (us/us)':>11}"
          f"{'accounts for us':>17}")
    order = np.argsort(-(coef[1:] * ov[sel].mean(axis=0)))
    for j in order:
        m = ov[sel, j].mean()
        if m <= 0:
            continue
        print(f"{fams[j]:<28}{100 * (ov[sel, j] > 0).mean():>17.0f}%{m:>17.1f}{coef[1 + j]:>11.3f}"
              f"{coef[1 + j] * m:>17.1f}")


if __name__ == "__main__":
    main()
