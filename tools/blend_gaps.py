# Blend durations alone vs in flight and the gaps between consecutive in-flight blends.
# python tools/blend_gaps.py kt_kernel_trace.csv
import csv, re, sys, numpy as np
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:30]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
b = [(s, e) for s, e, k in rows if k == "k_blend_w"]
b = np.array(b, dtype=np.int64)
dur = (b[:, 1] - b[:, 0]) / 1e3
gap = (b[1:, 0] - b[:-1, 1]) / 1e3
# classify: pipelined if any non-blend kernel overlaps the blend
starts = np.array([s for s, e, k in rows]); ends = np.array([e for s, e, k in rows]); names = [k for s, e, k in rows]
piped = []
for (s, e) in b:
    i0 = np.searchsorted(starts, s - 2_000_000); i1 = np.searchsorted(starts, e)
    ov = any(names[i] != "k_blend_w" and starts[i] < e and ends[i] > s for i in range(i0, i1))
    piped.append(ov)
piped = np.array(piped)
print("blends", len(b), "pipelined", piped.sum())
print("dur alone mean %.1f us, pipelined mean %.1f us" % (dur[~piped].mean(), dur[piped].mean()))
pg = gap[piped[1:] & piped[:-1]]
print("gap between consecutive pipelined blends: mean %.1f median %.1f p90 %.1f us" % (pg.mean(), np.median(pg), np.percentile(pg, 90)))
print("pipelined blend period (start to start) median %.1f us" % np.median(np.diff(b[piped][:, 0]) / 1e3))
