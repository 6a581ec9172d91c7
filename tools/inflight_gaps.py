# Gaps between consecutive blends in the frames-in-flight region of a rocprofv3 kernel trace:
# what ran in them, and one example timeline.  python tools/inflight_gaps.py kt_kernel_trace.csv
import csv, re, sys, collections, numpy as np
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:30]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
b = [(s, e) for s, e, k in rows if k == "k_blend_w"]
# pipelined blends: a non-blend kernel overlapping
starts = np.array([s for s, e, k in rows])
def overlapped(s, e):
    i0 = np.searchsorted(starts, s - 3_000_000); i1 = np.searchsorted(starts, e)
    return any(rows[i][2] != "k_blend_w" and rows[i][0] < e and rows[i][1] > s for i in range(i0, i1))
pb = [x for x in b if overlapped(*x)]
# for a window of consecutive pipelined blends, examine each gap
busy = collections.Counter(); cnt = 0; gaps = []
tl = []
for (s0, e0), (s1, e1) in zip(pb, pb[1:]):
    if s1 - e0 > 1_000_000 or s1 < e0: continue
    gaps.append(s1 - e0); cnt += 1
    # kernels running in the gap: time each family spends inside [e0, s1]
    i0 = np.searchsorted(starts, e0 - 3_000_000); i1 = np.searchsorted(starts, s1)
    for i in range(i0, i1):
        s, e, k = rows[i]
        ov = min(e, s1) - max(s, e0)
        if ov > 0: busy[k] += ov
    if cnt == 50:   # print one example timeline
        for i in range(np.searchsorted(starts, s0 - 400_000), np.searchsorted(starts, e1 + 1)):
            s, e, k = rows[i]
            if e > s0 - 50_000: tl.append(f"{(s - s0)/1e3:8.1f} {(e - s0)/1e3:8.1f} {k}")
print("gaps", cnt, "mean gap us", np.mean(gaps) / 1e3)
for k, v in busy.most_common(15): print(f"{k:28s} {v / cnt / 1e3:8.1f} us per gap")
print("\n".join(tl[:80]))
