#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 csv) into a text table.

Per kernel: calls, average duration (kernel trace), and per-launch HBM traffic
from the separate FETCH_SIZE / WRITE_SIZE passes.  Units and gfx950
corrections follow MI355X_MICROARCH.md section HBM: the counters are in KiB
(x1024) and FETCH_SIZE reads half the bytes of a wide coalesced stream but
exactly the bytes of scattered 64-B record gathers (own calibration), so the
corrected read traffic is reported next to the raw value: x2 for streaming
kernels, x1 for the blend (fetch_factor).

    python tools/summarize_prof.py gpurun_out/prof > profiles/r01_rocprof_summary.txt
    python tools/summarize_prof.py gpurun_out/prof --pmc-json gpurun_out/pmc_TAG.json
        (the PMC columns from the --json output, once the csv have been slimmed away)
"""
import collections
import csv
import os
import re
import sys


# FETCH_SIZE correction per access pattern (tools/microbench/gather_fetch.hip,
# profiles/r01_fetch_calibration.txt): wide coalesced streams issue 128-B
# requests tallied at 64 B (x2, the guide's correction); scattered 64-B record
# gathers (the blend's splat records, 48 or 64 B of a 64-B record per lane) issue
# one 64-B request each and are counted exactly (x1).
GATHER_KERNELS = ("k_blend_w",)


def fetch_factor(kernel: str) -> float:
    return 1.0 if kernel.startswith(GATHER_KERNELS) else 2.0


def short(name: str) -> str:
    m = re.search(r"(k_\w+(?:<[^>(]*>)?)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][:60]


def main(d, pmc_json=None):
    stats = list(csv.DictReader(open(os.path.join(d, "kt", "kt_kernel_stats.csv"))))
    pmc = {}
    if pmc_json:
        import json
        ks = json.load(open(pmc_json))["kernels"]
        pmc["FETCH_SIZE"] = {k: v["fetch_bytes_raw"] for k, v in ks.items() if "fetch_bytes_raw" in v}
        pmc["WRITE_SIZE"] = {k: v["write_bytes"] for k, v in ks.items() if "write_bytes" in v}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(d, f"pmc_{c}", "pmc_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
        pmc[c] = {k: sum(v) / len(v) for k, v in agg.items()}
    print("rocprofv3 --kernel-trace --stats; PMC FETCH_SIZE and WRITE_SIZE in separate passes")
    print(f"{'kernel':<34}{'calls':>7}{'avg_us':>10}{'pct':>7}{'FETCH_MB':>10}{'corrFETCH_MB':>13}{'WRITE_MB':>10}{'GB/s(cF+W)':>12}")
    for r in stats:
        k = short(r["Name"])
        avg_us = float(r["AverageNs"]) / 1e3
        f = pmc.get("FETCH_SIZE", {}).get(k)
        w = pmc.get("WRITE_SIZE", {}).get(k)
        fmt = lambda v: f"{v / 1e6:10.2f}" if v is not None else f"{'-':>10}"
        cf = fetch_factor(k) * f if f is not None else None
        gbs = (cf + w) / (avg_us * 1e-6) / 1e9 if (f is not None and w is not None and avg_us > 0) else None
        print(f"{k:<34}{int(r['Calls']):>7}{avg_us:>10.2f}{float(r['Percentage']):>7.2f}{fmt(f)}"
              f"{(f'{cf / 1e6:13.2f}' if f is not None else f'{chr(45):>13}')}{fmt(w)}"
              f"{(f'{gbs:12.1f}' if gbs is not None else f'{chr(45):>12}')}")


def write_json(d, out, config, source):
    """Per-kernel HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, bytes) for bench.py."""
    import json
    res = {}
    pm = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(d, f"pmc_{c}", "pmc_counter_collection.csv")
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
        pm[c] = {k: sum(v) / len(v) for k, v in agg.items()}
    for k in pm["FETCH_SIZE"]:
        if k in pm["WRITE_SIZE"]:
            res[k] = {"fetch_bytes_raw": pm["FETCH_SIZE"][k],
                      "fetch_bytes_corrected": fetch_factor(k) * pm["FETCH_SIZE"][k],
                      "fetch_correction": fetch_factor(k), "write_bytes": pm["WRITE_SIZE"][k]}
    # any other counter passes present (SQ_*): per-kernel mean per launch, latest process only
    import glob
    for f in glob.glob(os.path.join(d, "pmc_*", "pmc_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        last = max(int(r["Process_Id"]) for r in rows)
        agg = collections.defaultdict(list)
        for r in rows:
            if int(r["Process_Id"]) == last and not r["Counter_Name"].endswith("_SIZE"):
                agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in agg.items():
            res.setdefault(k, {})[c] = sum(v) / len(v)
    json.dump({"config": config, "source": source, "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--json":
        write_json(sys.argv[1], sys.argv[3], int(sys.argv[4]), sys.argv[5])
    elif len(sys.argv) > 3 and sys.argv[2] == "--pmc-json":
        main(sys.argv[1], sys.argv[3])
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
