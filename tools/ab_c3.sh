#!/bin/bash
# A/B of sort / binning knobs (tools/ab_tune.py) on the given configs:
#   KNOBS="10:1024,2048 9:4,8" CONFIGS="2 3" bash tools/ab_c3.sh
set -u
mkdir -p gpurun_out
for c in ${CONFIGS:-3}; do
for kv in ${KNOBS}; do
  k=${kv%%:*}; v=${kv#*:}
  timeout -k 10 200 python tools/ab_tune.py --knob $k --values $v --config $c --rounds 3 --k-frames 20 > gpurun_out/ab_c${c}_k$k.log 2>&1 || exit $?
  python3 - "$c" "$k" <<'PY'
import json,sys
s=open(f"gpurun_out/ab_c{sys.argv[1]}_k{sys.argv[2]}.log").read()
d=json.loads(s[s.index('{\n'):])
print("config", sys.argv[1], "knob", sys.argv[2], {v: (x["depth_sort"], x["emit"], x["tile_sort"], x["total"], x["identical_to_first"]) for v,x in d["median_ms"].items()})
PY
done
done
