#!/bin/bash
# The default bench line as the driver runs it (no profiler), then its summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5b}
mkdir -p "$O"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
print("headline", round(j["ms_per_step"], 4), "value", round(j["value"] / 1e9, 3), "frac", round(j["roofline"]["frac"], 3),
      "single", j.get("single_epoch", {}).get("device_ms"), "parity", j.get("parity"))
for k, v in (j.get("other_configs") or {}).items():
    print(k, {kk: v.get(kk) for kk in ("device_ms", "ms_per_epoch", "wall_ms", "parity", "rounds") if kk in v})
PY
