#!/bin/bash
# Round 5: the whole GPU suite, then the full bench line (secondaries included).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5q}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/gpu_suite.log" 2>&1 || { tail -30 "$O/gpu_suite.log"; exit 1; }
tail -2 "$O/gpu_suite.log"
timeout -k 10 500 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
if [ -z "$NOBENCH" ]; then
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
print("headline", round(j["ms_per_step"], 4), "ms/epoch", round(j["value"] / 1e9, 3), "G/s frac", round(j["roofline"]["frac"], 3), "lat", round(j["single_epoch"]["device_ms"], 4), "parity", j["epoch"]["parity_vs_oracle"])
for k, v in (j.get("other_configs") or {}).items():
    print(k, {x: v.get(x) for x in ("device_ms", "ms_per_epoch", "parity_vs_oracle", "device_ms_per_epoch")})
PY
fi
