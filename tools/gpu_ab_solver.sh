#!/bin/bash
# A/B of OCC solvers on the headline and C2 / C3 / C5 (device ms per epoch):
#   VARIANTS="3:0 4:1 4:2" tools/gpu_ab_solver.sh   (solver:ck_level)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-ab}"
mkdir -p "$O"
cd "$R"
for v in ${VARIANTS:-3:0 4:1 4:2 4:3}; do
  s=${v%%:*}; l=${v##*:}
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --solver $s --ck-level $l > "$O/h_$s_$l.json" 2> "$O/h.err" || { tail -5 "$O/h.err"; exit 1; }
  timeout -k 10 300 python -u bench.py --only C2,C3,C5 --steps 10 --warmup 3 --solver $s --ck-level $l > "$O/s_$s_$l.json" 2> "$O/s.err" || { tail -5 "$O/s.err"; exit 1; }
  python3 - "$O/h_$s_$l.json" "$O/s_$s_$l.json" "$v" <<'PY'
import json, sys
h = json.load(open(sys.argv[1])); s = json.load(open(sys.argv[2]))
e = h["epoch"]
print(f"{sys.argv[3]:6s} head dev {e['device_ms']:.4f} wall {h['ms_per_step']:.4f} rounds {e['rounds']} par {e['parity_vs_oracle']} | " +
      " ".join(f"{k} {v['device_ms']:.4f}/{v['rounds']}/{v['parity_vs_oracle']}" for k, v in s.items()))
PY
done
