#!/bin/bash
# A/B of library variants (deneva_amd/libdcc.so.exp-<V>) on one bench config:
# VARIANTS="A B" CFG=C4 tools/ab_cfg.sh -> rocprofv3 kernel stats per variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abc; mkdir -p "$O"
for v in ${VARIANTS:-A B}; do
  cp "$R/deneva_amd/libdcc.so.exp-$v" "$R/deneva_amd/libdcc.so"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$O/$v" -o run -- python3 "$R/bench.py" --only ${CFG:-C4} --steps 5 --warmup 2 > "$O/$v.json" 2> "$O/$v.err") || exit 1
  echo "== $v"; tail -c 400 "$O/$v.json"; echo
  f=$(find "$O/$v" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"  {r['Name'][:50]:50s} calls {r['Calls']:>4} avg_us {float(r['AverageNs'])/1e3:8.1f}")
PY
done
