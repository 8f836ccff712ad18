#!/bin/bash
# HBM traffic of the roofline kernel: rocprofv3 --pmc passes over a short
# bench run, one counter group per pass (FETCH_SIZE and WRITE_SIZE cannot
# share one), kernel trace only, each pass under its own kill timeout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" k_sw_ > "$OUT/summary.txt" 2>&1
cp -f "$R/profiles/traffic.json" "$OUT/traffic.json" 2>/dev/null || true
python3 "$R/tools/traffic.py" "$OUT" "k_sw_filter" "1048576:0.9:16:k_sw_filter" "$OUT/traffic.json" || exit 1
cp -f "$OUT/traffic.json" "$R/profiles/traffic.json"
echo "pmc done"
