#!/bin/bash
# PMC passes for the bench line's roofline.traffic and l2_hit fields
# (profiles/r03/pmc.json via tools/pmc_r03.py): for the headline OCC epoch
# and for C4 (Calvin), FETCH_SIZE, WRITE_SIZE and TCC_HIT_sum + TCC_MISS_sum,
# each in its own run (kernel trace only, own kill timeout).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${TAG:-pmc3}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
H="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
C="$R/bench.py --only C4 --steps 2 --warmup 1"
run() {  # name counters args...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$n" -o run \
    -- python3 "$@" > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
}
run h_fetch FETCH_SIZE $H
run h_write WRITE_SIZE $H
run h_l2 "TCC_HIT_sum TCC_MISS_sum" $H
run c_fetch FETCH_SIZE $C
run c_write WRITE_SIZE $C
run c_l2 "TCC_HIT_sum TCC_MISS_sum" $C
python3 "$R/tools/pmc_r03.py" "$OUT" "$OUT/pmc.json" || exit 1
echo "pmc done"
