#!/bin/bash
# PMC passes for profiles/r06/pmc.json (tools/pmc_r05.py): the headline OCC
# epoch, C4 (Calvin) and C2, C3, C5, MAAT_1M (back to back in one bench run
# per pass); FETCH_SIZE, WRITE_SIZE and TCC_HIT_sum + TCC_MISS_sum each in
# its own run (kernel trace only, own kill timeout).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${TAG:-pmc6}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
H="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --pipeline 0"
C="$R/bench.py --only C4 --steps 2 --warmup 1"
S="$R/bench.py --only C2,C3,C5,MAAT_1M --steps 2 --warmup 1"
run() {  # name counters args...
  local n=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$n" -o run \
    -- python3 "$@" > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "pass $n ok"
}
run h_fetch FETCH_SIZE $H
run h_write WRITE_SIZE $H
run h_l2 "TCC_HIT_sum TCC_MISS_sum" $H
run c4_fetch FETCH_SIZE $C
run c4_write WRITE_SIZE $C
run c4_l2 "TCC_HIT_sum TCC_MISS_sum" $C
run s_fetch FETCH_SIZE $S
run s_write WRITE_SIZE $S
run s_l2 "TCC_HIT_sum TCC_MISS_sum" $S
python3 "$R/tools/pmc_r05.py" "$OUT" "$OUT/pmc.json" || exit 1
echo "pmc done"
