#!/bin/bash
# Dataflow solver diagnostics: debug stamps of one headline epoch, then PMC
# passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss) of the headline bench under
# solver 4, summarised per kernel (tools/pmc_kernels.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${TAG:-dfdiag}"
mkdir -p "$OUT"
cd "$R"
DCC_DF_DEBUG=1 timeout -k 10 200 python -u tools/df_diag.py > "$OUT/diag.log" 2>&1 || { tail -20 "$OUT/diag.log"; exit 1; }
cat "$OUT/diag.log" | grep -v "^$" | tail -12
[ -n "$NO_PMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp
H="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --solver ${SOLVER:-4}"
run() {  # name counters args...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$n" -o run \
    -- python3 "$@" > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
}
run fetch FETCH_SIZE $H
run write WRITE_SIZE $H
run l2 "TCC_HIT_sum TCC_MISS_sum" $H
python3 "$R/tools/pmc_kernels.py" "$OUT" || exit 1
