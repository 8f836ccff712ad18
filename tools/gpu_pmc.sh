#!/bin/bash
# PMC passes over a short bench run: one counter group per rocprofv3 pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), kernel trace only, each
# pass under its own kill timeout; then a per-kernel summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_EXTRA}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1
echo "pmc done"
