#!/bin/bash
# SQ counters of the C4 epoch's kernels (bucket path): instruction mix, LDS
# waits and bank conflicts, wave cycles -- one pass per counter set, kernel
# trace only, each under its own kill timeout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${TAG:-sq_c4}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
C="$R/bench.py --only C4 --steps 2 --warmup 1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$R/bench.py" --only C4 --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 "$R/tools/pmc_summary.py" "$OUT" k_cb_ > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
