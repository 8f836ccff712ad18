#!/bin/bash
# PMC passes over the window-check A/B epoch (tools/hist_ab.py 0): k_hist rows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/histpmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local n=$1 c=$2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$n" -o run \
    -- python3 "$R/tools/hist_ab.py" 0 > "$OUT/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "pass $n ok"
}
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
run sq2 "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
run l2 "TCC_HIT_sum TCC_MISS_sum"
run fetch FETCH_SIZE
