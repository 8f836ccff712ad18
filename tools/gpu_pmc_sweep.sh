#!/bin/bash
# PMC passes over two sweep epochs (tools/sw_debug.py): instruction mix, LDS
# bank conflicts, waits and HBM bytes per dispatch of the sweep kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmcs"
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$R/tools/sw_debug.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
for k in k_sw_pre k_sw_seq k_sw_filter; do
  python3 "$R/tools/pmc_dispatch.py" "$OUT" $k 8 > "$OUT/$k.txt" 2>&1
  cat "$OUT/$k.txt"
done
