#!/bin/bash
# Level-schedule experiment: DCC_SW_PMAX variants of the headline epoch with
# the sweep's clock stamps (DCC_SW_DEBUG) and without (device ms).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/pmax"; mkdir -p "$O"; cd "$R"
for s in ${SCHEDS:-"1024,2048,4096,8192" "2048,4096,8192" "1024,4096,8192" "1024,8192" "512,2048,8192" "2048,8192"}; do
  echo "== $s"
  DCC_SW_PMAX=$s DCC_SW_DEBUG=1 timeout -k 10 120 python tools/sw_debug.py > "$O/dbg_$s.log" 2>&1 || { tail "$O/dbg_$s.log"; exit 1; }
  grep "seq:" "$O/dbg_$s.log" | tail -8 | cut -c1-90
  DCC_SW_PMAX=$s timeout -k 10 120 python tools/sw_debug.py 2>&1 | tail -1 || exit 1
done
