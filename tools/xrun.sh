#!/bin/bash
# GPU: stage-solver per-stage debug timeline (DCC_ST_DEBUG) on the headline epoch.
set -o pipefail
mkdir -p gpurun_out/dbg
for X in ${XS:-0}; do
  DCC_ST_X=$X DCC_ST_DEBUG=1 timeout -k 10 100 python -u tools/stage_check.py --quick --time 1 > gpurun_out/dbg/x_$X.log 2>&1 || { echo "fail X=$X"; tail -20 gpurun_out/dbg/x_$X.log; exit 1; }
  echo "== X=$X"; grep -E "^stage|^headline" gpurun_out/dbg/x_$X.log | tail -12 | cut -c1-400
done
