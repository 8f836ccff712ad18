#!/bin/bash
# kernel trace of the window-check A/B epoch (SHIM's device-resident shape)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/histprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o p -- python3 $R/tools/hist_ab.py 0 > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
grep -h "DCC_HIST_VAR" $O/log
