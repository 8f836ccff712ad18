#!/bin/bash
# Timing variants of the Calvin bucket kernels (DCC_CB_VARIANT; results are
# wrong by design, parity is not checked): per variant the C4 kernel times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/cbvar"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-0 1 2 4 6 7 8 16 24}; do
  DCC_CB_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/v$v" -o run \
    -- python3 "$R/tools/c4_only.py" > "$O/v$v.log" 2>&1 || { echo "variant $v failed"; tail -5 "$O/v$v.log"; exit 1; }
  echo "== variant $v"; python3 "$R/tools/kstats.py" "$O/v$v" 6 | grep k_cb_
done
