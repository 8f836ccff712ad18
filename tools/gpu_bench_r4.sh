#!/bin/bash
# The default bench line under a kernel trace (every config), then the
# headline epoch trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-bench4}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 -u "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -c 600 "$O/bench.json"
t=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$t" 2 > "$O/trace.txt" && tail -22 "$O/trace.txt"
