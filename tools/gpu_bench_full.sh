#!/bin/bash
# Default bench line (all configs, CPU baseline) + rocprofv3 kernel stats of
# the headline run; outputs under gpurun_out/full/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/full"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -1 "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
   -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > "$O/prof.log" 2>&1 || exit 1
f=$(find "$O/prof" -name '*kernel_stats.csv' | head -1)
head -20 "$f"
