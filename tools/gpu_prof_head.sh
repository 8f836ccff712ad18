#!/bin/bash
# rocprofv3 kernel stats + one epoch's timeline of the headline bench:
#   TAG=x [ARGS="--solver 3"] tools/gpu_prof_head.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-head}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 "$R/bench.py" --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-secondary $ARGS \
  > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
f=$(find "$O/prof" -name '*kernel_stats.csv' | head -1)
head -25 "$f" | cut -d, -f1-5 > "$O/stats.txt"
cat "$O/stats.txt"
t=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$t" > "$O/trace.txt" && cat "$O/trace.txt"
