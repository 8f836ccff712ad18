#!/bin/bash
# Round-end GPU session: the whole GPU suite, smoke, the default bench line
# (every config + CPU baselines), rocprofv3 kernel stats and trace of the
# headline.  Every GPU step has its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/final"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$O/gpu_suite.log" 2>&1 || { tail -30 "$O/gpu_suite.log"; exit 1; }
tail -1 "$O/gpu_suite.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -3 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -c 600 "$O/bench.json"; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
   -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > "$O/prof.log" 2>&1 || exit 1
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" 3 > "$O/trace.txt"
tail -3 "$O/trace.txt"
