#!/bin/bash
# Stage-solver loop: parity check on every shape, headline timing, and the
# kernel timeline of one headline epoch (rocprofv3 kernel trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-st}
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u tools/stage_check.py ${CHECK_ARGS} > "$O/check.log" 2>&1 || { tail -30 "$O/check.log"; exit 1; }
cat "$O/check.log" | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary \
   > "$O/tr.log" 2>&1 || { tail -5 "$O/tr.log"; exit 1; }
f=$(find "$O/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f"
