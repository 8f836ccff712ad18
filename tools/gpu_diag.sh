#!/bin/bash
# Sweep diagnostics: DCC_SW_DEBUG clock stamps of two headline epochs and the
# kernel timeline of one epoch (rocprofv3 kernel trace).  Output to stdout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/diag"
cd "$R"
DCC_SW_DEBUG=1 timeout -k 10 120 python tools/sw_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/diag/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary \
   > "$R/gpurun_out/diag/tr.log" 2>&1 || { tail -5 "$R/gpurun_out/diag/tr.log"; exit 1; }
f=$(find "$R/gpurun_out/diag/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f"
