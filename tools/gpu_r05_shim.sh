#!/bin/bash
# Round 5: history tests + SHIM legs and a kernel trace of the SHIM config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5s}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_history.py tests/test_gpu_occ_finish.py tests/test_gpu_compact.py tests/test_gpu_ro_split.py tests/test_gpu_golden.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 300 python bench.py --only SHIM,HIST --steps 10 > "$O/cfg.json" 2> "$O/cfg.err" || { tail -20 "$O/cfg.err"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python3 bench.py --only SHIM --steps 3 > "$O/trace.log" 2>&1 || { tail -20 "$O/trace.log"; exit 1; }
