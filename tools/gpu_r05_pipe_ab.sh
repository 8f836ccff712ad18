#!/bin/bash
# Round 5: pipeline lane / CU-reserve A/B at several hardware-queue counts,
# then a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5c}
mkdir -p "$O"
for Q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 tools/pipe_ab.py 2:0 3:0 3:4 4:0 4:4 4:8 > "$O/ab_q$Q.log" 2>&1 || { tail -20 "$O/ab_q$Q.log"; exit 1; }
  echo "== GPU_MAX_HW_QUEUES=$Q"; grep lanes "$O/ab_q$Q.log"
done
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 K=16 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o trace -- python3 tools/pipe_ab.py 4:4 > "$O/trace.log" 2>&1 || { tail -20 "$O/trace.log"; exit 1; }
