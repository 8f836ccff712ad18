#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5p}
mkdir -p "$O"
export GPU_MAX_HW_QUEUES=12 K=100
for i in 1 2 3; do
  for like in none e; do
    LIKE=$like timeout -k 10 300 python3 tools/pipe_ab.py 3 > "$O/ab_${like}_$i.log" 2>&1 || { tail -20 "$O/ab_${like}_$i.log"; exit 1; }
    echo "$like $i: $(grep lanes $O/ab_${like}_$i.log)"
  done
done
