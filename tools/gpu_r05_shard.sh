#!/bin/bash
# Round 5: key-sharded OCC (both forms) and the multi-GPU context on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5v}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_occ_finish.py > "$O/shard_tests.log" 2>&1 || { tail -40 "$O/shard_tests.log"; exit 1; }
grep -E "PASS|FAIL" "$O/shard_tests.log" | tail -40
