#!/bin/bash
# Round-4 checks: compact transfer forms, the advisor's multi-GPU / deferred
# finish fixes, the Calvin shim capture; the SHIM bench leg; the two-context
# concurrency probe.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r4a"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_occ_finish.py tests/test_gpu_multi.py \
  tests/test_host_shim.py tests/test_gpu_occ.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/r4a/tests.log 2>&1 || { tail -30 gpurun_out/r4a/tests.log; exit 1; }
tail -2 gpurun_out/r4a/tests.log
timeout -k 10 300 python -u bench.py --only SHIM --steps 4 --warmup 1 > gpurun_out/r4a/shim.json 2> gpurun_out/r4a/shim.err \
  || { tail -20 gpurun_out/r4a/shim.err; exit 1; }
tail -c 1500 gpurun_out/r4a/shim.json
timeout -k 10 300 python -u tools/pipe_probe.py 40 > gpurun_out/r4a/pipe.log 2>&1 || { tail -20 gpurun_out/r4a/pipe.log; exit 1; }
cat gpurun_out/r4a/pipe.log
