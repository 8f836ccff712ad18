#!/bin/bash
# Round 5: the headline bench line (no secondaries) and a kernel trace of the
# pipelined headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5d}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_occ_finish.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 100 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print(j['ms_per_step'], j['value'], j['roofline']['frac'], j['single_epoch'], j['pipeline'])"
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 K=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python3 tools/pipe_ab.py 3:0 > "$O/trace.log" 2>&1 || { tail -20 "$O/trace.log"; exit 1; }
