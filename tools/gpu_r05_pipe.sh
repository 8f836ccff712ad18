#!/bin/bash
# Round 5: pipelined epochs -- the pipeline tests, the whole GPU suite, and the
# headline at 0 / 2 / 3 / 4 lanes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5a}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py > "$O/pipe_tests.log" 2>&1 || { tail -30 "$O/pipe_tests.log"; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/gpu_suite.log" 2>&1 || { tail -30 "$O/gpu_suite.log"; exit 1; }
tail -2 "$O/gpu_suite.log"
for L in ${LANES:-0 2 3 4}; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --pipeline $L --steps 60 > "$O/bench_L$L.json" 2> "$O/bench_L$L.err" || { tail -20 "$O/bench_L$L.err"; exit 1; }
  python3 -c "import json,sys; j=json.load(open('$O/bench_L$L.json')); print('L=$L', round(j['ms_per_step'],4), 'ms/epoch', round(j['roofline']['frac'],3), 'frac', 'lat', round(j['single_epoch']['device_ms'],4), 'parity', j['epoch']['parity_vs_oracle'])"
done
