#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5x}
mkdir -p "$O"
for L in 4 3 5 4; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 100 --pipeline $L > "$O/bench_L$L.json" 2> "$O/bench_L$L.err" || { tail -20 "$O/bench_L$L.err"; exit 1; }
  python3 -c "import json; j=json.load(open('$O/bench_L$L.json')); print('L$L', round(j['ms_per_step'],4), round(j['roofline']['frac'],3), j['pipeline']['host_us_per_epoch'])"
done
