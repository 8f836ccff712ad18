#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5o}
mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 100 --pipeline 3 > "$O/bench_$i.json" 2> "$O/bench_$i.err" || { tail -20 "$O/bench_$i.err"; exit 1; }
  python3 -c "import json; j=json.load(open('$O/bench_$i.json')); print('bench', round(j['ms_per_step'],4), j['pipeline']['host_us_per_epoch'])"
  GPU_MAX_HW_QUEUES=12 K=100 timeout -k 10 300 python3 tools/pipe_ab.py 3 > "$O/ab_$i.log" 2>&1 || { tail -20 "$O/ab_$i.log"; exit 1; }
  grep lanes "$O/ab_$i.log"
done
