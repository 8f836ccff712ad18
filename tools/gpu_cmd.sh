#!/bin/bash
# parity tests of the OCC paths, bench lines (peel on / off), and a
# kernel-trace timeline of one epoch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_occ.py tests/test_gpu_peel.py -x -v --timeout 120 \
   --timeout-method thread -m gpu > gpurun_out/occ_tests.log 2>&1 || { tail -30 gpurun_out/occ_tests.log; exit 1; }
tail -2 gpurun_out/occ_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --peel 0 --solver 1 > gpurun_out/bench_rounds.log 2>&1 || { tail -20 gpurun_out/bench_rounds.log; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/bench.log','gpurun_out/bench_rounds.log'):
    j=json.loads(open(f).read().strip().splitlines()[-1]); e=j['epoch']
    print(f, round(j['ms_per_step'],3), 'ms', [round(x,3) for x in e['phase_ms']], e['phases'], 'roof', round(j['roofline']['frac'],3), 'parity', e['parity_vs_oracle'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_EXTRA} \
   > "$R/gpurun_out/tr.log" 2>&1 || exit 1
f=$(find "$R/gpurun_out/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" > "$R/gpurun_out/timeline.txt" 2>&1
tail -1 "$R/gpurun_out/timeline.txt"
