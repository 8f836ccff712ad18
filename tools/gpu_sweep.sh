#!/bin/bash
# sweep-solver parity, the OCC suites, a headline bench line and a kernel-trace
# timeline of one epoch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -v --timeout 120 \
   --timeout-method thread -m gpu > gpurun_out/sweep_tests.log 2>&1 || { tail -40 gpurun_out/sweep_tests.log; exit 1; }
tail -2 gpurun_out/sweep_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_occ.py tests/test_gpu_peel.py -x -q --timeout 120 \
   --timeout-method thread -m gpu > gpurun_out/occ_tests.log 2>&1 || { tail -30 gpurun_out/occ_tests.log; exit 1; }
tail -2 gpurun_out/occ_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "
import json
j=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); e=j['epoch']
print(round(j['value']/1e9,3),'Gtxn/s', round(j['ms_per_step'],3), 'ms', [round(x,3) for x in e['phase_ms']], 'levels', e['rounds'], 'prefix', e['peel_prefix'], 'surv', e['survivors'], 'roof', round(j['roofline']['frac'],3), 'parity', e['parity_vs_oracle'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary \
   > "$R/gpurun_out/tr.log" 2>&1 || exit 1
f=$(find "$R/gpurun_out/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" > "$R/gpurun_out/timeline.txt" 2>&1
tail -45 "$R/gpurun_out/timeline.txt"
