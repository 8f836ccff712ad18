#!/bin/bash
# Quick loop: OCC parity tests (sweep + rounds), a headline bench line and the
# kernel timeline of one epoch.  Every GPU step has its own limit; the first
# failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/q"
cd "$R"
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_sweep.py tests/test_gpu_occ.py} -x -q \
   --timeout 120 --timeout-method thread -m gpu > gpurun_out/q/tests.log 2>&1 \
   || { tail -40 gpurun_out/q/tests.log; exit 1; }
tail -2 gpurun_out/q/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-secondary --no-cpu-baseline ${BENCH_EXTRA} \
   > gpurun_out/q/bench.log 2>&1 || { tail -20 gpurun_out/q/bench.log; exit 1; }
python3 -c "
import json
j=json.loads(open('gpurun_out/q/bench.log').read().strip().splitlines()[-1]); e=j['epoch']
print('ms/step', round(j['ms_per_step'],4), 'device', round(e['device_ms'],4), [round(x,4) for x in e['phase_ms']], 'roof', round(j['roofline']['frac'],3), 'parity', e['parity_vs_oracle'], 'levels', e['rounds'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/q/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_EXTRA} \
   > "$R/gpurun_out/q/tr.log" 2>&1 || { tail -5 "$R/gpurun_out/q/tr.log"; exit 1; }
f=$(find "$R/gpurun_out/q/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f"
