#!/bin/bash
# OCC iteration loop: OCC parity tests, headline bench (no secondaries / CPU
# baseline), rocprofv3 kernel trace of the headline and one epoch's timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-occ}
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_occ.py tests/test_gpu_sweep.py tests/test_gpu_golden.py tests/test_gpu_ro_split.py tests/test_gpu_kat_branches.py} \
   tests/test_gpu_history.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1 \
 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-secondary --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('value',d['value'],'dev_ms',d['epoch']['device_ms'],'frac',d['roofline']['frac'],'filter',d['roofline']['streaming_kernel'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o run \
   -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-secondary > "$O/tr.log" 2>&1 || { tail -5 "$O/tr.log"; exit 1; }
f=$(find "$O/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" 3
