#!/bin/bash
# Calvin / sort check: the suites that sort (Calvin, golden, index dispatch,
# history levels, MaaT), then C4 bench + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-cv}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_calvin.py tests/test_gpu_golden.py tests/test_gpu_index.py tests/test_gpu_history.py tests/test_gpu_maat.py tests/test_gpu_kat_branches.py -x -q --timeout 120 --timeout-method thread \
  > "$O/suite.log" 2>&1 || { tail -30 "$O/suite.log"; exit 1; }
tail -1 "$O/suite.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 "$R/bench.py" --only C4 --steps 6 --warmup 2 > "$O/c4.json" 2> "$O/c4.err" || { tail -20 "$O/c4.err"; exit 1; }
python3 -c "import json;j=json.load(open('$O/c4.json'))['C4'];print('C4 dev',j['device_ms'],'wall',j['ms_per_epoch'],'parity',j['parity_vs_oracle'],'cpu',j.get('cpu_baseline',{}).get('txns_per_s'))"
f=$(find "$O/prof" -name '*kernel_stats.csv' | head -1)
head -20 "$f" | cut -d, -f1-4 | sed 's/(.*)"/"/'
python3 "$R/tools/kstats.py" "$O/prof" 20
t=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$t" > "$O/trace.txt" && cat "$O/trace.txt"
