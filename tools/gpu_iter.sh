#!/bin/bash
# Iteration session: a test subset, the headline bench line, optional
# secondary configs, and kernel stats / one epoch's timeline of each.  Every
# GPU step has its own limit; the first failure ends the session.
#   TESTS="tests/a.py tests/b.py"  ONLY="C4,MAAT_1M"  TAG=name  BENCH_EXTRA="..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-it}"
rm -rf "$O"; mkdir -p "$O"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -m gpu \
     > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
  tail -2 "$O/tests.log"
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-secondary --no-cpu-baseline ${BENCH_EXTRA} \
   > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
python3 -c "
import json
j=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); e=j['epoch']
print('headline ms/step', round(j['ms_per_step'],4), 'device', round(e['device_ms'],4), 'roof', round(j['roofline']['frac'],3), 'parity', e['parity_vs_oracle'], 'levels', e['rounds'], 'filter', round(j['roofline']['streaming_kernel']['avg_launch_ms']*1e3,1))
"
if [ -n "$ONLY" ]; then
  timeout -k 10 400 python bench.py --only "$ONLY" --steps 10 --warmup 3 > "$O/only.json" 2> "$O/only.err" \
     || { tail -20 "$O/only.err"; exit 1; }
  python3 -c "
import json
j=json.loads(open('$O/only.json').read().strip().splitlines()[-1])
for k,v in j.items(): print(k, 'device', round(v.get('device_ms', v.get('device_ms_per_epoch', 0)),4), 'parity', v['parity_vs_oracle'], {x: v[x] for x in ('rounds','commits') if x in v})
"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr" -o run \
   -- python3 "$R/bench.py" --steps 6 --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_EXTRA} \
   > "$O/tr.log" 2>&1 || { tail -5 "$O/tr.log"; exit 1; }
f=$(find "$O/tr" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" 2 > "$O/trace.txt"
cat "$O/trace.txt"
if [ -n "$ONLY" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ot" -o run \
     -- python3 "$R/bench.py" --only "$ONLY" --steps 4 --warmup 1 > "$O/ot.log" 2>&1 \
     || { tail -5 "$O/ot.log"; exit 1; }
  f=$(find "$O/ot" -name '*kernel_stats.csv' | head -1)
  python3 "$R/tools/kstats.py" "$f" | head -25
fi
