#!/bin/bash
# Round session: the whole GPU suite, smoke, the driver's bench command, and
# rocprofv3 kernel stats + one epoch's timeline of the headline.  Every GPU
# step has its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-round}"
mkdir -p "$O"
cd "$R"
if [ -z "$NOSUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$O/gpu_suite.log" 2>&1 || { tail -30 "$O/gpu_suite.log"; exit 1; }
tail -1 "$O/gpu_suite.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -3 "$O/smoke.log"
fi
T0=$(date +%s.%N); timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
echo "bench wall s: $(python3 -c "print(round($(date +%s.%N) - $T0, 1))")"
python3 -c "
import json;j=json.load(open('$O/bench.json'));e=j['epoch'];r=j['roofline']
print('value',round(j['value']/1e9,3),'G txns/s  ms',round(j['ms_per_step'],4),'dev',round(e['device_ms'],4),'frac',round(r['frac'],3),'traffic',r['traffic'],'l2',r['l2_hit'])
print('cpu',{k:round(v['txns_per_s']) for k,v in j['cpu_baseline']['variants'].items()}, j['cpu_baseline']['host']['threads_used'])
for k,v in j['other_configs'].items(): print(k,round(v.get('device_ms',v.get('device_ms_per_epoch',0)),4),v['parity_vs_oracle'],(v.get('cpu_baseline') or {}).get('txns_per_s'))
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
   -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > "$O/prof.log" 2>&1 || exit 1
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$f" 3 > "$O/trace.txt"
tail -3 "$O/trace.txt"
