#!/bin/bash
# Round-5 evidence in one call: the GPU suite + smoke, the default bench line,
# a kernel trace of the pipelined headline (overlap summary), its kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/${1:-r5final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print('bench', j['ms_per_step'], j['value'], j['roofline']['frac'], j['single_epoch'].get('device_ms'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 $R/tools/trace_overlap.py $O/trace/run_kernel_trace.csv > $O/overlap.txt && cat $O/overlap.txt
