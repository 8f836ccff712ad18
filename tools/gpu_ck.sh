#!/bin/bash
# Commit/kill solver check: its parity suite, the OCC suites, the headline
# bench line (no CPU legs) and the OCC secondary configs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/ck"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ck.py -x -v --timeout 120 --timeout-method thread \
  > "$O/ck_suite.log" 2>&1 || { tail -40 "$O/ck_suite.log"; exit 1; }
tail -2 "$O/ck_suite.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_occ.py tests/test_gpu_sweep.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread \
  > "$O/occ_suite.log" 2>&1 || { tail -40 "$O/occ_suite.log"; exit 1; }
tail -2 "$O/occ_suite.log"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json;j=json.load(open('$O/bench.json'));e=j['epoch'];print('value',j['value'],'ms',j['ms_per_step'],'dev',e['device_ms'],'rounds',e['rounds'],'parity',e['parity_vs_oracle'],'frac',j['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --only C2,C3,C5 --steps 10 --warmup 3 > "$O/sec.json" 2> "$O/sec.err" || { tail -20 "$O/sec.err"; exit 1; }
cat "$O/sec.json"
