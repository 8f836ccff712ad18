#!/bin/bash
# Calvin bucket path: parity (bucket tests, then the Calvin suite on the
# default path), the C4 bench under a kernel trace, then the FETCH / WRITE
# PMC passes of C4.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-r4b}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_calvin_bucket.py -x -q --timeout 120 --timeout-method thread \
  > "$O/bucket.log" 2>&1 || { tail -40 "$O/bucket.log"; exit 1; }
tail -1 "$O/bucket.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_calvin.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread \
  > "$O/calvin.log" 2>&1 || { tail -30 "$O/calvin.log"; exit 1; }
tail -1 "$O/calvin.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 "$R/bench.py" --only C4 --steps 6 --warmup 2 > "$O/c4.json" 2> "$O/c4.err" || { tail -20 "$O/c4.err"; exit 1; }
python3 -c "import json;j=json.load(open('$O/c4.json'))['C4'];print('C4 dev',j['device_ms'],'wall',j['ms_per_epoch'],'parity',j['parity_vs_oracle'])"
python3 "$R/tools/kstats.py" "$O/prof" 24
t=$(find "$O/prof" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/trace_epoch.py" "$t" > "$O/trace.txt" && tail -40 "$O/trace.txt"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$O/pmc/p$i" -o run \
      -- python3 "$R/bench.py" --only C4 --steps 2 --warmup 1 > "$O/pmc_p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$O/pmc_p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$O/pmc" k_cv_ k_rs_ k_cb_ > "$O/pmc_summary.txt" 2>&1
cat "$O/pmc_summary.txt"
