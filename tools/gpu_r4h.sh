#!/bin/bash
# Whole -m gpu suite, then C4 + MAAT_C2 + copy probe under a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-r4h}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
tail -2 "$O/suite.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 "$R/bench.py" --only C4,MAAT_C2 --steps 6 --warmup 2 > "$O/cfg.json" 2> "$O/cfg.err" || { tail -20 "$O/cfg.err"; exit 1; }
python3 -c "import json;j=json.load(open('$O/cfg.json'));[print(k,v['device_ms'],v['parity_vs_oracle']) for k,v in j.items()]"
python3 "$R/tools/kstats.py" "$O/prof" 14
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'$R')
import bench; print('copy', bench.stream_copy_both('cuda:0'))" 2>&1 | tail -1
