#!/bin/bash
# Round-end check: the whole -m gpu suite, smoke(), then the default bench
# line exactly as the driver runs it (no profiler).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-final4}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
tail -3 "$O/suite.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
tail -c 400 "$O/bench.json"
