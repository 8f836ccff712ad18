#!/bin/bash
# The whole -m gpu suite in one process (own limit), then smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-suite}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
tail -3 "$O/suite.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
