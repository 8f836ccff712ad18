#!/bin/bash
# GPU tests of the files named in $TESTS, then the bench configs named in $ONLY
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/step; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $O/tests.txt 2>&1
  rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$ONLY" ]; then
  timeout -k 10 600 python bench.py --only $ONLY --no-cpu-baseline > $O/only.json 2> $O/only.err || { tail -20 $O/only.err; exit 1; }
  python3 - $O/only.json <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
for k, v in (j.get("other_configs") or j).items():
    print(k, {kk: v.get(kk) for kk in ("device_ms", "device_ms_per_epoch", "ms_per_epoch", "parity_vs_oracle", "rounds") if kk in v},
          v.get("device_resident", ""))
PY
fi
