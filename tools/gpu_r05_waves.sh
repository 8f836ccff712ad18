#!/bin/bash
# Calvin wave levels: the GPU tests that ask for waves, then a kernel trace of
# the C4 epoch with waves
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/waves; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_golden.py tests/test_gpu_kat_branches.py tests/test_gpu_calvin.py tests/test_gpu_index.py \
  > $O/tests.txt 2>&1
rc=$?; grep -E "C4 waves|passed|failed|Error" $O/tests.txt | tail -8; [ $rc -eq 0 ] || exit $rc
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $R/tools/calvin.py --waves --reps 2 > $O/calvin.txt 2>&1
rc=$?; grep profiling $O/calvin.txt; [ $rc -eq 0 ] || { tail -5 $O/calvin.txt; exit $rc; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
