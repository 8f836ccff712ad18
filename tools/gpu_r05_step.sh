#!/bin/bash
# GPU tests of the files named in $TESTS, then the window-check A/B epoch profiled
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/step; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hist -o p -- python3 $R/tools/hist_ab.py 0 > $O/hist.log 2>&1 || exit 1
grep -h "DCC_HIST_VAR" $O/hist.log; head -14 $O/hist/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-90
