#!/bin/bash
# k_cb_part with sub-tile element prefetch: Calvin GPU tests, C4 bench and trace.
set -o pipefail
R=$PWD
O=$R/gpurun_out/cbpart
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_calvin.py tests/test_gpu_calvin_bucket.py > $O/t.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --only C4,C4_SHUF --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
