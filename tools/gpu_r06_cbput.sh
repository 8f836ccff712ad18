#!/bin/bash
# k_cb_put's wait bits without same-word LDS atomics: the bucket-path tests,
# then C4 (bench --only C4) and its kernel trace.
set -o pipefail
R=$PWD; O=$R/gpurun_out/cbput; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_calvin_bucket.py tests/test_gpu_calvin.py > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --only C4 > $O/c4_$i.json 2> $O/c4_$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c4_$i.json'));c=d['C4'] if 'C4' in d else d;print(json.dumps(c)[:300])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --only C4 --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1
