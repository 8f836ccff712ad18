#!/bin/bash
# Round-6 final evidence: the GPU suite, the default bench line, and a
# kernel-trace profile of the headline bench command.
set -o pipefail
R=$PWD
O=$R/gpurun_out/fin6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
