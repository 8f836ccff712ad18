#!/bin/bash
# Kernel-trace summaries of single secondary configs (C4, C2).
set -o pipefail
R=$PWD
O=$R/gpurun_out/profcfg
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-C4 C2}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$c -o run -- python3 $R/bench.py --only $c --no-cpu-baseline --steps 20 --warmup 5 > $O/$c.json 2> $O/$c.err || exit 1
done
