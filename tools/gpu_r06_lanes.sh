#!/bin/bash
# Pipelined headline: lanes x partition (DCC_OPT_PIPE_PARTITION), one box.
set -o pipefail
mkdir -p gpurun_out/lanes2
for cfg in "4 0" "4 1" "8 1" "2 1" "8 0"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 --pipeline $1 --partition $2 \
    --no-secondary --no-cpu-baseline > gpurun_out/lanes2/bench_L$1_P$2.json 2> gpurun_out/lanes2/bench_L$1_P$2.err || exit 1
done
