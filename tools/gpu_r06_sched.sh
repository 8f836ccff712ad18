#!/bin/bash
# Pipelined headline under other level schedules (DCC_SW_PMAX, experiments
# build) and lane counts: CU-time, not latency, bounds the pipelined epoch.
set -o pipefail
mkdir -p gpurun_out/sched2
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
for L in 4 6; do
for s in "1024,3072,8192" "2048,4096,16384" "2048,6144,16384" "1536,4096,16384"; do
  tag=L${L}_$(echo $s | tr ',' '_')
  DCC_SW_PMAX=$s timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --pipeline $L \
    --no-secondary --no-cpu-baseline > gpurun_out/sched2/b_$tag.json 2> gpurun_out/sched2/b_$tag.err || exit 1
done
done
