#!/bin/bash
# Pipelined headline (4 lanes) under other level schedules (DCC_SW_PMAX,
# experiments build): CU-time, not latency, bounds the pipelined epoch.
set -o pipefail
mkdir -p gpurun_out/sched
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
for s in "1024,3072,8192" "2048,8192,16384" "4096,16384" "2048,4096,16384" "1024,8192,16384" "512,2048,8192"; do
  tag=$(echo $s | tr ',' '_')
  DCC_SW_PMAX=$s timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --pipeline 4 \
    --no-secondary --no-cpu-baseline > gpurun_out/sched/b_$tag.json 2> gpurun_out/sched/b_$tag.err || exit 1
done
