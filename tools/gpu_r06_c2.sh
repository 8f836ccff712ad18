#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c2
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
timeout -k 10 120 python -u tools/c2_probe.py > gpurun_out/c2/default.txt 2>&1 || exit 1
for cfg in "1024,8192 2" "1024,16384 2" "2048,8192 2" "1024,4096,16384 3" "1024,3072,8192 4"; do
  set -- $cfg
  DCC_SW_PMAX=$1 timeout -k 10 120 python -u tools/c2_probe.py $2 > gpurun_out/c2/$1_$2.txt 2>&1 || exit 1
done
