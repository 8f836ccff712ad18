#!/bin/bash
set -o pipefail
O=gpurun_out/fprobe
mkdir -p $O
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so DCC_SW_DEBUG=1
for fg in 256 1024; do
  DCC_SW_FGRID=$fg timeout -k 10 120 python -u tools/filter_probe.py > $O/fg_$fg.txt 2>&1 || exit 1
done
