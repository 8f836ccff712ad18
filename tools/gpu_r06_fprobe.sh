#!/bin/bash
set -o pipefail
O=gpurun_out/fprobe
mkdir -p $O
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so DCC_SW_DEBUG=1
timeout -k 10 120 python -u tools/filter_probe.py 65536 > $O/c2.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/filter_probe.py > $O/h.txt 2>&1 || exit 1
