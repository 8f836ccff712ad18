#!/bin/bash
# C2: the mode-2 serial tail at 8,192 (default) against 4,096 (DCC_SW_PMAX,
# experiments build), twice each.
set -o pipefail
O=gpurun_out/c2b
mkdir -p $O
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
for rep in 1 2; do
  C2_ONLY=C2 timeout -k 10 120 python -u tools/c2_probe.py > $O/def_$rep.txt 2>&1 || exit 1
  DCC_SW_PMAX=1024,4096 C2_ONLY=C2 timeout -k 10 120 python -u tools/c2_probe.py 2 > $O/p4096_$rep.txt 2>&1 || exit 1
  DCC_SW_PMAX=1024,4096 DCC_SW_GBITS=16 C2_ONLY=C2 timeout -k 10 120 python -u tools/c2_probe.py 2 > $O/p4096g_$rep.txt 2>&1 || exit 1
done
grep -h "C2 " $O/*.txt
