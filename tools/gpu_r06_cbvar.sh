#!/bin/bash
# k_cb_part / k_cb_bucket timing variants (experiments build, DCC_CB_VARIANT:
# 1 no partition stores, 2 no ranking, 4 no element loads; 8/16/32/64 the
# bucket pass's phases) on C4, kernel trace each.
set -o pipefail
R=$PWD
O=$R/gpurun_out/cbvar
mkdir -p $O
export DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 4 8 16 32 64; do
  DCC_CB_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/v$v -o run -- python3 $R/bench.py --only C4 --no-cpu-baseline > $O/v$v.json 2> $O/v$v.err || exit 1
done
