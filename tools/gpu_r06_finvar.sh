#!/bin/bash
# k_fin phase variants on the SHIM epoch (experiments build, DCC_FIN_VAR: 1 no
# chain pushes, 2 no look-back wait, 4 no write-set emission, 8 no tn stores;
# wrong results by design), kernel trace each.
set -o pipefail
R=$PWD
O=$R/gpurun_out/finvar
mkdir -p $O
export DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 4 8 15; do
  DCC_FIN_VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $O/v$v -o run -- python3 $R/bench.py --only SHIM --no-cpu-baseline > $O/v$v.json 2> $O/v$v.err || exit 1
done
