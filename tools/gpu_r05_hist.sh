#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; mkdir -p $R/gpurun_out/hist
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-0 1 2 4}; do
  DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hist/p$v -o p -- python3 $R/tools/hist_ab.py $v > $R/gpurun_out/hist/p$v.log 2>&1 || exit 1
  grep -h "DCC_HIST_VAR" $R/gpurun_out/hist/p$v.log
done
