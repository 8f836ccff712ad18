#!/bin/bash
# k_fin timing variants on the window-check A/B epoch (experiments build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; mkdir -p $R/gpurun_out/finab
cd /tmp && export TMPDIR=/tmp
for v in 0 256 512 1024 2048 3840; do
  DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/finab/p$v -o p -- python3 $R/tools/hist_ab.py $v > $R/gpurun_out/finab/p$v.log 2>&1 || exit 1
  echo "var $v: $(grep -h 'DCC_HIST_VAR' $R/gpurun_out/finab/p$v.log)  k_fin $(grep -h 'k_fin(' $R/gpurun_out/finab/p$v/p_kernel_stats.csv | cut -d, -f4)"
done
