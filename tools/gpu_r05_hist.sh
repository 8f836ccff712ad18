#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; mkdir -p $R/gpurun_out/hist
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_history.py tests/test_gpu_occ_finish.py tests/test_gpu_snapshot.py tests/test_gpu_pipeline.py > gpurun_out/hist/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/hist/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-0 1}; do for S in ${SLOTS:-2 4}; do
  DCC_HIST_SLOTS=$S DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hist/p$v$S -o p -- python3 $R/tools/hist_ab.py $v > $R/gpurun_out/hist/p$v$S.log 2>&1 || exit 1
  echo "slots $S"; grep -h "DCC_HIST_VAR" $R/gpurun_out/hist/p$v$S.log; head -12 $R/gpurun_out/hist/p$v$S/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-90
done; done
