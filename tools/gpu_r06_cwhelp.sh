#!/bin/bash
# Calvin wave walk with helper workgroups (calvin_wave.hip HELP): the tests
# that ask for waves on the product library (32 helpers), then the C4 walk's
# time and the staging split at 0 / 16 / 32 / 64 helpers (experiments build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/cwhelp; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_golden.py tests/test_gpu_kat_branches.py tests/test_gpu_calvin.py tests/test_gpu_index.py \
  > $O/tests.txt 2>&1
rc=$?; grep -E "C4 waves|passed|failed|Error" $O/tests.txt | tail -8; [ $rc -eq 0 ] || exit $rc
for nh in ${NHS:-0 16 32 64}; do
  DENEVA_AMD_LIB=$R/deneva_amd/libdcc_exp.so DCC_CW_DBG=1 DCC_CW_HELPERS=$nh \
    timeout -k 10 120 python3 -u tools/calvin.py --waves --reps 3 > $O/nh$nh.txt 2>&1 || { tail -5 $O/nh$nh.txt; exit 1; }
  echo "nh=$nh"; grep -E "^cw:|profiling\": false" $O/nh$nh.txt | tail -2
done
