#!/bin/bash
# k_fin txns-per-thread A/B (FIN_T 2 / 4 / 8 builds): the pipeline and finish
# tests, then PIPE_FIN, on each.
set -o pipefail
O=gpurun_out/fint
mkdir -p $O
for v in ${VARS:-fin4 fin8 dcc}; do
  lib=$PWD/deneva_amd/libdcc_${v}.so
  [ $v = dcc ] && lib=$PWD/deneva_amd/libdcc.so
  DENEVA_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_occ_finish.py tests/test_gpu_history.py > $O/t_$v.txt 2>&1 || exit 1
  for rep in 1 2; do
    DENEVA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --only PIPE_FIN --no-cpu-baseline > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 1
  done
done
