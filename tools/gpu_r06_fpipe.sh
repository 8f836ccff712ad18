#!/bin/bash
# Pipelined filter tiles (DCC_F_PIPE: next tile's words and first key round
# loaded behind this tile's first exact probes): the OCC parity tests on the
# variant, then the headline interleaved against the default build.
set -o pipefail
O=gpurun_out/fpipe
mkdir -p $O
DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_fp4.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_occ.py tests/test_gpu_sweep.py tests/test_gpu_ro_split.py tests/test_gpu_multi.py tests/test_gpu_golden.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
one() {  # tag lib
  local tag=$1 lib=$2
  env DENEVA_AMD_LIB=$PWD/deneva_amd/$lib timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || return 1
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['ms_per_step'],4), round(d['single_epoch']['device_ms'],4), round(d['roofline']['streaming_kernel']['avg_launch_ms']*1e3,1), flush=True)"
}
for rep in 1 2 3; do
  one base_$rep libdcc_exp.so || exit 1
  one fp4_$rep libdcc_fp4.so || exit 1
  one fp1_$rep libdcc_fp1.so || exit 1
done
