#!/bin/bash
# Level-0 filter at 5 workgroups per CU (1,024 exact-set slots, 96 VGPRs:
# build libdcc_f5.so) against the default 4, pipelined headline, interleaved;
# then the OCC parity tests on the variant.
set -o pipefail
O=gpurun_out/f5
mkdir -p $O
one() {  # tag lib [env]
  local tag=$1 lib=$2; shift 2
  env DENEVA_AMD_LIB=$PWD/deneva_amd/$lib "$@" timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || return 1
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['ms_per_step'],4), round(d['single_epoch']['device_ms'],4), round(d['roofline']['streaming_kernel']['avg_launch_ms']*1e3,1), flush=True)"
}
for rep in 1 2 3; do
  one base_$rep libdcc_exp.so || exit 1
  one f5_$rep libdcc_f5.so || exit 1
  one f5g_$rep libdcc_f5.so DCC_SW_FGRID=1280 || exit 1
done
DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_f5.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_occ.py tests/test_gpu_sweep.py tests/test_gpu_ro_split.py > $O/t.txt 2>&1 || exit 1
