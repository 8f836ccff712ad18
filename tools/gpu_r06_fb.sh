#!/bin/bash
# PIPE_FIN: k_fin 1,024-thread workgroups x 2 txns (default) against 512 x 4,
# four interleaved repetitions each.
set -o pipefail
O=gpurun_out/fb
mkdir -p $O
for rep in 1 2 3 4; do
  for v in dcc fb512; do
    lib=$PWD/deneva_amd/libdcc_$v.so
    [ $v = dcc ] && lib=$PWD/deneva_amd/libdcc.so
    DENEVA_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --only PIPE_FIN --no-cpu-baseline > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 1
    python -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));v=d.get('other_configs',d)['PIPE_FIN'];print('$v $rep',round(v['ms_per_epoch'],4))"
  done
done
