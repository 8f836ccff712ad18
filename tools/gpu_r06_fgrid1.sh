#!/bin/bash
# The later levels' filter / compaction grid (DCC_SW_FGRID1, experiments
# build) on the pipelined headline, interleaved repetitions.
set -o pipefail
O=gpurun_out/fgrid1
mkdir -p $O
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
for rep in 1 2 3; do
  for fg in 0 128 256 512; do
    if [ $fg = 0 ]; then unset DCC_SW_FGRID1; else export DCC_SW_FGRID1=$fg; fi
    timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline > $O/fg_${fg}_$rep.json 2> $O/fg_${fg}_$rep.err || exit 1
    python -c "import json;d=json.load(open('$O/fg_${fg}_$rep.json'));print('$fg $rep', round(d['ms_per_step'],4), round(d['single_epoch']['device_ms'],4), flush=True)"
  done
done
