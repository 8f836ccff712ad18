#!/bin/bash
# Small-kernel grid A/B on the pipelined headline: the read-only check's grid
# (DCC_SW_ROGRID) and the level-0 validation pass's workgroups (builds with
# DCC_SW_PREP_BLOCKS 256 / 512 vs 1024), each twice, interleaved.
set -o pipefail
O=gpurun_out/grids
mkdir -p $O
one() {  # tag lib [env...]
  local tag=$1 lib=$2; shift 2
  env DENEVA_AMD_LIB=$PWD/deneva_amd/$lib "$@" timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || return 1
  python - $O/$tag.json $tag <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "pipelined", round(d["ms_per_step"], 4), "single", round(d["single_epoch"]["device_ms"], 4), flush=True)
PY
}
for rep in 1 2; do
  one base_$rep libdcc_exp.so || exit 1
  one ro256_$rep libdcc_exp.so DCC_SW_ROGRID=256 || exit 1
  one pb256_$rep libdcc_pb256.so || exit 1
  one pb512_$rep libdcc_pb512.so || exit 1
  one both_$rep libdcc_pb256.so DCC_SW_ROGRID=256 || exit 1
done
