#!/bin/bash
# Level-0 filter grid A/B (experiments build, DCC_SW_FGRID): pipelined and
# single-epoch headline per grid.
set -o pipefail
O=gpurun_out/fgrid
mkdir -p $O
export DENEVA_AMD_LIB=$PWD/deneva_amd/libdcc_exp.so
for fg in 1024 512 768 1536 1024; do
  DCC_SW_FGRID=$fg timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 > $O/fg_$fg.json 2> $O/fg_$fg.err || exit 1
  python - $O/fg_$fg.json $fg <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "pipelined", round(d["ms_per_step"], 4), "single", round(d["single_epoch"]["device_ms"], 4),
      "filter", round(d["roofline"]["streaming_kernel"]["avg_launch_ms"], 4), flush=True)
PY
done
unset DENEVA_AMD_LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_occ.py tests/test_gpu_sweep.py tests/test_gpu_ro_split.py > $O/tests.txt 2>&1 || exit 1
