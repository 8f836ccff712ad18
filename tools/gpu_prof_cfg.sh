#!/bin/bash
# rocprofv3 kernel stats of one secondary bench config: CFG=C4 TAG=x tools/gpu_prof_cfg.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-cfg}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in ${CFG//,/ }; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$c" -o run \
    -- python3 "$R/bench.py" --only "$c" --steps ${STEPS:-5} --warmup 2 > "$O/$c.json" 2> "$O/$c.err" || exit 1
  echo "== $c"; tail -c 700 "$O/$c.json"; echo
  f=$(find "$O/$c" -name '*kernel_stats.csv' | head -1)
  head -12 "$f" | cut -d, -f1-5
done
