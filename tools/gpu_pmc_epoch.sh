#!/bin/bash
# Whole-epoch HBM traffic of the headline OCC epoch: rocprofv3 --pmc passes
# over a short bench run (FETCH_SIZE and WRITE_SIZE in separate passes,
# kernel trace only, each pass under its own kill timeout), then
# tools/epoch_traffic.py -> profiles/r02/traffic.json (read by bench.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${TAG:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 $ARGS > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -5 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 $ARGS > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -5 "$OUT/write.log"; exit 1; }
python3 "$R/tools/epoch_traffic.py" "$OUT" "1048576:0.9:16:1" "$OUT/traffic.json" \
    "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, ${TAG:-pmc}" || exit 1
echo "pmc done"
