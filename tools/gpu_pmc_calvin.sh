#!/bin/bash
# HBM traffic of the Calvin C4 epoch's kernels (write amplification of the
# random group stores): rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate
# passes, kernel trace only, each under its own kill timeout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc_cv"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$R/bench.py" --only C4 --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" k_cv_ k_rs_ > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
