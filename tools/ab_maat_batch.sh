#!/bin/bash
# MAAT_1M device time per DCC_MT_BATCH (rounds per host check).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/mtb"
mkdir -p "$O"
cd "$R"
for b in ${BATCHES:-8 10 12 16}; do
  EPOCHS=7 DCC_MT_BATCH=$b timeout -k 10 120 python3 tools/maat_rounds.py > "$O/b$b.log" 2>&1 || { tail -5 "$O/b$b.log"; exit 1; }
  echo "batch $b: $(grep median $O/b$b.log)"
done
