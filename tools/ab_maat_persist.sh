#!/bin/bash
# MAAT_1M device time with / without the persistent round batches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/mtper"
mkdir -p "$O"
cd "$R"
for p in 1 0; do
  EPOCHS=7 DCC_MT_PERSIST=$p timeout -k 10 120 python3 tools/maat_rounds.py > "$O/p$p.log" 2>&1 || { tail -5 "$O/p$p.log"; exit 1; }
  echo "persist $p: $(grep median $O/p$p.log)"
done
