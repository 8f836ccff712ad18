#!/bin/bash
# MAAT_1M device time per DCC_MT_PREFIX (prefix-level txns; 0 = none).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/mtpre"
mkdir -p "$O"
cd "$R"
for p in ${PREFIXES:-256 512 1024 2048 0}; do
  DCC_MT_DEBUG=1 EPOCHS=7 DCC_MT_PREFIX=$p timeout -k 10 120 python3 tools/maat_rounds.py > "$O/p$p.log" 2>&1 || { tail -5 "$O/p$p.log"; exit 1; }
  echo "prefix $p: $(grep median $O/p$p.log) $(grep -m1 'maat prefix' $O/p$p.log)"
done
