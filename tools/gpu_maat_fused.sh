#!/bin/bash
# MaaT fused round scan: parity tests, 1M timing fused vs unfused, kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-mtf}"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_maat.py tests/test_gpu_kat_branches.py -x -q --timeout 200 \
  --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
DCC_MT_DEBUG=1 DCC_MT_FUSED=1 timeout -k 10 120 python3 tools/maat_rounds.py > "$O/fused.log" 2>&1 || { tail -5 "$O/fused.log"; exit 1; }
DCC_MT_FUSED=0 timeout -k 10 120 python3 tools/maat_rounds.py > "$O/split.log" 2>&1 || { tail -5 "$O/split.log"; exit 1; }
grep epoch "$O/fused.log" "$O/split.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
  -- python3 "$R/tools/maat_rounds.py" > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$O/prof" 12
