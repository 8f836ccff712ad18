#!/bin/bash
# A/B of sweep schedules on the headline: each line one bench run (its own
# time limit) with DCC_SW_PMAX / sweep levels / read-only split as given.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-sched}"
mkdir -p "$O"; cd "$R"
i=0
while read -r pmax lv ro; do
  [ -z "$pmax" ] && continue
  i=$((i+1))
  DCC_SW_PMAX=$pmax timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-secondary --no-cpu-baseline \
     --sweep-levels $lv --ro-split $ro > "$O/s$i.json" 2>&1 || { tail -5 "$O/s$i.json"; exit 1; }
  python3 -c "
import json
j=json.loads(open('$O/s$i.json').read().strip().splitlines()[-1]); e=j['epoch']
print('$pmax lv $lv ro $ro: device', round(e['device_ms'],4), 'ms/step', round(j['ms_per_step'],4), 'parity', e['parity_vs_oracle'])"
done <<< "${SCHED}"
