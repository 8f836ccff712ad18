#!/bin/bash
# Level-schedule A/B of the headline epoch: DCC_SW_PMAX variants, device ms
# and wall ms/step of the bench line (no secondaries, no CPU leg).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-sched}"; mkdir -p "$O"; cd "$R"
for s in ${SCHEDS:-"1024,3072,8192" "1024,4096,8192" "1024,2048,8192" "2048,4096,8192" "768,3072,8192" "1024,3072,8192"}; do
  DCC_SW_PMAX=$s timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline \
    > "$O/b_$s.json" 2> "$O/b_$s.err" || { tail -5 "$O/b_$s.err"; exit 1; }
  python3 -c "
import json;j=json.loads(open('$O/b_$s.json').read().strip().splitlines()[-1]);e=j['epoch']
print('$s', 'device', round(e['device_ms'],4), 'wall', round(j['ms_per_step'],4), 'levels', e['rounds'], 'parity', e['parity_vs_oracle'])"
done
