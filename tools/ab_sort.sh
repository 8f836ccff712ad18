# A/B of libdcc.so variants on the radix sort users: their GPU suites, then
# the C4 bench leg under a kernel trace (per-kernel averages per variant).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/${TAG:-abs}"
mkdir -p "$O"
for v in ${VARIANTS:-A B}; do
  cp "$R/deneva_amd/libdcc.so.exp-$v" "$R/deneva_amd/libdcc.so"
  cd "$R"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_calvin.py tests/test_gpu_golden.py tests/test_gpu_index.py tests/test_gpu_history.py tests/test_gpu_maat.py -x -q --timeout 120 --timeout-method thread > "$O/t_$v.log" 2>&1 || { tail -20 "$O/t_$v.log"; exit 1; }
  tail -1 "$O/t_$v.log"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run \
    -- python3 "$R/bench.py" --only C4 --steps 6 --warmup 2 > "$O/c4_$v.json" 2> "$O/c4_$v.err" || { tail -20 "$O/c4_$v.err"; exit 1; }
  python3 -c "import json;j=json.load(open('$O/c4_$v.json'))['C4'];print('$v C4 dev',j['device_ms'],'wall',j['ms_per_epoch'],'parity',j['parity_vs_oracle'])"
  python3 "$R/tools/kstats.py" "$O/prof_$v" 12
done
