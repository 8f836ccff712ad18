set -o pipefail
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-A B}; do
  cp deneva_amd/libdcc.so.exp-$v deneva_amd/libdcc.so
  timeout -k 10 200 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t_$v.log 2>&1 || { tail -20 gpurun_out/ab/t_$v.log; exit 1; }
  tail -1 gpurun_out/ab/t_$v.log
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-secondary --no-cpu-baseline > gpurun_out/ab/b_$v.json 2> gpurun_out/ab/b_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/b_$v.json').read().strip().splitlines()[-1]);print('$v','dev_ms',d['epoch']['device_ms'],'filter_ms',d['roofline']['streaming_kernel']['avg_launch_ms'])"
done
