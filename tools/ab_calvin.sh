# A/B of libdcc.so variants on Calvin: GPU Calvin tests, then the C4 bench leg
set -o pipefail
mkdir -p gpurun_out/abc
for v in ${VARIANTS:-A B}; do
  cp deneva_amd/libdcc.so.exp-$v deneva_amd/libdcc.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_calvin.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abc/t_$v.log 2>&1 || { tail -20 gpurun_out/abc/t_$v.log; exit 1; }
  tail -1 gpurun_out/abc/t_$v.log
  timeout -k 10 200 python -u bench.py --only C4 --steps 10 --warmup 2 > gpurun_out/abc/b_$v.json 2> gpurun_out/abc/b_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abc/b_$v.json').read().strip().splitlines()[-1]);c=d['C4'];print('$v', {k:c[k] for k in c if 'ms' in k})"
done
