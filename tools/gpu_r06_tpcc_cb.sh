#!/bin/bash
set -o pipefail
O=gpurun_out/tpcc_cb
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_calvin_bucket.py tests/test_gpu_calvin.py > $O/t.txt 2>&1 || exit 1
timeout -k 10 150 python -u tools/calvin_tpcc_probe.py > $O/probe.txt 2>&1 || exit 1
