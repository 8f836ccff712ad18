#!/bin/bash
# Chained central_finish: the GPU suite, then the PIPE_FIN and SHIM_PIPE bench legs.
set -o pipefail
O=gpurun_out/chain
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --only PIPE_FIN,SHIM_PIPE --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
