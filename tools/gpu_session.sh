#!/bin/bash
# One GPU session: parity suite, smoke, bench, rocprofv3 kernel stats of the
# bench, then (optional) the stage-solver check.  Every GPU step has its own
# time limit; steps are chained with && so the first failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-s}
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
 && timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err" \
 && (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 5 \
      --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_ARGS} > "$O/prof.log" 2>&1) \
 && { [ -z "$STAGE" ] || timeout -k 10 300 python -u tools/stage_check.py > "$O/stage.log" 2>&1; }
rc=$?
echo "session exit $rc"
tail -3 "$O/pytest_gpu.log"; tail -2 "$O/smoke.log"; tail -c 600 "$O/bench.json"; tail -3 "$O/stage.log" 2>/dev/null
exit $rc
