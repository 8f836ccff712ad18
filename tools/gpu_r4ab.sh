#!/bin/bash
# r4b (Calvin bucket path: parity, C4 trace + PMC) then r4a (compact forms,
# advisor fixes, SHIM leg, two-context probe).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_r4b.sh || exit 1
cd "$R"
bash tools/gpu_r4a.sh
