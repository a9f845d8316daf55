#!/bin/bash
# GPU suite + the driver's bench command three times.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out; mkdir -p "$O"
TESTS=1 PROFILE=0 MODES="" bash tools/gpu_check.sh || exit $?
grep -q " passed" "$O/pytest_gpu.log" && ! grep -q "failed" "$O/pytest_gpu.log" || { echo "GPU tests not green"; exit 6; }
bash tools/r03_bench3.sh
