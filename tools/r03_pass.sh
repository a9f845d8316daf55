#!/bin/bash
# Round-3 pass: full GPU suite + smoke, PPO and env bench lines with rocprofv3 kernel stats, and a
# 20-iteration PPO bench line (the driver's step count).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out; mkdir -p "$O"
TESTS=1 PROFILE=1 MODES="ppo env" bash tools/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > "$O/bench_ppo_4096_s20.log" 2>&1 || { tail -20 "$O/bench_ppo_4096_s20.log"; exit 7; }
tail -1 "$O/bench_ppo_4096_s20.log" | cut -c1-200
