#!/bin/bash
# r03 profiling pass: env + ppo bench lines, rocprofv3 kernel stats of the PPO iteration and the env step
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=$ROOT/gpurun_out/${TAG:-r03}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --mode env --no-cpu-baseline > "$O/bench_env_4096.log" 2>&1 || exit 4
tail -1 "$O/bench_env_4096.log" | cut -c1-200
timeout -k 10 600 python bench.py --steps ${PPO_STEPS:-10} --warmup 2 --no-cpu-baseline > "$O/bench_ppo_4096.log" 2>&1 || exit 5
tail -1 "$O/bench_ppo_4096.log" | cut -c1-200
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || exit 6
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_env" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --mode env --no-cpu-baseline > "$O/trace_env.log" 2>&1 || exit 7
fi
echo "r03_prof done"
