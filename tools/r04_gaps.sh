#!/bin/bash
# kernel trace of the PPO bench command + the idle-gap breakdown of one iteration (tools/trace_gaps.py)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-r04_gaps}; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || { tail -5 "$O/trace_ppo.log"; exit 6; }
f=$(find "$O/trace_ppo" -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py "$f" 16 > "$O/gaps.txt"; cat "$O/gaps.txt"
timeout -k 10 300 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.log" 2>&1 && tail -1 "$O/bench.log" | cut -c1-300
