#!/bin/bash
# round-4 pass p: the full PPO iteration with the articulated physics and with AMP + bf16 on the final tree
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04p; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --physics articulated --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_ppo_articulated.log" 2>&1 || { tail -5 "$O/bench_ppo_articulated.log"; exit 3; }
tail -1 "$O/bench_ppo_articulated.log" | cut -c1-200
timeout -k 10 400 python bench.py --amp --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_ppo_amp_bf16.log" 2>&1 || { tail -5 "$O/bench_ppo_amp_bf16.log"; exit 4; }
tail -1 "$O/bench_ppo_amp_bf16.log" | cut -c1-200
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -5 "$O/smoke.log"; exit 5; }
tail -2 "$O/smoke.log"
