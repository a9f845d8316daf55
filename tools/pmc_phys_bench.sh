#!/bin/bash
# VALU / LDS instruction counts of k_physics_step over the articulated env bench's own launches
# (contact and self-collision state as the bench runs it) -> profiles/physics_valu_4096_bench.json when
# OUT=profiles (bench.py --physics articulated prefers this file for its VALU-issue roofline), then the
# env-only and PPO articulated bench lines.  Run from the repo root on the box: TAG=r06v bash tools/pmc_phys_bench.sh
set -eu
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-physb}; mkdir -p "$O"; export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "k_physics_step" \
  -d "$O/pmc" -o run --output-format csv -- python3 "$ROOT/bench.py" --mode env --physics articulated --steps 20 --warmup 5 \
  --no-cpu-baseline > "$O/pmc.log" 2>&1
python3 "$ROOT/tools/physics_valu_summary.py" "$O/pmc" 4096 "$O/physics_valu_4096_bench.json"
timeout -k 10 300 python3 bench.py --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_articulated.log" 2>&1
timeout -k 10 600 python3 bench.py --physics articulated --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_ppo_articulated.log" 2>&1
tail -n 1 "$O/bench_env_articulated.log" | cut -c1-200
