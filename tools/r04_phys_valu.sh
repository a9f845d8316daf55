#!/bin/bash
# Recount the physics kernel's VALU instructions on the current tree: the standing probe
# (tools/profile_physics.sh) and the articulated env bench's own launches (the workload the bench
# times).  Writes under gpurun_out/phys_prof/.
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
O=$ROOT/gpurun_out/phys_prof
bash "$ROOT/tools/profile_physics.sh"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "k_physics_step" -d "$O/pmc_bench" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --mode env --physics articulated --no-cpu-baseline --steps 20 --warmup 5 > "$O/pmc_bench.log" 2>&1
python "$ROOT/tools/physics_valu_summary.py" "$O/pmc_bench" 4096 "$O/physics_valu_4096_bench.json"
timeout -k 10 300 python3 "$ROOT/bench.py" --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_articulated.log" 2>&1
tail -1 "$O/bench_env_articulated.log" | cut -c1-400
echo done
