#!/bin/bash
# N3 physics step profile: rocprofv3 kernel stats of tools/physics_probe.py (4096 envs, 50 launches)
# and one PMC pass of SQ issue counters on k_physics_step.  Writes under gpurun_out/phys_prof/.
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
O=$ROOT/gpurun_out/phys_prof
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$ROOT/tools/physics_probe.py" 4096 50 > "$O/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "k_physics_step" -d "$O/pmc" -o run --output-format csv -- \
  python3 "$ROOT/tools/physics_probe.py" 4096 20 > "$O/pmc.log" 2>&1

python "$ROOT/tools/physics_valu_summary.py" "$O/pmc" 4096 "$O/physics_valu_4096.json"
echo done
