#!/bin/bash
# SQ counters for k_env_step (VALU vs memory wait diagnosis), one pass.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
ENVS=${ENVS:-32768}
K=${KERNEL:-k_env_step}
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --kernel-include-regex "$K" -T -d "$OUT/prof_sq_$ENVS" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --mode env --steps 10 --warmup 3 --envs "$ENVS" --no-cpu-baseline > "$OUT/prof_sq_$ENVS.log" 2>&1 || { tail -20 "$OUT/prof_sq_$ENVS.log"; exit 5; }
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES \
  --kernel-include-regex "$K" -T -d "$OUT/prof_sq2_$ENVS" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --mode env --steps 10 --warmup 3 --envs "$ENVS" --no-cpu-baseline > "$OUT/prof_sq2_$ENVS.log" 2>&1 || { tail -20 "$OUT/prof_sq2_$ENVS.log"; exit 5; }
echo done
