# SQ / occupancy counters of the fused env kernel (k_env_step) at the bench's sizes, one pass per counter set.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/env_sq; mkdir -p "$O"; export TMPDIR=/tmp
for envs in ${ENVS_LIST:-4096 32768}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_env_step" -d "$O/sq${i}_$envs" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --mode env --steps 20 --warmup 5 --envs $envs --no-cpu-baseline > "$O/sq${i}_$envs.log" 2>&1 || { tail -5 "$O/sq${i}_$envs.log"; exit 5; }
  done
done
echo env_sq done
