#!/bin/bash
# SQ / LDS / MFMA counters for k_twin_gemm on one twin-trunk shape (tools/twin_gemm_probe.py one).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; OUT=$ROOT/gpurun_out/pmc_gemm; mkdir -p "$OUT"; export TMPDIR=/tmp
SHAPE=${SHAPE:-L2}
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "k_twin_gemm" -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/twin_gemm_probe.py" fp16 one "$SHAPE" > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 5; }
done
echo done
