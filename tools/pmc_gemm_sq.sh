#!/bin/bash
# SQ counters of the trunk GEMMs (tools/gemm_mb_probe.py, REPS=2): where a wave's cycles go in the
# main loop (PHC_GEMM_DISCARD=1, which only the measurement library libphc_hip_measure.so reads:
# tools/build_variants.sh measure "-DPHC_MEASURE_GEMM=1") and with the epilogue (LIB, default the product library).  One pass per counter set, each under its
# own kill timeout; then tools/sq_summary.py prints per-GEMM ratios.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=${SQOUT:-$ROOT/gpurun_out}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for mode in main full; do
  D="PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/${LIB:-libphc_hip.so}"
  [ $mode = main ] && D="PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/${MAINLIB:-libphc_hip_measure.so} PHC_GEMM_DISCARD=1"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    env $D REPS=2 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_twin_gemm" -d "$OUT/sq_${mode}_$i" -o run \
      --output-format csv -- python3 tools/gemm_mb_probe.py > "$OUT/sq_${mode}_$i.log" 2>&1 || { tail -5 "$OUT/sq_${mode}_$i.log"; exit 5; }
  done
done
python3 tools/sq_summary.py "$OUT"
