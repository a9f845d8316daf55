#!/bin/bash
# main loop only (DISCARD=1) and epilogue without global stores (DISCARD=2): LDS-image vs register-direct forward epilogue
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/discard; mkdir -p "$O"
for D in 1 2; do
  for so in libphc_hip_lds.so libphc_hip_fwd.so; do
    PHC_GEMM_DISCARD=$D PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/gemm_mb_probe.py > "$O/${so}_$D.log" 2>&1 || { tail -5 "$O/${so}_$D.log"; exit 4; }
    echo "D=$D $so: $(grep -E '^(fwd|TOTAL)' "$O/${so}_$D.log" | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}')"
  done
done
