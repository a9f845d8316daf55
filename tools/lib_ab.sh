#!/bin/bash
# A/B library builds on one minibatch's GEMMs: VARIANTS="libphc_hip.so libphc_hip_x.so", ROUNDS rounds, interleaved
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/lib_ab; mkdir -p "$O"
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ${VARIANTS}; do
    echo "== $so round $r"
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/gemm_mb_probe.py > "$O/${so}_$r.log" 2>&1 || { tail -5 "$O/${so}_$r.log"; exit 4; }
    grep -E "^(fwd|dgrad|TOTAL)" "$O/${so}_$r.log" | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}'; echo
  done
done
