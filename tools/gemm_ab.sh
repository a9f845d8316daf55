#!/bin/bash
# A/B the per-minibatch GEMM probe over library builds (VARIANTS="libphc_hip.so libphc_hip_x.so"),
# interleaved ROUNDS times in fresh processes; each step under its own timeout.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for so in ${VARIANTS}; do
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/gemm_mb_probe.py > "$OUT/gemm_${so}_$r.log" 2>&1 || { tail -5 "$OUT/gemm_${so}_$r.log"; exit 4; }
  done
done
for so in ${VARIANTS}; do echo "== $so"; cat "$OUT/gemm_${so}_1.log"; for r in $(seq 2 ${ROUNDS:-1}); do tail -1 "$OUT/gemm_${so}_$r.log"; done; done
