#!/bin/bash
# A/B the per-minibatch GEMM probe over library builds and run-time settings, interleaved ROUNDS
# times in fresh processes; each step under its own timeout.  A variant is a library file name under
# puffer-phc_amd/lib/, optionally followed by +VAR=value settings for the probe's environment:
#   VARIANTS="libphc_hip.so libphc_hip_measure.so+PHC_GEMM_DISCARD=1 libphc_hip.so+YONLY=1"
# (PHC_GEMM_DISCARD is read only by a measurement build: tools/build_variants.sh measure "-DPHC_MEASURE_GEMM=1")
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS}; do
    IFS=+ read -r so settings <<< "$v"
    tag=${v//[+=]/_}
    env PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so ${settings//+/ } timeout -k 10 120 python tools/gemm_mb_probe.py ${PROBE_ARGS:-} \
      > "$OUT/gemm_${tag}_$r.log" 2>&1 || { tail -5 "$OUT/gemm_${tag}_$r.log"; exit 4; }
  done
done
for v in ${VARIANTS}; do
  tag=${v//[+=]/_}
  echo "== $v"; cat "$OUT/gemm_${tag}_1.log"; for r in $(seq 2 ${ROUNDS:-1}); do tail -1 "$OUT/gemm_${tag}_$r.log"; done
done
