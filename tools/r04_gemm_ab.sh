# GEMM variant check + A/B: correctness tests of each variant library, then interleaved probe rounds.
#   VARIANTS="libphc_hip.so libphc_hip_p8.so"  TESTS="tests/test_gpu_gemm.py ..."  ROUNDS=2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/gemm_ab; mkdir -p "$O"
for so in ${VARIANTS}; do
  if [ -n "${TESTS:-}" ] && [ "$so" != "libphc_hip.so" ]; then
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 600 python -u -m pytest ${TESTS} -x -q --timeout 300 --timeout-method thread > "$O/tests_$so.log" 2>&1
    rc=$?; echo "tests $so rc=$rc"; tail -3 "$O/tests_$so.log"
    [ $rc -eq 0 ] || exit $rc
  fi
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ${VARIANTS}; do
    for mode in full main; do
      if [ $mode = main ]; then D=1; else D=; fi
      env ${D:+PHC_GEMM_DISCARD=$D} PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/gemm_mb_probe.py > "$O/${so}_${mode}_$r.log" 2>&1 || { tail -5 "$O/${so}_${mode}_$r.log"; exit 4; }
      echo "$so $mode r$r: $(grep -E '^(fwd|dgrad|wgrad)' "$O/${so}_${mode}_$r.log" | awk '{printf "%s%s=%s ", substr($1,1,1), $2, $(NF-3)}') $(grep TOTAL "$O/${so}_${mode}_$r.log")"
    done
  done
done
