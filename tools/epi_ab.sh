#!/bin/bash
# GEMM CU-stagger A/B on one PPO minibatch's GEMMs (PHC_GEMM_STAGGER = fraction of a tile's
# main loop that every other CU starts late; 0 = off)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/epi_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
for r in 1 2; do
for v in 0 0.25 0.5 0.75 1.0; do
  echo "== stagger=$v round $r"
  PHC_GEMM_STAGGER=$v timeout -k 10 120 python tools/gemm_mb_probe.py > $O/s_${v}_$r.log 2>&1 || { tail -5 $O/s_${v}_$r.log; exit 5; }
  grep -E "^(fwd|dgrad|TOTAL)" $O/s_${v}_$r.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}'; echo
done
done
