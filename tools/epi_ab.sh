#!/bin/bash
# GEMM main-loop schedule A/B on one PPO minibatch's GEMMs: the two-buffer K-step loop (sched 0)
# vs the phased loop (sched 1); full epilogue and main loop only
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/epi_ab; mkdir -p $O
PHC_GEMM_SCHED=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_twin_mlp.py > $O/tests_pp.log 2>&1 || { tail -30 $O/tests_pp.log; exit 4; }
tail -1 $O/tests_pp.log
for r in 1 2; do
for v in "0 0" "1 0" "0 1" "1 1"; do
  set -- $v
  echo "== sched=$1 discard=$2 round $r"
  env PHC_GEMM_SCHED=$1 $( [ $2 != 0 ] && echo PHC_GEMM_DISCARD=$2 ) timeout -k 10 120 python tools/gemm_mb_probe.py > $O/s_$1_$2_$r.log 2>&1 || { tail -5 $O/s_$1_$2_$r.log; exit 5; }
  grep -E "^(fwd|dgrad|TOTAL)" $O/s_$1_$2_$r.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}'; echo
done
done
