#!/bin/bash
# two-workgroups-per-CU GEMM (cfg 3: 256x128, BK 32) with the second workgroup of each CU held
# back by half a tile (PHC_GEMM_STAGGER=f,256,512) vs the default 256x256 configuration
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/epi_ab; mkdir -p $O
for r in 1 2; do
for v in "2 0" "3 0" "3 0.5" "3 0.25" "3 1.0"; do
  set -- $v
  echo "== cfg=$1 stagger=$2 round $r"
  env PHC_GEMM_CFG=$1 $( [ $2 != 0 ] && echo PHC_GEMM_STAGGER=$2,256,512 ) timeout -k 10 120 python tools/gemm_mb_probe.py > $O/g_$1_$2_$r.log 2>&1 || { tail -5 $O/g_$1_$2_$r.log; exit 5; }
  grep -E "^(fwd|dgrad|TOTAL)" $O/g_$1_$2_$r.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}'; echo
done
done
