#!/bin/bash
# main loop alone (PHC_GEMM_DISCARD=1) vs full epilogue, 256x256 default tiles and 128x128 tiles
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python tools/gemm_mb_probe.py > "$OUT/dp_$name.log" 2>&1 || { tail -5 "$OUT/dp_$name.log"; exit 4; }
  echo "== $name"; grep -v amdgpu.ids "$OUT/dp_$name.log" | grep -v checksums
}
run base PHC_GEMM_PP_MIN=0
run base_discard PHC_GEMM_DISCARD=1
run c128_discard PHC_GEMM_CFG=0 PHC_GEMM_DISCARD=1
run pp_discard PHC_GEMM_PP_MIN=1 PHC_GEMM_DISCARD=1
