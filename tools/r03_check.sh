#!/bin/bash
# Round-3 GPU pass: store-pattern probe, GEMM A/B of two library builds, GEMM tests, full GPU suite + bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out; mkdir -p "$O"
timeout -k 10 60 ./tools/store_probe 256 > "$O/store_probe.log" 2>&1 || { echo "store_probe failed"; exit 3; }
ROUNDS=2 VARIANTS="libphc_hip_lds.so libphc_hip_fwd.so libphc_hip.so" bash tools/lib_ab.sh || exit 4
echo "== direct, temporal stores"
PHC_GEMM_NT_OUT_MB=100000 PHC_GEMM_NT_AUX=0 timeout -k 10 120 python tools/gemm_mb_probe.py > "$O/gemm_direct_temporal.log" 2>&1 || exit 4
grep -E "^(fwd|dgrad|TOTAL)" "$O/gemm_direct_temporal.log" | awk '{printf "%s %s %s | ", $1, $2, $(NF-3)}'; echo
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_twin_mlp.py -x -q --timeout 120 --timeout-method thread > "$O/pytest_gemm.log" 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -5 "$O/pytest_gemm.log"; [ $rc -eq 0 ] || exit 5
TESTS=1 PROFILE=0 MODES=ppo bash tools/gpu_check.sh
