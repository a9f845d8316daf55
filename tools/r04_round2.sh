# Round-4 pass 2: full GPU suite (staged env kernel), GEMM DMA-stagger A/B, env staged vs unstaged A/B,
# the driver's bench command, kernel stats, env SQ counters.  Every step has its own time limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
TAG=${TAG:-r04q} SKIP_TESTS=0 BENCH_RUNS="1" bash tools/r04_pass.sh || exit $?
VARIANTS="libphc_hip.so libphc_hip_stg13.so libphc_hip_stg24.so" TESTS="tests/test_gpu_gemm.py tests/test_gpu_twin_mlp.py" ROUNDS=2 bash tools/r04_gemm_ab.sh || exit $?
VARIANTS="libphc_hip.so libphc_hip_st0.so" ROUNDS=2 bash tools/r04_env_ab.sh || exit $?
bash tools/r04_env_sq.sh
