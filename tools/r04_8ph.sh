# 8-phase GEMM main loop vs the 2-phase default: correctness, interleaved probe rounds, SQ counters of both.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
VARIANTS="libphc_hip.so libphc_hip_8ph.so libphc_hip_8phb.so" TESTS="tests/test_gpu_gemm.py tests/test_gpu_twin_mlp.py" ROUNDS=2 bash tools/r04_gemm_ab.sh || exit $?
SQOUT=$ROOT/gpurun_out/sq_default bash tools/pmc_gemm_sq.sh || exit $?
PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/libphc_hip_8ph.so SQOUT=$ROOT/gpurun_out/sq_8ph bash tools/pmc_gemm_sq.sh || exit $?
