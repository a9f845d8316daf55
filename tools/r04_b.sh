set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
VARIANTS="libphc_hip.so libphc_hip_p8.so" TESTS="tests/test_gpu_gemm.py tests/test_gpu_twin_mlp.py" ROUNDS=2 bash tools/r04_gemm_ab.sh || exit $?
VARIANTS="libphc_hip.so libphc_hip_obs0.so" ROUNDS=2 bash tools/r04_env_ab.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_sizes.py tests/test_gpu_env_trainer.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b_env_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04b_env_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_env_sq.sh
