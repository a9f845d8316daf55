set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_gemm.py tests/test_gpu_amp.py tests/test_gpu_ppo_loss.py -x -v --timeout 300 --timeout-method thread > gpurun_out/disc.log 2>&1
rc=$?; tail -30 gpurun_out/disc.log; exit $rc
