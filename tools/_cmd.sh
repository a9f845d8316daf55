set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_env_trainer.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in 0 1 0 1; do
  PHC_WGRAD_STREAM=$v timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_$v.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/b_$v.log').read().strip().splitlines()[-1]); print('stream=$v', round(d['ms_per_step'],2), 'ms', round(d['value']), d['roofline']['achieved'])"
done
