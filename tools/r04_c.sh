set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_env_sizes.py tests/test_gpu_env_trainer.py tests/test_gpu_policy_fused.py tests/test_gpu_kernels.py tests/test_gpu_physics.py tests/test_lstm_golden.py tests/test_gpu_optim.py tests/test_gpu_trainer_edges.py tests/test_gpu_rccl.py tests/test_bench_accounting.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    PHC_FUSED_OBS_OPERAND=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_op${v}_$r.log 2>&1 || { tail -5 $O/bench_op${v}_$r.log; exit 4; }
    python -c "import json,sys; d=json.loads([l for l in open('$O/bench_op${v}_$r.log') if l.startswith('{')][-1]); print('op$v r$r', round(d['value']/1e6,4), round(d['ms_per_step'],2), d['config']['phase_gpu_ms_per_step'])"
  done
done
for cfg in default 0 2; do
  if [ $cfg = default ]; then E=""; else E="PHC_GEMM_CFG=$cfg"; fi
  env $E WGRAD=0 timeout -k 10 120 python tools/gemm_mb_probe.py 4096 > $O/probe4096_$cfg.log 2>&1 || { tail -3 $O/probe4096_$cfg.log; exit 5; }
  echo "cfg $cfg: $(grep -E '^(fwd)' $O/probe4096_$cfg.log | awk '{printf "%s=%s ", $2, $(NF-3)}')"
done
