# Round-4 pass 4: env tests + physics wave-sync A/B + env staged/unstaged A/B (PPO and env mode) + rollout
# graph vs eager + rollout tile threshold + same-shape library ceiling.  Each step under its own limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/envppo; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_sizes.py tests/test_gpu_env_trainer.py tests/test_gpu_kernels.py tests/test_gpu_amp.py tests/test_gpu_weight_cache.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/r04_phys_ab.sh || exit $?
for r in 1 2; do
  for so in libphc_hip.so libphc_hip_st0.so; do
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/ppo_${so}_$r.log" 2>&1 || { tail -5 "$O/ppo_${so}_$r.log"; exit 4; }
    python -c "import json; d=json.loads(open('$O/ppo_${so}_$r.log').read().strip().splitlines()[-1]); e=d['roofline_env_step']; print('$so', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms  env', round(e['kernel_us'],2), 'us frac', round(e['frac'],3), d['config']['phase_gpu_ms_per_step'])"
  done
done
VARIANTS="libphc_hip.so libphc_hip_st0.so" ROUNDS=1 bash tools/r04_env_ab.sh || exit $?
for gph in 1 0; do
  PHC_ROLLOUT_GRAPH=$gph timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/graph_${gph}.log" 2>&1 || { tail -5 "$O/graph_${gph}.log"; exit 4; }
  python -c "import json; d=json.loads(open('$O/graph_${gph}.log').read().strip().splitlines()[-1]); c=d['config']; print('graph $gph', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', c['phase_gpu_ms_per_step'], c['phase_host_wall_ms_per_step'])"
done
for bm in 192; do
  PHC_GEMM_BIG_MIN=$bm timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bigmin_${bm}.log" 2>&1 || { tail -5 "$O/bigmin_${bm}.log"; exit 4; }
  python -c "import json; d=json.loads(open('$O/bigmin_${bm}.log').read().strip().splitlines()[-1]); print('big_min $bm', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', d['config']['phase_gpu_ms_per_step'])"
done
timeout -k 10 180 python tools/lib_ceiling.py > "$O/lib_ceiling.log" 2>&1 || { tail -5 "$O/lib_ceiling.log"; exit 7; }
PHC_GEMM_DISCARD=1 timeout -k 10 180 python tools/lib_ceiling.py > "$O/lib_ceiling_main.log" 2>&1 || { tail -5 "$O/lib_ceiling_main.log"; exit 7; }
tail -16 "$O/lib_ceiling.log"; tail -16 "$O/lib_ceiling_main.log"
