# Round-4 pass 7: GPU suite on the env-step load fixes + physics hit compaction default; PPO bench x2,
# env-mode 4096 / 32768, articulated env bench, PPO kernel stats
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04h; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_4096_s20_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_4096_s20_$r.log"; exit 4; }
  tail -1 "$O/bench_ppo_4096_s20_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['roofline_env_step']; print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms gemm', round(d['roofline']['frac'],4), 'env', round(e['kernel_us'],2), round(e['frac'],3), d['config']['phase_gpu_ms_per_step'])"
done
for E in 4096 32768; do
  timeout -k 10 300 python bench.py --mode env --envs $E --no-cpu-baseline > "$O/bench_env_$E.log" 2>&1 || { tail -5 "$O/bench_env_$E.log"; exit 4; }
  tail -1 "$O/bench_env_$E.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('env $E', round(d['value']/1e6,1), 'M/s', round(r['kernel_us'],2), 'us', round(r['frac'],3))"
done
timeout -k 10 300 python bench.py --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_articulated.log" 2>&1 || { tail -5 "$O/bench_env_articulated.log"; exit 4; }
tail -1 "$O/bench_env_articulated.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline_physics']; print('articulated env', round(d['value']/1e6,2), 'M/s physics', round(r['kernel_us'],1), 'us frac', round(r['frac'],3))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || { tail -5 "$O/trace_ppo.log"; exit 6; }
cp "$(find "$O/trace_ppo" -name '*kernel_stats.csv' | head -1)" "$O/ppo_4096_kernel_stats.csv"; rm -rf "$O/trace_ppo"
grep -E "k_env_step|k_rms_partial|k_ppo_fwd" "$O/ppo_4096_kernel_stats.csv" | cut -d, -f1-4
