#!/bin/bash
# Round-4 evidence pass on the final tree: GPU suite, the driver's bench command x3, rocprofv3 kernel stats
# of the PPO iteration, HBM counters (separate FETCH_SIZE / WRITE_SIZE passes) of the trunk GEMMs and of the
# env step (env mode, 4096 / 32768 envs, plus the rollout-context step with the fused operand), the
# articulated-physics env bench, and the AMP + bf16 kernel stats.  Each GPU step under its own limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-r04f}; mkdir -p "$O"; export TMPDIR=/tmp
fail() { echo "FAILED: $1"; tail -5 "$2"; exit 9; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || fail pytest "$O/pytest_gpu.log"
  tail -1 "$O/pytest_gpu.log"
fi
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_4096_s20_$r.log" 2>&1 || fail bench "$O/bench_ppo_4096_s20_$r.log"
  tail -1 "$O/bench_ppo_4096_s20_$r.log" | cut -c1-140
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || fail trace "$O/trace_ppo.log"
cp "$(find "$O/trace_ppo" -name '*kernel_stats.csv' | head -1)" "$O/ppo_4096_kernel_stats.csv"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_twin_gemm|k_wgrad|k_env_step" -d "$O/pmc_ppo_$C" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_ppo_$C.log" 2>&1 || fail pmc "$O/pmc_ppo_$C.log"
done
python tools/pmc_summary.py "$O/pmc_ppo_FETCH_SIZE" "$O/pmc_ppo_WRITE_SIZE" train_gemm "$O/traffic_gemm_4096.json" "$O/trace_ppo" || true
python tools/pmc_summary.py "$O/pmc_ppo_FETCH_SIZE" "$O/pmc_ppo_WRITE_SIZE" k_env_step "$O/traffic_fused_ppo_4096.json" "$O/trace_ppo" $((13634 * 4096)) || true
for E in 4096 32768; do
  timeout -k 10 300 python bench.py --mode env --envs $E --no-cpu-baseline > "$O/bench_env_$E.log" 2>&1 || fail env "$O/bench_env_$E.log"
  tail -1 "$O/bench_env_$E.log" | cut -c1-120
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_env_$E" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --mode env --envs $E --no-cpu-baseline > "$O/trace_env_$E.log" 2>&1 || fail envtrace "$O/trace_env_$E.log"
  cp "$(find "$O/trace_env_$E" -name '*kernel_stats.csv' | head -1)" "$O/env_${E}_kernel_stats.csv"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_step" -d "$O/pmc_env_${E}_$C" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --mode env --steps 20 --warmup 5 --envs $E --no-cpu-baseline \
      > "$O/pmc_env_${E}_$C.log" 2>&1 || fail envpmc "$O/pmc_env_${E}_$C.log"
  done
  python tools/pmc_summary.py "$O/pmc_env_${E}_FETCH_SIZE" "$O/pmc_env_${E}_WRITE_SIZE" k_env_step "$O/traffic_fused_$E.json" \
    "$O/trace_env_$E" $((11714 * E)) || true
done
timeout -k 10 300 python bench.py --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_articulated.log" 2>&1 || fail phys "$O/bench_env_articulated.log"
tail -1 "$O/bench_env_articulated.log" | cut -c1-120
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo_amp_bf16" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --amp --precision bf16 --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_ppo_amp_bf16.log" 2>&1 || fail amp "$O/trace_ppo_amp_bf16.log"
cp "$(find "$O/trace_ppo_amp_bf16" -name '*kernel_stats.csv' | head -1)" "$O/ppo_4096_amp_bf16_kernel_stats.csv"
rm -rf "$O"/trace_* "$O"/pmc_*/ 2>/dev/null; ls "$O"
echo r04_final done
