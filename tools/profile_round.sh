#!/bin/bash
# One GPU-box pass producing this round's judged evidence under gpurun_out/round/: the default
# bench line, rocprofv3 kernel stats of the PPO iteration, HBM counters (FETCH_SIZE / WRITE_SIZE,
# separate passes) for the trunk GEMM (PPO mode) and the env step (env mode, 4096 and 32768 envs).
# Every GPU step has its own timeout; the first failure ends the pass.
set -eu
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=$ROOT/gpurun_out/round
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > "$O/bench_ppo_4096.log" 2>&1
tail -1 "$O/bench_ppo_4096.log" | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_twin_gemm|k_wgrad" -d "$O/pmc_gemm_$C" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_gemm_$C.log" 2>&1
done
for E in 4096 32768; do
  timeout -k 10 600 python bench.py --mode env --envs $E --no-cpu-baseline > "$O/bench_env_$E.log" 2>&1
  tail -1 "$O/bench_env_$E.log" | cut -c1-120
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_env_$E" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --mode env --envs $E --no-cpu-baseline > "$O/trace_env_$E.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_step" -d "$O/pmc_env_${E}_$C" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --mode env --steps 20 --warmup 5 --envs $E --no-cpu-baseline \
      > "$O/pmc_env_${E}_$C.log" 2>&1
  done
done

# HBM bytes per launch (+ the trace's mean duration) of the same launches bench.py times
python tools/pmc_summary.py "$O/pmc_gemm_FETCH_SIZE" "$O/pmc_gemm_WRITE_SIZE" train_gemm "$O/traffic_gemm_4096.json" "$O/trace_ppo"
for E in 4096 32768; do
  # the default env phase is the fused replay step (phc_env_step_replay: k_env_step<true, true>)
  python tools/pmc_summary.py "$O/pmc_env_${E}_FETCH_SIZE" "$O/pmc_env_${E}_WRITE_SIZE" k_env_step "$O/traffic_fused_$E.json" \
    "$O/trace_env_$E" $((11714 * E))
done
# the AMP + bf16 configuration (BASELINE C5): kernel stats, to show which kernels the discriminator runs on
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo_amp_bf16" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --amp --precision bf16 --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_ppo_amp_bf16.log" 2>&1
echo "profile_round done"
