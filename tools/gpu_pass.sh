#!/bin/bash
# The one GPU-box measurement recipe (replaces the per-pass r0N_*.sh drivers).  Run from the repo root
# on the box, e.g.  TAG=r05a STAGES="tests bench trace" bash tools/gpu_pass.sh
#
#   TAG       output directory under gpurun_out/ (default: pass)
#   STAGES    any of, in this order:
#     tests   pytest -m gpu (TESTS= a test path / -k expression list; default: the whole GPU suite)
#     bench   the driver's command `bench.py --steps 20 --warmup 5`, BENCH_RUNS times (default 2)
#     trace   rocprofv3 kernel trace + stats of the PPO iteration; idle gaps and phase split
#     pmc     FETCH_SIZE / WRITE_SIZE passes (separate) over the trunk GEMMs and the env step
#     env     bench --mode env at 4096 and 32768 envs, their kernel stats and HBM counters
#     phys    the articulated-physics env bench
#     amp     AMP + bf16 PPO kernel stats (BASELINE C5 on one GPU)
#     timeline  host-side timeline + cProfile of PPO iterations (tools/host_timeline.py)
#     hostgap   rocprofv3 kernel + HIP API trace: the host calls inside every GPU idle gap (tools/host_gaps.py)
#     gemm      the per-minibatch GEMM probe over GEMM_VARIANTS (tools/gemm_ab.sh, GEMM_ROUNDS rounds)
#     ab        bench lines over AB_VARIANTS (tools/bench_ab.sh, AB_ROUNDS rounds, AB_ARGS bench args)
#     extra   EXTRA_CMD (a python command line, run under its own limit)
# The round-2..4 per-pass drivers (tools/r0N_*.sh, profile_round.sh, gpu_check.sh, variants.sh, lib_ab.sh,
# ppo_ab.sh, ab_time.sh, ...) named in older profiles/ notes are folded into these stages and into
# gemm_ab.sh / bench_ab.sh (their text stays in the git history).
# Every GPU step runs under its own time limit; the first failure ends the pass (nothing after a failed
# or killed GPU step is started).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-pass}; mkdir -p "$O"; export TMPDIR=/tmp
STAGES=${STAGES:-"tests bench trace"}
has() { case " $STAGES " in *" $1 "*) return 0 ;; esac; return 1; }
fail() { echo "FAILED: $1"; tail -8 "$2"; exit 9; }
stats() { cp "$(find "$1" -name '*kernel_stats.csv' | head -1)" "$2"; }

if has tests; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q ${PYTEST_ARGS:-} --timeout 240 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1 || fail pytest "$O/pytest_gpu.log"
  tail -1 "$O/pytest_gpu.log"
fi
if has bench; then
  for r in $(seq 1 "${BENCH_RUNS:-2}"); do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$O/bench_ppo_4096_s20_$r.log" 2>&1 \
      || fail bench "$O/bench_ppo_4096_s20_$r.log"
    tail -1 "$O/bench_ppo_4096_s20_$r.log" | cut -c1-160
  done
fi
if has trace; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/trace_ppo.log" 2>&1 \
    || fail trace "$O/trace_ppo.log"
  tail -1 "$O/trace_ppo.log" | cut -c1-160
  stats "$O/trace_ppo" "$O/ppo_4096_kernel_stats.csv"
  T=$(find "$O/trace_ppo" -name '*kernel_trace.csv' | head -1)
  cp "$T" "$O/ppo_kernel_trace.csv"
  python tools/trace_gaps.py "$T" 16 > "$O/gaps.txt" 2>&1 || true
  python tools/trace_phases.py "$T" > "$O/phases.txt" 2>&1 || true
  head -40 "$O/gaps.txt"
fi
if has pmc; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_twin_gemm|k_wgrad|k_env_step|k_env_replay" -d "$O/pmc_ppo_$C" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$O/pmc_ppo_$C.log" 2>&1 \
      || fail pmc "$O/pmc_ppo_$C.log"
  done
  python tools/pmc_summary.py "$O/pmc_ppo_FETCH_SIZE" "$O/pmc_ppo_WRITE_SIZE" train_gemm "$O/traffic_gemm_4096.json" "$O/trace_ppo" || true
  python tools/pmc_summary.py "$O/pmc_ppo_FETCH_SIZE" "$O/pmc_ppo_WRITE_SIZE" k_env_ "$O/traffic_fused_ppo_4096.json" \
    "$O/trace_ppo" $((13634 * 4096)) || true
fi
if has env; then
  for E in 4096 32768; do
    timeout -k 10 300 python bench.py --mode env --envs $E --no-cpu-baseline > "$O/bench_env_$E.log" 2>&1 || fail env "$O/bench_env_$E.log"
    tail -1 "$O/bench_env_$E.log" | cut -c1-140
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_env_$E" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --mode env --envs $E --no-cpu-baseline > "$O/trace_env_$E.log" 2>&1 || fail envtrace "$O/trace_env_$E.log"
    stats "$O/trace_env_$E" "$O/env_${E}_kernel_stats.csv"
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_step|k_env_replay" -d "$O/pmc_env_${E}_$C" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" --mode env --steps 20 --warmup 5 --envs $E --no-cpu-baseline \
        > "$O/pmc_env_${E}_$C.log" 2>&1 || fail envpmc "$O/pmc_env_${E}_$C.log"
    done
    python tools/pmc_summary.py "$O/pmc_env_${E}_FETCH_SIZE" "$O/pmc_env_${E}_WRITE_SIZE" k_env_ "$O/traffic_fused_$E.json" \
      "$O/trace_env_$E" $((11714 * E)) || true
  done
fi
if has phys; then
  timeout -k 10 300 python bench.py --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_articulated.log" 2>&1 \
    || fail phys "$O/bench_env_articulated.log"
  tail -1 "$O/bench_env_articulated.log" | cut -c1-140
fi
if has amp; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo_amp_bf16" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --amp --precision bf16 --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace_ppo_amp_bf16.log" 2>&1 \
    || fail amp "$O/trace_ppo_amp_bf16.log"
  tail -1 "$O/trace_ppo_amp_bf16.log" | cut -c1-140
  stats "$O/trace_ppo_amp_bf16" "$O/ppo_4096_amp_bf16_kernel_stats.csv"
fi
if has timeline; then
  timeout -k 10 300 python -u tools/host_timeline.py ${BENCH_ARGS:-} > "$O/host_timeline.txt" 2>&1 || fail timeline "$O/host_timeline.txt"
  head -40 "$O/host_timeline.txt"
fi
if has hostgap; then
  timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace -d "$O/trace_api" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/trace_api.log" 2>&1 \
    || fail hostgap "$O/trace_api.log"
  python tools/host_gaps.py "$(find "$O/trace_api" -name '*kernel_trace.csv' | head -1)" \
    "$(find "$O/trace_api" -name '*hip_api_trace.csv' | head -1)" 15 > "$O/host_gaps.txt" 2>&1 || true
  head -30 "$O/host_gaps.txt"
fi
if has gemm; then
  VARIANTS="${GEMM_VARIANTS:-libphc_hip.so}" ROUNDS=${GEMM_ROUNDS:-2} bash tools/gemm_ab.sh > "$O/gemm_ab.txt" 2>&1 \
    || fail gemm "$O/gemm_ab.txt"
  grep -E "^==|TOTAL" "$O/gemm_ab.txt"
  if [ -n "${GEMM_ROLLOUT:-}" ]; then  # the rollout's 4096-row forward GEMMs per tile configuration
    VARIANTS="$GEMM_ROLLOUT" ROUNDS=1 PROBE_ARGS=4096 WGRAD=0 bash tools/gemm_ab.sh > "$O/gemm_rollout.txt" 2>&1 \
      || fail gemm_rollout "$O/gemm_rollout.txt"
    grep -E "^==|fwd" "$O/gemm_rollout.txt"
  fi
fi
if has ab; then
  VARIANTS="${AB_VARIANTS:-libphc_hip.so}" ROUNDS=${AB_ROUNDS:-2} BENCH_ARGS="${AB_ARGS:-}" bash tools/bench_ab.sh \
    > "$O/bench_ab.txt" 2>&1 || fail ab "$O/bench_ab.txt"
  cat "$O/bench_ab.txt"
fi
if has extra; then
  timeout -k 10 "${EXTRA_LIMIT:-300}" python -u $EXTRA_CMD > "$O/extra.log" 2>&1 || fail extra "$O/extra.log"
  tail -20 "$O/extra.log"
fi
# the raw traces are large; keep the summaries
find "$O" -maxdepth 1 -type d \( -name 'trace_*' -o -name 'pmc_*' \) -exec rm -rf {} + 2>/dev/null
echo "gpu_pass $TAG done"
