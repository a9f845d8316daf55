#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats + HBM counters.
# Every GPU step runs under its own timeout; anything other than a test failure stops the pass.
#   TESTS=0|1  PROFILE=0|1  ENVS_LIST="4096 32768"  MODES="ppo env"  BENCH_ARGS="..."
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
ENVS_LIST=${ENVS_LIST:-4096}
MODES=${MODES:-ppo env}
BENCH_ARGS=${BENCH_ARGS:-}

if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 3; }
  tail -1 "$OUT/smoke.log"
fi
for MODE in $MODES; do
  for ENVS in $ENVS_LIST; do
    EXTRA=""
    if [ "$ENVS" != "4096" ] || [ "$MODE" != "ppo" ]; then EXTRA="--no-cpu-baseline"; fi
    LOG="$OUT/bench_${MODE}_$ENVS.log"
    timeout -k 10 900 python bench.py --mode "$MODE" --envs "$ENVS" $EXTRA $BENCH_ARGS > "$LOG" 2>&1 || { tail -20 "$LOG"; exit 4; }
    tail -1 "$LOG"
    if [ "${PROFILE:-1}" = "1" ]; then
      export TMPDIR=/tmp
      P="$OUT/prof_trace_${MODE}_$ENVS"
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d "$P" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --mode "$MODE" --envs "$ENVS" --no-cpu-baseline $BENCH_ARGS > "$P.log" 2>&1 || { tail -20 "$P.log"; exit 5; }
      if [ "$MODE" = "env" ]; then
        for C in FETCH_SIZE WRITE_SIZE; do
          timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_env_step" -T -d "$OUT/prof_${C}_$ENVS" -o run --output-format csv -- \
            python3 "$ROOT/bench.py" --mode env --steps 20 --warmup 5 --envs "$ENVS" --no-cpu-baseline > "$OUT/prof_${C}_$ENVS.log" 2>&1 || { tail -20 "$OUT/prof_${C}_$ENVS.log"; exit 6; }
        done
      fi
    fi
  done
done
echo "gpu_check done"
