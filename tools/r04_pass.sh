# Round-4 evidence pass: GPU suite, the driver's bench command, rocprofv3 kernel stats of the PPO bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-r04p}; mkdir -p "$O"; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for r in ${BENCH_RUNS:-1 2}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_4096_s20_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_4096_s20_$r.log"; exit 4; }
  tail -1 "$O/bench_ppo_4096_s20_$r.log" | cut -c1-160
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || { tail -5 "$O/trace_ppo.log"; exit 6; }
f=$(find "$O/trace_ppo" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/ppo_4096_kernel_stats.csv"
t=$(find "$O/trace_ppo" -name "*kernel_trace.csv" | head -1); python tools/glue_kernels.py "$t" 2 > "$O/glue.txt" 2>&1 || true
head -25 "$O/ppo_4096_kernel_stats.csv" | cut -d, -f1-6
