set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-r04_trace}; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || { tail -5 "$O/trace_ppo.log"; exit 6; }
f=$(find "$O/trace_ppo" -name "*kernel_trace.csv" | head -1)
python tools/glue_kernels.py "$f" 2 > "$O/glue.txt"; head -80 "$O/glue.txt"
