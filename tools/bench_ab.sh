#!/bin/bash
# A/B bench.py lines over library builds and run-time settings, interleaved ROUNDS times, one process
# per run, each under its own time limit.  A variant is a library file name under puffer-phc_amd/lib/,
# optionally followed by +VAR=value settings for the run's environment (the same form as gemm_ab.sh):
#   VARIANTS="libphc_hip.so libphc_hip.so+PHC_BLOCK_GRAPH=0 libphc_hip_x.so" ROUNDS=2 bash tools/bench_ab.sh
#   BENCH_ARGS="--mode env --envs 32768" ...   (default: the PPO line, --steps ${STEPS:-5} --warmup ${WARMUP:-5})
# Prints value, ms per step and the dominant kernel's roofline fraction / time per run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS:-libphc_hip.so}; do
    IFS=+ read -r so settings <<< "$v"
    tag=${v//[+=]/_}
    log="$OUT/bench_${tag}_$r.log"
    env PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so ${settings//+/ } timeout -k 10 300 python bench.py \
      --steps ${STEPS:-5} --warmup ${WARMUP:-5} --no-cpu-baseline ${BENCH_ARGS:-} > "$log" 2>&1 || { tail -5 "$log"; exit 4; }
    python - "$log" "$v" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:48s} {d['value'] / 1e6:8.4f} M {d['ms_per_step']:8.2f} ms  {r['kernel'][:28]:28s} "
      f"frac {r['frac']:.4f} {r.get('kernel_us', 0):8.2f} us")
EOF
  done
done
