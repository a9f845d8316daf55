#!/bin/bash
# Default PPO bench line against alternative builds of libphc_hip.so (VARIANTS), ROUNDS times interleaved.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for so in ${VARIANTS}; do
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/ppo_${so}_$r.log" 2>&1 || { tail -5 "$OUT/ppo_${so}_$r.log"; exit 4; }
    python -c "import json; d=json.loads(open('$OUT/ppo_${so}_$r.log').read().strip().splitlines()[-1]); print('$so', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', 'gemm frac', round(d['roofline']['frac'],4))"
  done
done
