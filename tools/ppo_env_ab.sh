#!/bin/bash
# Default PPO bench line under alternative environment settings (CONFIGS, ';'-separated lists of
# VAR=value), ROUNDS times interleaved, one process each.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
IFS=';' read -ra CFG <<< "${CONFIGS}"
for r in $(seq 1 ${ROUNDS:-1}); do
  i=0
  for c in "${CFG[@]}"; do
    i=$((i + 1))
    env $c timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/ppoenv_${i}_$r.log" 2>&1 || { tail -5 "$OUT/ppoenv_${i}_$r.log"; exit 4; }
    python -c "import json; d=json.loads(open('$OUT/ppoenv_${i}_$r.log').read().strip().splitlines()[-1]); print('[$c]', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', 'gemm frac', round(d['roofline']['frac'],4))"
  done
done
