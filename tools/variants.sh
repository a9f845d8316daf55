#!/bin/bash
# Time bench.py against alternative builds of libphc_hip.so (PHC_HIP_LIB) in one process each.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for so in ${VARIANTS}; do
  for e in ${ENVS_LIST:-4096 32768}; do
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 python bench.py --mode env --steps 200 --warmup 20 --envs $e --no-cpu-baseline > "$OUT/var_${so}_$e.log" 2>&1 || { tail -5 "$OUT/var_${so}_$e.log"; exit 4; }
    python -c "import json,sys; d=json.loads(open('$OUT/var_${so}_$e.log').read().strip().splitlines()[-1]); print('$so', $e, round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_us'],2), 'us kernel', round(d['roofline']['frac'],3))"
  done
done
