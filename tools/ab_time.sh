#!/bin/bash
# A/B kernel timing of two libphc_hip.so builds on the same box: bench.py --mode env, alternating.
#   tools/ab_time.sh <libA> <libB> "<envs list>" [rounds]
set -u
A=$1; B=$2; ENVS=${3:-4096}; R=${4:-2}
for r in $(seq $R); do
  for L in "$A" "$B"; do
    for E in $ENVS; do
      PHC_HIP_LIB=$L timeout -k 10 300 python bench.py --mode env --envs $E --no-cpu-baseline > gpurun_out/ab_t.log 2>&1 || exit 4
      tail -1 gpurun_out/ab_t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$(basename $L)', $E, round(r['kernel_us'],2), round(r['frac'],3))"
    done
  done
done
