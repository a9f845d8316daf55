#!/bin/bash
# Bench repeatability: the driver's command three times, then a 3-step line.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/bench3; mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/s20_$i.log" 2>&1 || { tail -20 "$O/s20_$i.log"; exit 4; }
  tail -1 "$O/s20_$i.log" | cut -c1-190
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$O/s3.log" 2>&1 || exit 5
tail -1 "$O/s3.log" | cut -c1-190
