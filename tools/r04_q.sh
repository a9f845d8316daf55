#!/bin/bash
# round-4 pass q: A/B of PHC_NOISE_AHEAD (the rollout's next noise draw between the policy graph and the env step)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04q2; mkdir -p "$O"; export TMPDIR=/tmp
for r in 1 2; do for a in 0 1; do
  PHC_NOISE_AHEAD=$a timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_ahead${a}_$r.log" 2>&1 || { tail -5 "$O/bench_ahead${a}_$r.log"; exit 6; }
  echo -n "ahead=$a r$r: "; tail -1 "$O/bench_ahead${a}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', d['config']['phase_gpu_ms_per_step'])"
done; done
PHC_NOISE_AHEAD=1 TAG=r04q2/gaps bash tools/r04_gaps.sh > "$O/gaps_run.log" 2>&1 || { tail -5 "$O/gaps_run.log"; exit 5; }
head -8 "$O/gaps/gaps.txt"
