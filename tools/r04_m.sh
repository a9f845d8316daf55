#!/bin/bash
# round-4 pass m: full GPU suite, driver bench x2, idle-gap breakdown
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04m; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 3; }
tail -1 "$O/pytest_gpu.log"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_4096_s20_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_4096_s20_$r.log"; exit 6; }
  tail -1 "$O/bench_ppo_4096_s20_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['roofline_env_step']; print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms gemm', round(d['roofline']['frac'],4), 'env', round(e['kernel_us'],2), d['config']['phase_gpu_ms_per_step'])"
done
TAG=r04m/gaps bash tools/r04_gaps.sh > "$O/gaps_run.log" 2>&1 || { tail -5 "$O/gaps_run.log"; exit 5; }
head -30 "$O/gaps/gaps.txt"
