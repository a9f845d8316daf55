#!/bin/bash
# round-4 pass k: changed-kernel tests, kernel-trace gap breakdown + kernel stats, PPO bench x2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04k; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_row_store.py \
  tests/test_gpu_fused_ppo.py tests/test_gpu_optim.py tests/test_gpu_env_sizes.py tests/test_gpu_physics.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 3; }
tail -1 "$O/pytest.log"
TAG=r04k/gaps bash tools/r04_gaps.sh || exit 5
f=$(find "$O/gaps/trace_ppo" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$O/kstats.txt" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
d=collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name']].append(int(r['End_Timestamp'])-int(r['Start_Timestamp']))
for k,v in sorted(d.items(), key=lambda kv:-sum(kv[1]))[:30]:
    print(f"{sum(v)/1e6:8.2f} ms n={len(v):5d} avg={sum(v)/len(v)/1e3:8.1f} {k[:90]}")
PY
head -30 "$O/kstats.txt"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_$r.log"; exit 6; }
  tail -1 "$O/bench_ppo_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['roofline_env_step']; print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms gemm', round(d['roofline']['frac'],4), 'env', round(e['kernel_us'],2), d['config']['phase_gpu_ms_per_step'])"
done
timeout -k 10 300 python tools/host_profile.py 3 > "$O/host_profile.txt" 2>&1 || { tail -5 "$O/host_profile.txt"; exit 7; }
grep -A30 "tottime" "$O/host_profile.txt" | head -45
