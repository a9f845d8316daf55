# Rollout GEMM tile threshold A/B (PHC_GEMM_BIG_MIN: fewest 256 x 256 tiles that select the 256 x 256 kernel)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/bigmin; mkdir -p "$O"
for r in 1 2; do
  for bm in ${BIGMINS:-256 192 128}; do
    PHC_GEMM_BIG_MIN=$bm timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/ppo_${bm}_${r}.log" 2>&1 || { tail -5 "$O/ppo_${bm}_${r}.log"; exit 4; }
    python -c "import json; d=json.loads(open('$O/ppo_${bm}_${r}.log').read().strip().splitlines()[-1]); print('big_min $bm', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', d['config']['phase_gpu_ms_per_step'])"
  done
done
