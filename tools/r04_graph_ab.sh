# Rollout: captured-graph replay vs eager launches (PHC_ROLLOUT_GRAPH), PPO bench lines, interleaved
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/graph_ab; mkdir -p "$O"
for r in 1 2; do
  for gph in 1 0; do
    PHC_ROLLOUT_GRAPH=$gph timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/ppo_${gph}_${r}.log" 2>&1 || { tail -5 "$O/ppo_${gph}_${r}.log"; exit 4; }
    python -c "import json; d=json.loads(open('$O/ppo_${gph}_${r}.log').read().strip().splitlines()[-1]); c=d['config']; print('graph $gph', round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', c['phase_gpu_ms_per_step'], c['phase_host_wall_ms_per_step'])"
  done
done
