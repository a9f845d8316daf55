#!/bin/bash
# round-4 pass j: row-store + policy tests, policy_act unroll A/B, kernel-trace gap breakdown, PPO bench x2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04j; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_row_store.py \
  tests/test_gpu_policy_fused.py tests/test_gpu_weight_cache.py tests/test_gpu_env_trainer.py tests/test_gpu_fused_ppo.py tests/test_gpu_optim.py tests/test_gpu_twin_mlp.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 3; }
tail -2 "$O/pytest.log"
for so in libphc_hip_u2.so libphc_hip.so libphc_hip_u16.so libphc_hip_u2.so libphc_hip.so libphc_hip_u16.so; do
  echo -n "$so: "; PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/act_probe.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 4
done
TAG=r04j/gaps bash tools/r04_gaps.sh || exit 5
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_$r.log"; exit 6; }
  tail -1 "$O/bench_ppo_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['roofline_env_step']; print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms gemm', round(d['roofline']['frac'],4), 'env', round(e['kernel_us'],2), d['config']['phase_gpu_ms_per_step'])"
done
