# Round-4 pass 6: GPU suite (RMS partial / PPO forward load hoisting), physics hit compaction A/B, PPO bench x2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04g; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/libphc_hip_pc1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_physics.py -x -q --timeout 300 --timeout-method thread > "$O/tests_pc1.log" 2>&1
rc=$?; tail -2 "$O/tests_pc1.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for so in libphc_hip.so libphc_hip_pc1.so; do
    echo -n "$so r$r: "; PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 90 python tools/physics_probe.py 4096 30 2>&1 | grep -v amdgpu | tail -1
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 python bench.py --mode env --physics articulated --no-cpu-baseline > "$O/art_${so}_$r.log" 2>&1 || { tail -5 "$O/art_${so}_$r.log"; exit 4; }
    tail -1 "$O/art_${so}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline_physics']; print('   bench env articulated', round(d['value']/1e6,2), 'M/s  physics', round(r['kernel_us'],1), 'us frac', round(r['frac'],3))"
  done
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_ppo_4096_s20_$r.log" 2>&1 || { tail -5 "$O/bench_ppo_4096_s20_$r.log"; exit 4; }
  tail -1 "$O/bench_ppo_4096_s20_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,4), 'M', round(d['ms_per_step'],2), 'ms', d['config']['phase_gpu_ms_per_step'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_ppo" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/trace_ppo.log" 2>&1 || { tail -5 "$O/trace_ppo.log"; exit 6; }
cp "$(find "$O/trace_ppo" -name '*kernel_stats.csv' | head -1)" "$O/ppo_4096_kernel_stats.csv"; rm -rf "$O/trace_ppo"
grep -E "k_rms_partial|k_ppo_fwd|k_rms_merge" "$O/ppo_4096_kernel_stats.csv" | cut -d, -f1-4
