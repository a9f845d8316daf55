# Physics step: wave-local LDS ordering (default build) vs workgroup barriers (ws0): oracle tests, then
# interleaved probe rounds (tools/physics_probe.py: kernel time per 4096-env step) and the articulated env bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/phys_ab; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_physics.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for so in libphc_hip.so libphc_hip_ws0.so; do
    echo -n "$so r$r: "; PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 90 python tools/physics_probe.py 4096 30 2>&1 | grep -v amdgpu | tail -1
  done
done
timeout -k 10 300 python bench.py --mode env --physics articulated --no-cpu-baseline > "$O/bench_env_art.log" 2>&1 || { tail -5 "$O/bench_env_art.log"; exit 4; }
tail -1 "$O/bench_env_art.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('roofline_physics'))"
