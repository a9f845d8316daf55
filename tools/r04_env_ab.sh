# Env-step variant A/B (bench.py --mode env, kernel time from its dispatch events), interleaved rounds.
#   VARIANTS="libphc_hip.so libphc_hip_obs0.so"  ENVS_LIST="4096 32768"  ROUNDS=2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/env_ab; mkdir -p "$O"
for r in $(seq 1 ${ROUNDS:-2}); do
  for envs in ${ENVS_LIST:-4096 32768}; do
    for so in ${VARIANTS}; do
      PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 python bench.py --mode env --envs $envs --steps 200 --warmup 20 --no-cpu-baseline > "$O/${so}_${envs}_$r.log" 2>&1 || { tail -5 "$O/${so}_${envs}_$r.log"; exit 4; }
      python - "$O/${so}_${envs}_$r.log" "$so" "$envs" << 'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[2]:24s} envs {sys.argv[3]:>6s}: {r['kernel_us']:7.2f} us  frac {r['frac']:.3f}  value {d['value']/1e6:.1f} M/s")
PY
    done
  done
done
