#!/bin/bash
# Env-kernel A/B on the box: rocprofv3 kernel stats of `bench.py --mode env` per library build and env
# count (the rocprof duration: dispatch-inclusive, the basis the roofline reports).
#   LIBS="libphc_hip.so libphc_hip_x.so libphc_hip.so+PHC_REF_CACHE=0" SIZES="4096 32768" ROUNDS=2 TAG=r06a bash tools/env_ab.sh
# (a variant is a library under puffer-phc_amd/lib/, optionally followed by +VAR=value settings)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-envab}; mkdir -p "$O"; export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-1}"); do
  for E in ${SIZES:-4096 32768}; do
    for v in ${LIBS:-libphc_hip.so}; do
      IFS=+ read -r so settings <<< "$v"
      tag=${v//[+=]/_}
      d="$O/t_${E}_${tag%.so}_$r"
      env PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so ${settings//+/ } timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$d" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" --mode env --envs "$E" --steps "${STEPS:-100}" --warmup 20 \
        --no-cpu-baseline ${BENCH_ARGS:-} > "$d.log" 2>&1 || { echo "FAILED $E $so"; tail -20 "$d.log"; exit 9; }
      s=$(find "$d" -name '*kernel_stats.csv' | head -1)
      python3 - "$s" "$E" "$v" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if "k_env" in row["Name"]:
        print(f"envs {sys.argv[2]:>6} {sys.argv[3]:26s} {float(row['AverageNs'])/1e3:8.2f} us  min {float(row['MinNs'])/1e3:8.2f}"
              f"  n={row['Calls']:>5}  {row['Name'][:48]}")
PY
      rm -rf "$d"
    done
  done
done
