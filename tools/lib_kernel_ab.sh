#!/bin/bash
# Kernel-time A/B of library builds: rocprofv3 kernel stats of a short PPO bench per build, ROUNDS times
# interleaved; prints the mean duration of the kernels matching KERNELS (a regex) per build and round.
#   LIBS="libphc_hip.so libphc_hip_x.so" KERNELS="k_tail_ln_fwd|k_head" TAG=r05mm bash tools/lib_kernel_ab.sh
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/${TAG:-libab}; mkdir -p "$O"; export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-2}"); do
  for so in ${LIBS}; do
    d="$O/t_${so%.so}_$r"
    PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline > "$d.log" 2>&1 \
      || { echo "FAILED $so"; tail -5 "$d.log"; exit 9; }
    s=$(find "$d" -name '*kernel_stats.csv' | head -1)
    python3 - "$s" "$so" "$r" "${KERNELS}" <<'PY'
import csv, re, sys
path, so, r, pat = sys.argv[1:5]
for row in csv.DictReader(open(path)):
    if re.search(pat, row["Name"]):
        print(f"{so:28s} round {r}  {float(row['AverageNs']) / 1e3:8.2f} us  n={row['Calls']:>5}  {row['Name'][:70]}")
PY
    tail -1 "$d.log" | cut -c1-120
    rm -rf "$d"
  done
done
