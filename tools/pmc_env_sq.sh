#!/bin/bash
# SQ counters of the fused env step (bench.py --mode env) at ENVS (default "4096 32768"): VALU
# instructions per wave, VALU-active and wait fractions.  One pass per counter set, each under its own
# kill timeout.  LIB: the library under puffer-phc_amd/lib/ (default the product one).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=${SQOUT:-$ROOT/gpurun_out/env_sq}; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
for E in ${ENVS:-4096 32768}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    env PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/${LIB:-libphc_hip.so} timeout -s KILL 120 rocprofv3 --pmc $P \
      --kernel-include-regex "k_env_replay" -d "$OUT/env_${E}_$i" -o run --output-format csv -- \
      python3 bench.py --mode env --envs $E --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/env_${E}_$i.log" 2>&1 \
      || { tail -5 "$OUT/env_${E}_$i.log"; exit 5; }
  done
  python3 - "$OUT" "$E" <<'PY'
import csv, glob, sys, collections
out, E = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{out}/env_{E}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
w = m.get("SQ_WAVES", 1) or 1
wc = m.get("SQ_WAVE_CYCLES", 1) or 1
print(f"envs {E}: waves {w:.0f}  VALU/wave {m.get('SQ_INSTS_VALU', 0) / w:.0f}  TRANS/wave {m.get('SQ_INSTS_VALU_TRANS_F', 0) / w:.0f}"
      f"  SALU/wave {m.get('SQ_INSTS_SALU', 0) / w:.0f}  LDS/wave {m.get('SQ_INSTS_LDS', 0) / w:.0f}"
      f"  VMEM rd/wr per wave {m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f}/{m.get('SQ_INSTS_VMEM_WR', 0) / w:.0f}"
      f"  branch/wave {m.get('SQ_INSTS_BRANCH', 0) / w:.0f}")
g = m.get("GRBM_GUI_ACTIVE", 0) / 8
simd_cycles = g * 1024  # GPU-active cycles x SIMDs (GRBM summed over the 8 XCDs)
if simd_cycles:
    print(f"   VALU busy (ACTIVE_INST_VALU x 4 / SIMD cycles) {m.get('SQ_ACTIVE_INST_VALU', 0) * 4 / simd_cycles:.2f}"
          f"   wave-cycles: WAIT_ANY {m.get('SQ_WAIT_ANY', 0) / wc:.2f}  WAIT_INST_ANY {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
          f"  ACTIVE_INST_ANY {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  thread-cycles VALU / (64 x VALU insts)"
          f" {m.get('SQ_THREAD_CYCLES_VALU', 0) / max(1.0, 64 * m.get('SQ_INSTS_VALU', 1)):.2f}"
          f"  GRBM_GUI_ACTIVE/8 {g:.0f} cycles per launch")
PY
done
