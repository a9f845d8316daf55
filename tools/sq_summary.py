"""Per-GEMM SQ counter ratios from tools/pmc_gemm_sq.sh passes (grouped by grid size)."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
for mode in ("main", "full"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{out}/sq_{mode}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {mode}")
    for grid, cs in sorted(agg.items(), key=lambda kv: -kv[0]):
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        line = [f"grid {grid:8d}"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in m:
                line.append(f"{k[3:]} {m[k] / wc:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # MFMA busy cycles summed over the SIMDs vs GPU-active cycles (8 XCDs summed) x 32 SIMDs per XCD
            line.append(f"mfma_util {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
        for k in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES"):
            if k in m:
                line.append(f"{k[3:] if k.startswith('SQ_') else k} {m[k]:.3g}")
        print("  ".join(line))
