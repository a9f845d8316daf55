"""VALU instructions per k_physics_step launch from a rocprofv3 --pmc pass of
tools/profile_physics.sh -> profiles/physics_valu_<envs>.json (read by bench.py --physics
articulated for the physics kernel's VALU-issue roofline).
Usage: python tools/physics_valu_summary.py <pmc dir> <envs> <out.json>"""
import collections
import csv
import glob
import json
import sys

d, envs, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = []
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "k_physics_step" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
res = {"kernel": "k_physics_step", "envs": envs, "substeps_per_launch": 16, "launches": len(agg["SQ_INSTS_VALU"]),
       "valu_instr_per_launch": m["SQ_INSTS_VALU"], "lds_instr_per_launch": m.get("SQ_INSTS_LDS"),
       "waves_per_launch": m.get("SQ_WAVES"),
       "note": "SQ_INSTS_VALU = wave-level VALU instructions issued per launch (scales with the envs: one wave per 2 envs)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
