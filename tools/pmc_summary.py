"""HBM bytes per launch of one kernel family from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE), with the gfx950 correction of MI355X_MICROARCH.md §HBM (fetch bytes = 2 x
FETCH_SIZE KiB x 1024; WRITE_SIZE exact for wide stores), plus the same launches' mean duration
from a --kernel-trace pass when given.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel_regex> <out.json> [trace_dir] [alg_per_launch]

kernel_regex "train_gemm" selects the launches bench.py's GEMM timer records (the PPO update's
trunk GEMMs, launched outside the rollout graph): every k_wgrad* dispatch, and k_twin_gemm
dispatches of the 256 x 256 configuration (512-thread workgroups) with more than 256 workgroups
or of the persistent instantiation (template flag `Lb1E`: the wave-specialised forward GEMMs run
one workgroup per CU) — the minibatch's 32768-row GEMMs; the rollout's 4096-row GEMMs have at most
256 workgroups and never run persistent.
"""
import csv
import json
import re
import sys


def selected(r, kernel, grid="Grid_Size", wg="Workgroup_Size"):
    name = r["Kernel_Name"]
    if kernel != "train_gemm":
        return re.search(kernel, name) is not None
    if "k_wgrad" in name:
        return True
    return "k_twin_gemm" in name and int(r[wg]) == 512 and (int(r[grid]) // 512 > 256 or "Lb1E" in name)


def counter(d, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{d}/run_counter_collection.csv"))
            if selected(r, kernel)]
    return sum(vals) / len(vals), len(vals)


def main():
    fd, wd, kernel, out = sys.argv[1:5]
    f, nf = counter(fd, kernel)
    w, nw = counter(wd, kernel)
    res = {"kernel_regex": kernel, "launches": [nf, nw], "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
           "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024, "bytes_per_launch": 2 * f * 1024 + w * 1024,
           "note": "fetch = 2 x FETCH_SIZE (gfx950 half-count correction); includes Infinity-Cache hits"}
    if len(sys.argv) > 5:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                for r in csv.DictReader(open(f"{sys.argv[5]}/run_kernel_trace.csv"))
                if selected(r, kernel, "Grid_Size_X", "Workgroup_Size_X")]
        res["trace_launches"] = len(durs)
        res["trace_mean_us"] = sum(durs) / len(durs) / 1e3
    if len(sys.argv) > 6:
        res["algorithmic_bytes_per_launch"] = float(sys.argv[6])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
