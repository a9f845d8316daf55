"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) for one kernel into HBM bytes
per launch, with the gfx950 correction from MI355X_MICROARCH.md §HBM: FETCH_SIZE reports
half the bytes of a wide coalesced read, so fetch bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE
(KiB) is exact for wide stores.

usage: python tools/pmc_traffic.py <prof_dir_root> <envs> <kernel_regex> <out.json>
"""
import csv
import json
import re
import sys


def mean_counter(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if re.search(kernel, r["Kernel_Name"])]
    return sum(vals) / len(vals), len(vals)


def main():
    root, envs, kernel, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    f, nf = mean_counter(f"{root}/prof_FETCH_SIZE_{envs}/run_counter_collection.csv", kernel)
    w, nw = mean_counter(f"{root}/prof_WRITE_SIZE_{envs}/run_counter_collection.csv", kernel)
    fetch = 2 * f * 1024
    write = w * 1024
    res = {"kernel": kernel, "envs": envs, "launches": [nf, nw], "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
           "fetch_bytes_corrected": fetch, "write_bytes": write, "bytes_per_launch": fetch + write,
           "algorithmic_bytes_per_launch": 10886 * envs,
           "note": "fetch = 2 x FETCH_SIZE (gfx950 half-count correction); includes Infinity-Cache hits"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
