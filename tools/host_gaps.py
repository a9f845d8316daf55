"""Where the host holds the GPU idle: a rocprofv3 `--hip-trace --kernel-trace` run of `bench.py --mode ppo`;
for the second-to-last PPO iteration, every GPU idle gap longer than MIN_US (default 20) together with
the HIP API calls the host was inside during that gap (blocking calls such as hipStreamSynchronize /
hipEventSynchronize / hipMemcpy show up as long calls; hipGraphLaunch as the host-side cost of a replay).

usage: python tools/host_gaps.py <run_kernel_trace.csv> <run_hip_api_trace.csv> [min_us]
"""
import csv
import sys
from collections import Counter


def main():
    ker = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    api = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    idx = [i for i, r in enumerate(ker) if ("k_env_step" in r["Kernel_Name"] or "k_env_replay" in r["Kernel_Name"])]
    its, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if b - a > 300:
            its.append(cur)
            cur = [b]
        else:
            cur.append(b)
    its.append(cur)
    k = len(its) - 2
    lo, hi = its[k][0], its[k + 1][0]
    t_lo, t_hi = int(ker[lo]["Start_Timestamp"]), int(ker[hi]["Start_Timestamp"])
    name = "Function" if "Function" in api[0] else ("Kind" if "Kind" not in api[0] else list(api[0].keys())[3])
    # long API calls of the iteration
    calls = Counter()
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t_lo and e <= t_hi:
            calls[r.get("Function", r.get(name))] += e - s
    print(f"iteration span {(t_hi - t_lo) / 1e6:.3f} ms; host time inside HIP calls by function (ms):")
    for f, v in calls.most_common(12):
        print(f"  {v / 1e6:8.3f}  {f}")
    print(f"GPU idle gaps > {min_us} us and the HIP calls overlapping them:")
    for a, b in zip(ker[lo:hi], ker[lo + 1:hi + 1]):
        g0, g1 = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
        if (g1 - g0) / 1e3 < min_us:
            continue
        over = [r for r in api if int(r["Start_Timestamp"]) < g1 and int(r["End_Timestamp"]) > g0]
        desc = ", ".join(f"{r.get('Function', r.get(name))}({(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f})"
                         for r in over[:6])
        print(f"  {(g1 - g0) / 1e3:8.1f} us  {a['Kernel_Name'][:40]} -> {b['Kernel_Name'][:40]} | {desc}")


if __name__ == "__main__":
    main()
