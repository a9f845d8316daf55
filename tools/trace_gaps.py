"""Idle gaps of the GPU timeline in a rocprofv3 kernel trace of `bench.py --mode ppo`: for the last
complete PPO iteration (phases split at the k_env_step launches as tools/trace_phases.py does), the
gaps between consecutive kernels of the rollout and of the train phase, summed by the (previous ->
next) kernel pair.

usage: python tools/trace_gaps.py <run_kernel_trace.csv> [top]
"""
import csv
import sys
from collections import Counter


def short(n):
    n = n.split("(")[0]
    for p in ("void ", "phc::", "at::native::"):
        n = n.replace(p, "")
    return n[:48]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    idx = [i for i, r in enumerate(rows) if ("k_env_step" in r["Kernel_Name"] or "k_env_replay" in r["Kernel_Name"])]
    its, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if b - a > 400:
            its.append(cur)
            cur = [b]
        else:
            cur.append(b)
    its.append(cur)
    k = len(its) - 2
    phases = {"rollout": rows[its[k][0] - 20:its[k][-1] + 1], "train": rows[its[k][-1] + 1:its[k + 1][0] - 20]}
    for name, rs in phases.items():
        gaps, cnt = Counter(), Counter()
        tot = 0
        for a, b in zip(rs, rs[1:]):
            g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
            if g <= 0:
                continue
            tot += g
            key = f"{short(a['Kernel_Name'])} -> {short(b['Kernel_Name'])}"
            gaps[key] += g
            cnt[key] += 1
        span = int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])
        print(f"{name}: {len(rs)} kernels, span {span / 1e6:.3f} ms, idle {tot / 1e6:.3f} ms")
        for key, v in gaps.most_common(top):
            print(f"  {v / 1e3:9.1f} us  n={cnt[key]:4d}  mean {v / cnt[key] / 1e3:6.2f} us  {key}")


if __name__ == "__main__":
    main()
