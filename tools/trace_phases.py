"""Split a rocprofv3 kernel trace of `bench.py --mode ppo` into rollout / train phases per
PPO iteration (phase boundary = the k_env_step launches) and list the top kernels of each.

usage: python tools/trace_phases.py <run_kernel_trace.csv> [top]
"""
import csv
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if ("k_env_step" in r["Kernel_Name"] or "k_env_replay" in r["Kernel_Name"])]
    its, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if b - a > 400:
            its.append(cur)
            cur = [b]
        else:
            cur.append(b)
    its.append(cur)
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
    span = lambda rs: (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e6  # noqa: E731
    for k in range(len(its) - 1):
        roll, train = rows[its[k][0]:its[k][-1] + 1], rows[its[k][-1] + 1:its[k + 1][0]]
        print(f"iteration {k}: rollout {len(roll)} kernels span {span(roll):.1f} ms busy "
              f"{sum(map(dur, roll)) / 1e6:.1f} ms | train {len(train)} kernels span {span(train):.1f} ms busy "
              f"{sum(map(dur, train)) / 1e6:.1f} ms")
    for name, rs in (("train", train), ("rollout", roll)):
        c, n = Counter(), Counter()
        for r in rs:
            c[r["Kernel_Name"][:70]] += dur(r)
            n[r["Kernel_Name"][:70]] += 1
        print(f"top {name} kernels (last iteration):")
        for key, v in c.most_common(top):
            print(f"  {key:70s} {n[key]:5d} {v / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
