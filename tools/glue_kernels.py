"""List the library (non-phc) kernels of one PPO iteration in a rocprofv3 kernel trace with their phc
neighbours, to find torch glue launches (elementwise / reduce / copy kernels) on the hot path.

usage: python tools/glue_kernels.py <run_kernel_trace.csv> [iteration]
"""
import csv
import sys
from collections import Counter


def short(n):
    n = n.replace("void ", "")
    return n[:90]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    it = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    idx = [i for i, r in enumerate(rows) if "k_env_step" in r["Kernel_Name"] or "k_env_replay" in r["Kernel_Name"]]
    its, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if b - a > 400:
            its.append(cur)
            cur = [b]
        else:
            cur.append(b)
    its.append(cur)
    lo, hi = its[it][0], its[it + 1][0] if it + 1 < len(its) else len(rows)
    seq = rows[lo:hi]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    glue = Counter()
    gt = Counter()
    ctx = {}
    for i, r in enumerate(seq):
        n = r["Kernel_Name"]
        is_phc = "phc" in n or n.startswith("k_")
        if not is_phc:
            prev = next((short(seq[j]["Kernel_Name"]) for j in range(i - 1, -1, -1)
                         if "phc" in seq[j]["Kernel_Name"] or seq[j]["Kernel_Name"].startswith("k_")), "-")
            nxt = next((short(seq[j]["Kernel_Name"]) for j in range(i + 1, len(seq))
                        if "phc" in seq[j]["Kernel_Name"] or seq[j]["Kernel_Name"].startswith("k_")), "-")
            key = (short(n), prev, nxt)
            glue[key] += 1
            gt[key] += dur(r)
    tot = sum(gt.values())
    print(f"iteration {it}: {len(seq)} kernels, {sum(map(dur, seq)) / 1e3:.2f} ms busy; glue {sum(glue.values())} "
          f"kernels {tot / 1e3:.2f} ms")
    for key, c in sorted(glue.items(), key=lambda kv: -gt[kv[0]]):
        print(f"{c:4d} x {gt[key] / c:7.1f} us = {gt[key]:8.1f} us | {key[0]}\n      after {key[1]}\n      before {key[2]}")


if __name__ == "__main__":
    main()
