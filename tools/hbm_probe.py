"""Practical HBM ceiling on this box: torch's device copy (read + write), a read-only sum and a fill
(write only) over buffers the size of the env step's per-launch traffic (48 MB at 4096 envs, 384 MB
at 32768), timed with HIP events over repeated launches.  Context for roofline_env_step.frac, whose
peak is the 8 TB/s data-sheet figure.  Usage: python tools/hbm_probe.py [MB ...]"""
import json
import sys

import torch


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [48, 384, 2048]
    out = []
    for mb in sizes:
        n = mb * (1 << 20) // 4
        a = torch.randn(n, device="cuda")
        b = torch.empty_like(a)
        reps = max(20, 4096 // mb)
        t_copy = timed(lambda: b.copy_(a), reps)
        t_sum = timed(lambda: a.sum(), reps)
        t_fill = timed(lambda: b.fill_(1.0), reps)
        nb = n * 4
        row = {"MB": mb, "copy_TBps": 2 * nb / t_copy / 1e12, "read_TBps": nb / t_sum / 1e12,
               "write_TBps": nb / t_fill / 1e12, "copy_us": t_copy * 1e6}
        out.append(row)
        print(json.dumps(row), flush=True)
    return out


if __name__ == "__main__":
    main()
