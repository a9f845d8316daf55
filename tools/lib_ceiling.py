"""Same-shape library ceiling: hipBLASLt (torch.bmm / torch.mm, fp16 operands, fp16 out) on every
trunk GEMM shape of one PPO minibatch (32768 rows), beside phc_twin_gemm with its epilogue discarded
(PHC_GEMM_DISCARD=1 is read at load by the measurement library only, PHC_HIP_LIB=.../libphc_hip_measure.so: run this script twice, with and without it).

usage: python tools/lib_ceiling.py [rows]
"""
import sys

import torch

DIMS = [960, 2048, 1536, 1024, 1024, 512, 512]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    dev = "cuda:0"
    dt = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return (torch.rand(shape, device=dev, generator=g) * 2 - 1).to(dt)

    rows = []
    x = rnd(M, DIMS[0])
    w = rnd(2 * DIMS[1], DIMS[0])
    rows.append(("fwd L1", M, 2 * DIMS[1], DIMS[0], 1, timeit(lambda: torch.mm(x, w.t()))))
    for l in range(2, 7):
        k, n = DIMS[l - 1], DIMS[l]
        a, b = rnd(2, M, k), rnd(2, n, k)
        rows.append((f"fwd L{l}", M, n, k, 2, timeit(lambda: torch.bmm(a, b.transpose(1, 2)))))
    for l in range(6, 1, -1):
        nout, nin = DIMS[l], DIMS[l - 1]
        a, b = rnd(2, M, nout), rnd(2, nin, nout)
        rows.append((f"dgrad L{l}", M, nin, nout, 2, timeit(lambda: torch.bmm(a, b.transpose(1, 2)))))
    for l in range(5, 0, -1):
        nout, nin = DIMS[l], DIMS[l - 1]
        bt = 1 if l == 1 else 2
        gg = rnd(bt, M, nout * (2 if l == 1 else 1))
        zz = rnd(bt, M, nin)
        rows.append((f"wgrad L{l}", nout * (2 if l == 1 else 1), nin, M, bt,
                     timeit(lambda: torch.bmm(gg.transpose(1, 2), zz, out_dtype=torch.float32))))
    tot_us = tot_fl = 0.0
    for name, m, n, k, b, us in rows:
        fl = 2.0 * m * n * k * b
        tot_us += us
        tot_fl += fl
        print(f"{name:10s} m={m:6d} n={n:5d} k={k:6d} b={b} {us:8.1f} us {fl / us / 1e6:7.0f} TF/s", flush=True)
    print(f"TOTAL hipBLASLt {tot_us:.1f} us {tot_fl / tot_us / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
