"""Probe: an fp32 GEMM as ONE bf16 GEMM over a tripled K (bf16x3: a_hi b_hi + a_lo b_hi + a_hi b_lo,
fp32 accumulate / output) vs hipBLASLt's xf32 ("high") on the twin-trunk shapes.  Prints time and
the rel. L2 error of each against a float64 product (debug / tuning aid).

usage: python tools/x3_probe.py
"""
import time

import torch

dev = "cuda:0"
M = 32768


def split(x):
    hi = x.bfloat16()
    lo = (x - hi.float()).bfloat16()
    return hi, lo


def x3_operands(a, b):
    ah, al = split(a)
    bh, bl = split(b)
    return torch.cat([ah, al, ah], 1), torch.cat([bh, bh, bl], 0)


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [("fwd L1 934->4096", M, 934, 4096), ("fwd 2048->1536", M, 2048, 1536),
              ("fwd 1536->1024", M, 1536, 1024), ("fwd 1024->512", M, 1024, 512),
              ("dX 1536->2048", M, 1536, 2048), ("dW 2048x1536 over M", 1536, M, 2048),
              ("dW 4096x934 over M", 4096, M, 934)]
    for name, m, k, n in shapes:
        a = torch.randn((m, k), device=dev, generator=g)
        b = torch.randn((k, n), device=dev, generator=g) / k ** 0.5
        ref = (a.double() @ b.double())
        fl = 2.0 * m * k * n
        torch.set_float32_matmul_precision("high")
        t_x = timeit(lambda: a @ b)
        e_x = float((a @ b - ref).norm() / ref.norm())
        torch.set_float32_matmul_precision("highest")
        t_f = timeit(lambda: a @ b, 5)
        a3, b3 = x3_operands(a, b)
        t_3 = timeit(lambda: torch.mm(a3, b3, out_dtype=torch.float32))
        e_3 = float((torch.mm(a3, b3, out_dtype=torch.float32) - ref).norm() / ref.norm())
        t_s = timeit(lambda: x3_operands(a, b))
        ah, bh = a.bfloat16(), b.bfloat16()
        t_1 = timeit(lambda: torch.mm(ah, bh, out_dtype=torch.float32))
        e_1 = float((torch.mm(ah, bh, out_dtype=torch.float32) - ref).norm() / ref.norm())
        # TF32 emulation: inputs rounded to a 10-bit mantissa, exact-ish product
        def tf32(x):
            i = x.view(torch.int32)
            return ((i + 0x1000) & ~0x1FFF).view(torch.float32)
        e_t = float((tf32(a).double() @ tf32(b).double() - ref).norm() / ref.norm())
        print(f"{name:22s} xf32 {t_x:7.3f} ms {fl / t_x / 1e9:6.0f} TF/s err {e_x:.1e} | fp32 {t_f:7.3f} ms | "
              f"bf16x3 {t_3:7.3f} ms {fl / t_3 / 1e9:6.0f} TF/s err {e_3:.1e} (+split {t_s:.3f} ms) | "
              f"bf16 {t_1:7.3f} ms err {e_1:.1e} | tf32-emul err {e_t:.1e}", flush=True)


if __name__ == "__main__":
    main()
