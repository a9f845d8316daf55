"""Time phc_twin_gemm (hand-written MFMA GEMM + fused epilogue) against hipBLASLt (torch.mm with
fp32 output) plus the separate epilogue kernel, on the twin-trunk shapes at 32768 rows.

usage: python tools/twin_gemm_probe.py [fp16|bf16]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
dt = torch.bfloat16 if len(sys.argv) > 1 and sys.argv[1] == "bf16" else torch.float16
M = 32768


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def split_costs():
    """Main loop alone (PHC_GEMM_DISCARD=1 with the measurement library, PHC_HIP_LIB=.../libphc_hip_measure.so) vs with each epilogue."""
    import os
    g = torch.Generator(device=dev).manual_seed(0)
    for name, batch, k, n in [("L2 fwd 2048->1536", 2, 2048, 1536), ("L4 fwd 1024->1024", 2, 1024, 1024)]:
        a = torch.randn((batch, M, k), device=dev, generator=g).to(dt)
        w = (torch.randn((batch, n, k), device=dev, generator=g) / k ** 0.5).to(dt)
        bias = torch.randn(batch * n, device=dev, generator=g)
        pre = torch.empty((batch, M, n), device=dev)
        z = torch.empty((batch, M, n), dtype=dt, device=dev)
        fl = 2.0 * batch * M * n * k
        t = timeit(lambda: N.twin_gemm(a, w, N.EPI_STORE, z, (batch, n)))
        print(f"{name:20s} discard={os.environ.get('PHC_GEMM_DISCARD')} store-f16 {t:.3f} ms {fl / t / 1e9:.0f} TF/s",
              flush=True)


def one(name_prefix, reps=50):
    """Run only phc_twin_gemm (BIAS_SILU) on one shape, for counter collection."""
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = {"L2": (2, 2048, 1536), "L1": (1, 960, 4096), "L4": (2, 1024, 1024)}
    batch, k, n = shapes[name_prefix]
    a = torch.randn((batch, M, k), device=dev, generator=g).to(dt)
    w = (torch.randn((batch, n, k), device=dev, generator=g) / k ** 0.5).to(dt)
    bias = torch.randn(batch * n, device=dev, generator=g)
    pre = torch.empty((batch, M, n), device=dev)
    z = torch.empty((batch, M, n), dtype=dt, device=dev)
    for _ in range(reps):
        N.twin_gemm(a, w, N.EPI_BIAS_SILU, z, (batch, n), bias=bias, aux=pre)
    torch.cuda.synchronize()


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "split":
        return split_costs()
    if len(sys.argv) > 3 and sys.argv[2] == "one":
        return one(sys.argv[3])
    g = torch.Generator(device=dev).manual_seed(0)
    # (name, batch, k, n): forward layers; "dX" rows use the transposed weight
    shapes = [("L1 fwd 960->4096", 1, 960, 4096), ("L2 fwd 2048->1536", 2, 2048, 1536),
              ("L3 fwd 1536->1024", 2, 1536, 1024), ("L4 fwd 1024->1024", 2, 1024, 1024),
              ("L5 fwd 1024->512", 2, 1024, 512), ("L2 dX 1536->2048", 2, 1536, 2048),
              ("L3 dX 1024->1536", 2, 1024, 1536)]
    for name, batch, k, n in shapes:
        a = torch.randn((batch, M, k), device=dev, generator=g).to(dt)
        w = (torch.randn((batch, n, k), device=dev, generator=g) / k ** 0.5).to(dt)
        bias = torch.randn(batch * n, device=dev, generator=g)
        pre = torch.empty((batch, M, n), device=dev)
        z = torch.empty((batch, M, n), dtype=dt, device=dev)
        fl = 2.0 * batch * M * n * k
        t_ours = timeit(lambda: N.twin_gemm(a, w, N.EPI_BIAS_SILU, z, (batch, n), bias=bias, aux=pre))
        t_store = timeit(lambda: N.twin_gemm(a, w, N.EPI_STORE, pre, (batch, n)))
        wt = w.transpose(1, 2)
        if batch == 1:
            t_lib = timeit(lambda: torch.mm(a[0], wt[0], out_dtype=torch.float32))
        else:
            t_lib = timeit(lambda: torch.bmm(a, wt, out_dtype=torch.float32))
        y = torch.bmm(a, wt, out_dtype=torch.float32)
        t_epi = timeit(lambda: N.bias_act_fwd(y, N.GROUPED, bias, None, z, N.GROUPED, M, batch, n, N.ACT_SILU))
        ref = y + bias.view(batch, 1, n)
        N.twin_gemm(a, w, N.EPI_BIAS_SILU, z, (batch, n), bias=bias, aux=pre)
        err = float((pre - ref).norm() / ref.norm())
        print(f"{name:20s} ours(fused) {t_ours:7.3f} ms {fl / t_ours / 1e9:6.0f} TF/s | ours(store f32) "
              f"{t_store:7.3f} ms {fl / t_store / 1e9:6.0f} TF/s | hipBLASLt {t_lib:7.3f} ms "
              f"{fl / t_lib / 1e9:6.0f} TF/s + epilogue {t_epi:.3f} ms | rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
