"""The rollout's trunk GEMMs (4,096 rows per step, twin trunks, BIAS_SILU epilogue with no aux, f16 out)
under the library's tile choice against hipBLASLt (torch.bmm, f16 out, no epilogue): per-layer launch
time by HIP events.  PHC_GEMM_CFG=0 / 2 in the environment forces the 128 x 128 / 256 x 256 tiles.
usage: python tools/rollout_gemm_probe.py [rows]"""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def timed(fn, reps=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [("L1 960->2048", 2, 960, 2048), ("L2 2048->1536", 2, 2048, 1536), ("L3 1536->1024", 2, 1536, 1024),
              ("L4 1024->1024", 2, 1024, 1024), ("L5 1024->512", 2, 1024, 512)]
    tot_o = tot_l = 0.0
    for name, batch, k, n in shapes:
        a = torch.randn((batch, M, k), device=dev, generator=g).half()
        w = (torch.randn((batch, n, k), device=dev, generator=g) / k ** 0.5).half()
        bias = torch.randn(batch * n, device=dev, generator=g)
        z = torch.empty((batch, M, n), dtype=torch.float16, device=dev)
        fl = 2.0 * batch * M * n * k
        t_o = timed(lambda: N.twin_gemm(a, w, N.EPI_BIAS_SILU, z, (batch, n), bias=bias))
        wt = w.transpose(1, 2)
        t_l = timed(lambda: torch.bmm(a, wt))
        tot_o += t_o
        tot_l += t_l
        print(f"{name:16s} ours {t_o:7.1f} us {fl / t_o / 1e6:6.0f} TF/s | hipBLASLt (no epilogue) {t_l:7.1f} us "
              f"{fl / t_l / 1e6:6.0f} TF/s", flush=True)
    print(f"total ours {tot_o:.1f} us, hipBLASLt {tot_l:.1f} us (rows {M})", flush=True)


if __name__ == "__main__":
    main()
