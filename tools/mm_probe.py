"""Time torch.mm / bmm variants used by the twin MLP backward (dW GEMMs) on the GPU."""
import time

import torch

torch.set_float32_matmul_precision("high")
dev = "cuda:0"
M, K, N = 32768, 1536, 2048
for dt in (torch.float16, torch.bfloat16):
    g = torch.randn((2, M, N), device=dev).to(dt)
    z = torch.randn((2, M, K), device=dev).to(dt)
    for name, fn in [("bmm", lambda: torch.bmm(g.transpose(1, 2), z)),
                     ("bmm_out_f32", lambda: torch.bmm(g.transpose(1, 2), z, out_dtype=torch.float32)),
                     ("mm_out_f32", lambda: torch.mm(g[0].t(), z[0], out_dtype=torch.float32)),
                     ("mm", lambda: torch.mm(g[0].t(), z[0]))]:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 0.5 and n < 50:
            fn()
            n += 1
        torch.cuda.synchronize()
        dt_ms = (time.perf_counter() - t0) / n * 1e3
        fl = 2 * M * K * N * (2 if name.startswith("bmm") else 1)
        print(f"{str(dt):15s} {name:12s} {dt_ms:8.3f} ms  {fl / dt_ms / 1e9:8.1f} TF/s", flush=True)
