"""Time the twin-trunk GEMM shapes (forward / dX / dW) for one 32768-row minibatch at a given
precision, with the first layer's K = 934 or padded (debug / tuning aid).

usage: python tools/gemm_shapes.py [xf32|fp16|bf16] [pad]
"""
import sys
import time

import torch

torch.set_float32_matmul_precision("high")
dev = "cuda:0"
prec = sys.argv[1] if len(sys.argv) > 1 else "xf32"
pad = int(sys.argv[2]) if len(sys.argv) > 2 else 934
dt = {"xf32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[prec]
M = 32768
sizes = [pad, 2048, 1536, 1024, 1024, 512, 512]


def bench(name, fn, flops):
    fn()
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while n < 20:
        fn()
        n += 1
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    print(f"{name:28s} {ms:7.3f} ms {flops / ms / 1e9:7.1f} TF/s", flush=True)
    return ms


tot = 0.0
x = torch.randn((M, sizes[0]), device=dev).to(dt)
W1 = torch.randn((2 * sizes[1], sizes[0]), device=dev).to(dt)
g1 = torch.randn((M, 2 * sizes[1]), device=dev).to(dt)
f = 2 * M * sizes[0] * 2 * sizes[1]
tot += bench(f"L1 fwd K={sizes[0]}", lambda: torch.mm(x, W1.t()), f)
tot += bench(f"L1 dW K={sizes[0]}", lambda: torch.mm(g1.t(), x), f)
for l in range(1, 6):
    k, n = sizes[l], sizes[l + 1]
    z = torch.randn((2, M, k), device=dev).to(dt)
    W = torch.randn((2, n, k), device=dev).to(dt)
    g = torch.randn((2, M, n), device=dev).to(dt)
    f = 2 * 2 * M * k * n
    if dt == torch.bfloat16:
        tot += bench(f"L{l + 1} fwd {k}->{n}", lambda: [torch.mm(z[i], W[i].t()) for i in range(2)], f)
        tot += bench(f"L{l + 1} dX", lambda: [torch.mm(g[i], W[i]) for i in range(2)], f)
        tot += bench(f"L{l + 1} dW", lambda: [torch.mm(g[i].t(), z[i]) for i in range(2)], f)
    else:
        tot += bench(f"L{l + 1} fwd {k}->{n}", lambda: torch.bmm(z, W.transpose(1, 2)), f)
        tot += bench(f"L{l + 1} dX", lambda: torch.bmm(g, W), f)
        tot += bench(f"L{l + 1} dW", lambda: torch.bmm(g.transpose(1, 2), z), f)
print(f"total per minibatch {tot:.2f} ms (x16 = {tot * 16:.1f} ms per PPO iteration)")

if dt != torch.bfloat16:
    print("-- split-K weight gradients (batched chunks + fp32 sum)")
    for l in range(0, 6):
        k, n = sizes[l], sizes[l + 1]
        G = 1 if l == 0 else 2
        if l == 0:
            n = 2 * n
        z = torch.randn((G, M, k), device=dev).to(dt)
        g = torch.randn((G, M, n), device=dev).to(dt)
        f = 2 * G * M * k * n
        for S in (1, 4, 8, 16, 32):
            def fn(S=S):
                gs = g.reshape(G * S, M // S, n)
                zs = z.reshape(G * S, M // S, k)
                if dt == torch.float32:
                    p = torch.bmm(gs.transpose(1, 2), zs)
                else:
                    p = torch.bmm(gs.transpose(1, 2), zs, out_dtype=torch.float32)
                return p.view(G, S, n, k).sum(1)
            bench(f"L{l + 1} dW {n}x{k} S={S}", fn, f)
