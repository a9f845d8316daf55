"""Weight-gradient GEMM split-K sweep: for each trunk layer, dW[b] = g[b]^T z[b] over 32768 rows
as S batched hipBLASLt GEMMs of M/S rows + phc_reduce_into of the S fp32 partials, for
S in 1..32; prints us per (GEMM + reduce) and the current _split_k choice."""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402
from puffer_phc_amd.policies.twin_mlp import _split_k  # noqa: E402

dev = "cuda:0"
M = 32768
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


for l in range(6, 0, -1):
    nout, nin = DIMS[l], DIMS[l - 1]
    B = 1 if l == 1 else 2
    n = nout * (2 if l == 1 else 1)
    g = torch.randn((B, M, n), device=dev).half()
    z = torch.randn((B, M, nin), device=dev).half()
    dst = [torch.zeros((n, nin), device=dev) for _ in range(B)]
    res = []
    for S in (1, 2, 4, 8, 16, 32):
        def run():
            part = torch.bmm(g.reshape(B * S, M // S, n).transpose(1, 2), z.reshape(B * S, M // S, nin),
                             out_dtype=torch.float32).view(B, S, n, nin)
            N.reduce_into([(part[b], dst[b]) for b in range(B)], accumulate=True)
        res.append((S, timeit(run)))
    best = min(res, key=lambda t: t[1])
    print(f"L{l} n={n} k={nin} B={B} cur S={_split_k(M, n, nin, B)} " +
          " ".join(f"S{S}:{t:.0f}" for S, t in res) + f" best S={best[0]}", flush=True)
