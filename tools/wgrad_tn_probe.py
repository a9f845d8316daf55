"""Weight-gradient GEMMs of the default trunk at 32768 rows: the current library path
(twin_mlp._weight_grad_parts, hipBLASLt split-K) vs phc_weight_grad (transposed-read MFMA kernel)
at S = 1..16 splits, each followed by phc_reduce_into of the partials into fp32 gradient buffers.
Prints us per layer (GEMM + reduce) and the GEMM alone; checks the two paths agree."""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402
from puffer_phc_amd.policies.twin_mlp import _weight_grad_parts  # noqa: E402

dev = "cuda:0"
M = 32768
DIMS = [960, 2048, 1536, 1024, 1024, 512]


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


tot_lib, tot_best = 0.0, 0.0
for l in range(5, 0, -1):
    nout, nin = DIMS[l], DIMS[l - 1]
    B = 1 if l == 1 else 2
    n = nout * (2 if l == 1 else 1)
    g = (torch.randn((B, M, n), device=dev) * 0.1).half()
    z = torch.randn((B, M, nin), device=dev).half()
    dst = [torch.zeros((n, nin), device=dev) for _ in range(B)]

    def lib_run():
        part = _weight_grad_parts(g, z)  # [B, S, n, k]
        N.reduce_into([(part[b], dst[b]) for b in range(B)], accumulate=True)

    def tn_run(S, reduce=True):
        part = N.weight_grad(g, z, S)  # [S, B, n, k]
        if reduce:
            N.reduce_into([(part[:, b], dst[b]) for b in range(B)], accumulate=True)

    ref = _weight_grad_parts(g, z).sum(1)
    got = N.weight_grad(g, z, 4).sum(0)
    err = float((got - ref).abs().max() / ref.abs().max())
    t_lib = timeit(lib_run)
    res = []
    for S in (1, 2, 4, 8, 16):
        if M % (64 * S):
            continue
        res.append((S, timeit(lambda: tn_run(S)), timeit(lambda: tn_run(S, False))))
    best = min(res, key=lambda t: t[1])
    flops = 2.0 * B * n * nin * M
    tot_lib += t_lib
    tot_best += best[1]
    print(f"L{l} n={n} k={nin} B={B} lib {t_lib:.0f}us | " +
          " ".join(f"S{S}:{t:.0f}({tg:.0f})" for S, t, tg in res) +
          f" | best S={best[0]} {best[1]:.0f}us = {flops / best[2] / 1e6:.0f} TF/s gemm-only, relerr {err:.1e}",
          flush=True)
print(f"total lib {tot_lib:.0f}us, tn best {tot_best:.0f}us")

# the grouped launch over all five layers (no split), as the trunk backward issues it
probs = []
keep = []
for l in range(5, 0, -1):
    nout, nin = DIMS[l], DIMS[l - 1]
    if l == 1:
        g = (torch.randn((M, 2 * nout), device=dev) * 0.1).half()
        z = torch.randn((M, nin), device=dev).half()
        d = [torch.zeros((nout, 934), device=dev) for _ in range(2)]
        probs.append((g, z, d, nout, 934))
    else:
        g = (torch.randn((2, M, nout), device=dev) * 0.1).half()
        z = torch.randn((2, M, nin), device=dev).half()
        d = [torch.zeros((nout, nin), device=dev) for _ in range(2)]
        probs.append((g, z, d, nout, nin))
t = timeit(lambda: N.weight_grad_group(probs, accumulate=True))
print(f"grouped all layers: {t:.0f}us = {2 * 32768 * sum(p[0].shape[-1] * p[1].shape[-1] * (2 if p[0].dim() == 3 else 1) for p in probs) / t / 1e6:.0f} TF/s")
