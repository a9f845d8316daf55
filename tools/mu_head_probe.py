"""Time the fp32 mu-head kernels (phc_mu_head_*) against the library GEMMs they replace, at one
PPO minibatch (32768 x 512 -> 69).  usage: python tools/mu_head_probe.py"""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
M, H, A = 32768, 512, 69
h = torch.randn((M, H), device=dev)
w = torch.randn((A, H), device=dev) * 0.05
b = torch.randn(A, device=dev)
dmu = torch.randn((M, A), device=dev)


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


rows = [("h.clone (67 MB read+write)", lambda: h.clone()), ("h.sum (67 MB read)", lambda: h.sum()),
        ("fwd kernel", lambda: N.mu_head_fwd(h, w, b)), ("fwd addmm", lambda: torch.addmm(b, h, w.t())),
        ("dgrad kernel", lambda: N.mu_head_dgrad(dmu, w)), ("dgrad mm", lambda: torch.mm(dmu, w))]
for s in (128,):
    rows.append((f"wgrad kernel S={s}", lambda s=s: N.mu_head_wgrad_parts(dmu, h, s)))
    rows.append((f"wgrad kernel S={s} + sum", lambda s=s: N.mu_head_wgrad_parts(dmu, h, s).sum(0)))
rows.append(("wgrad mm", lambda: torch.mm(dmu.t(), h)))
for name, fn in rows:
    us = timeit(fn)
    print(f"{name:26s} {us:8.1f} us  {2.0 * M * H * A / us / 1e6:6.1f} TF/s", flush=True)
