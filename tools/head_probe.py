"""Time the mu-head kernels (phc_mu_head_fwd / _dgrad / _wgrad) at one PPO minibatch (32768 rows, hidden 512,
69 actions) with HIP events; prints us per launch and a checksum (to compare library builds).

usage: [PHC_HIP_LIB=...] python tools/head_probe.py [rows]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
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
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn((M, 512), device="cuda", generator=g)
    dmu = torch.randn((M, 69), device="cuda", generator=g) * 1e-3
    out = {}
    out["wgrad"] = timeit(lambda: N.mu_head_wgrad_parts(dmu, h, 128))
    p = N.mu_head_wgrad_parts(dmu, h, 128)
    print(f"mu head wgrad {out['wgrad']:.2f} us  checksum {float(p.double().sum()):.9e} "
          f"{float(p.double().abs().sum()):.9e}  lib={os.environ.get('PHC_HIP_LIB', 'default')}")


if __name__ == "__main__":
    main()
