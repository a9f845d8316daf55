"""Time phc_policy_act (the rollout tail) at 4096 rows, and phc_obs_half, with HIP events.
usage: [PHC_HIP_LIB=...] python tools/act_probe.py"""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
R, H, A = 4096, 512, 69
y = torch.randn((2, R, H), device=dev, generator=g)
ln = [(torch.rand(H, device=dev) + 0.5, torch.randn(H, device=dev) * 0.1) for _ in range(2)]
w_mu = torch.randn((A, H), device=dev, generator=g) * 0.04
b_mu, w_v, b_v = torch.randn(A, device=dev) * 0.1, torch.randn((1, H), device=dev) * 0.04, torch.zeros(1, device=dev)
sigma = torch.full((A,), -2.9, device=dev)
noise = torch.randn((R, A), device=dev, generator=g)
act, lp, val, mu = torch.empty((R, A), device=dev), torch.empty(R, device=dev), torch.empty(R, device=dev), torch.empty((R, A), device=dev)
obs = torch.randn((R, 934), device=dev, generator=g)
mean, var = torch.randn(934, device=dev) * 0.1, torch.rand(934, device=dev) + 0.5
out = torch.zeros((R, 960), dtype=torch.float16, device=dev)


def run_act():
    N.policy_act(y, ln[0], ln[1], 1e-5, w_mu, b_mu, w_v, b_v, sigma, noise, act, lp, val, mu=mu)


w_mu_t = torch.zeros((H, 72), device=dev)
w_mu_t[:, :A] = w_mu.t()


def run_act_t():
    N.policy_act(y, ln[0], ln[1], 1e-5, w_mu, b_mu, w_v, b_v, sigma, noise, act, lp, val, mu=mu, w_mu_t=w_mu_t)


def run_obs():
    N.obs_half(obs, mean, var, 1e-5, 5.0, out, None)


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


t_wt = timeit(run_act_t)
lp_t = float(lp.double().sum())
print(f"policy_act w_mu_t {t_wt:.1f} us (lp_sum {lp_t:.6f})  policy_act {timeit(run_act):.1f} us  obs_half {timeit(run_obs):.1f} us  lp_sum {float(lp.double().sum()):.6f}")
