"""Fused PPO minibatch tail (phc_tail.hip, policies/fused_ppo.py) vs the reference's unfused
math (needs an MI355X).

* kernel level (phc_tail_ln_fwd / _bwd): LayerNorm + SiLU of both trunks and the value head
  (policies/phc_policy.py:16-61) against float64 torch autograd on the same fp32 trunk output and
  upstream gradients.  Tolerances: h_a / value 1e-5; dy (rounded once to f16) rel 2^-10 of its
  magnitude + 1e-4 of the row scale + 2^-24; column-sum gradients rel. L2 1e-5.
* policy level: fused_ppo_loss vs forward_train + ppo_objective under fp16 autocast on the same
  policy / minibatch: loss and statistics rel 1e-4 (the KL means abs 5e-5: fp32 log-probs of
  ~230 carry 1.4e-5 per row), gradients rel. L2 2e-3 (both share the MFMA trunks and the fp32
  heads; they differ in fp32 summation order only), with FlatGrads-bound (direct) gradients and
  with autograd-returned ones.  Log-ratios and value deltas are kept >= 5e-3 away from the clip
  edges so float32 rounding cannot flip a row's branch.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LOG2PI = 0.5 * np.log(2 * np.pi)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _make_case(M, A=69, H=512, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    r = lambda *s, sc=1.0: torch.randn(s, device=DEV, generator=g) * sc  # noqa: E731
    y = r(2, M, H, sc=2.0) + 0.5
    p = dict(ga=1 + r(H, sc=0.2), ba=r(H, sc=0.2), gc=1 + r(H, sc=0.2), bc=r(H, sc=0.2),
             wmu=r(A, H, sc=0.25), bmu=r(A, sc=0.1), wv=r(1, H, sc=0.05), bv=r(1, sc=0.1))
    log_sigma = torch.full((A,), -2.9, device=DEV)
    # reference mu / value (fp64) to place the PPO data around
    with torch.no_grad():
        mu0, v0 = _ref_heads(y.double(), {k: v.double() for k, v in p.items()})
    pick = lambda vals: torch.tensor(vals, device=DEV)[torch.randint(len(vals), (M,), device=DEV, generator=g)]  # noqa
    sg = torch.exp(log_sigma).double()
    atn = (mu0 + 0.05 * torch.randn(mu0.shape, device=DEV, generator=g, dtype=torch.float64)).float()
    lp0 = (-((atn.double() - mu0) ** 2) / (2 * sg ** 2) - sg.log() - LOG2PI).sum(1)
    old_lp = (lp0 - pick([-0.05, -0.02, 0.0, 0.004, 0.02, 0.05]).double()).float()
    adv = r(M)
    val = (v0 - pick([-0.5, -0.05, 0.05, 0.5]).double()).float()
    ret = val + r(M)
    ms = torch.stack([adv.mean(), adv.std()])
    return y, p, log_sigma, atn, old_lp, adv, ms, val, ret


def _ref_heads(y, p, eps=1e-5):
    H = y.shape[2]
    za = torch.nn.functional.silu(torch.nn.functional.layer_norm(y[0], (H,), p["ga"], p["ba"], eps))
    zc = torch.nn.functional.silu(torch.nn.functional.layer_norm(y[1], (H,), p["gc"], p["bc"], eps))
    mu = za @ p["wmu"].t() + p["bmu"]
    v = (zc @ p["wv"].t() + p["bv"]).view(-1)
    return mu, v


@pytest.mark.parametrize("M", [1000, 4096])
def test_tail_ln_kernels_vs_float64_autograd(M):
    """phc_tail_ln_fwd / _bwd against float64 autograd of LayerNorm + SiLU + value head, driven
    by the same upstream gradients (d h_a, d mu, d value) the PPO backward produces."""
    from puffer_phc_amd import _native as N

    y, p, *_ = _make_case(M)
    g = torch.Generator(device=DEV).manual_seed(5)
    A, H = 69, 512
    tail = N.TailLN(y, (p["ga"], p["ba"]), (p["gc"], p["bc"]), 1e-5, p["wv"], p["bv"])
    h_a, value = tail.forward()
    dh_a = torch.randn((M, H), device=DEV, generator=g)
    dmu = torch.randn((M, A), device=DEV, generator=g)
    dv = torch.randn(M, device=DEV, generator=g)
    dy, part, lay = tail.backward(dh_a, dmu, dv, torch.float16)
    torch.cuda.synchronize()

    yd = y.double().requires_grad_(True)
    pd = {k: v.double().requires_grad_(True) for k, v in p.items()}
    za = torch.nn.functional.silu(torch.nn.functional.layer_norm(yd[0], (H,), pd["ga"], pd["ba"], 1e-5))
    zc = torch.nn.functional.silu(torch.nn.functional.layer_norm(yd[1], (H,), pd["gc"], pd["bc"], 1e-5))
    v = (zc @ pd["wv"].t() + pd["bv"]).view(-1)
    torch.testing.assert_close(h_a.double(), za.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(value.double(), v.detach(), rtol=1e-5, atol=1e-5)
    (za * dh_a.double()).sum().backward(retain_graph=True)
    (v * dv.double()).sum().backward()
    gy = yd.grad
    scale = gy.abs().amax(dim=2, keepdim=True)
    # f16 rounding (2^-11 relative, 2^-24 absolute in the subnormal range) + fp32 summation order
    assert float(((dy.double() - gy).abs() - (2.0 ** -10) * gy.abs() - 1e-4 * scale - 2.0 ** -24).max()) <= 0
    sums = part.double().sum(0)
    w = lambda key, n, o=0: sums[lay[key] + o:lay[key] + o + n]  # noqa: E731
    assert _rel(w("b_mu", A), dmu.double().sum(0)) < 1e-5
    assert _rel(w("w_value", H), pd["wv"].grad.view(-1)) < 1e-5
    assert _rel(w("b_value", 1), pd["bv"].grad) < 1e-5
    assert _rel(w("gamma", H), pd["ga"].grad) < 1e-5
    assert _rel(w("gamma", H, H), pd["gc"].grad) < 1e-5
    assert _rel(w("beta", H), pd["ba"].grad) < 1e-5
    assert _rel(w("beta", H, H), pd["bc"].grad) < 1e-5
    assert _rel(w("b6", 2 * H).view(2, H), gy.sum(1)) < 1e-5


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


@pytest.mark.parametrize("direct", [False, True])
def test_fused_minibatch_matches_unfused(direct):
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs, ppo_objective
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss, fused_ppo_supported

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(_Env(), hidden_size=512, layer_sizes=(256, 128))).to(DEV)
    pol = policy.policy
    cfg = TrainConfig(ent_coef=0.01)
    g = torch.Generator(device=DEV).manual_seed(3)
    M = 2048
    obs = torch.randn((M, 934), device=DEV, generator=g)
    with torch.autocast("cuda", dtype=torch.float16):
        xh = pol.obs_half_input(obs)
        with torch.no_grad():
            mu0, v0 = pol.forward_train(xh)
        assert fused_ppo_supported(pol, xh)
    mu0 = mu0.float()
    atn = mu0 + 0.05 * torch.randn(mu0.shape, device=DEV, generator=g)
    sg = torch.exp(pol.sigma)
    lp0 = (-((atn - mu0) ** 2) / (2 * sg ** 2) - sg.log() - LOG2PI).sum(1)
    pick = lambda vals: torch.tensor(vals, device=DEV)[torch.randint(len(vals), (M,), device=DEV, generator=g)]  # noqa
    old_lp = lp0 - pick([-0.05, -0.02, 0.0, 0.004, 0.02, 0.05])
    adv = torch.randn(M, device=DEV, generator=g)
    val = v0.view(-1).float() - pick([-0.5, -0.05, 0.05, 0.5])
    ret = val + torch.randn(M, device=DEV, generator=g)
    ms = torch.stack([adv.mean(), adv.std()])
    params = [q for q in policy.parameters() if q.requires_grad]

    def run(fused):
        if direct:
            fg = FlatGrads(params)
            fg.zero()
        else:
            policy.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            if fused:
                loss, st = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, ppo_coefs(cfg, pol.soft_bound))
            else:
                mu, nv = pol.forward_train(xh)
                loss, st = ppo_objective(mu, nv, pol.sigma, atn, old_lp, adv, ms, None, val, ret, cfg,
                                         pol.soft_bound)
        (loss * 256.0).backward()
        torch.cuda.synchronize()
        grads = [q.grad.detach().clone() for q in params]
        for q in params:
            q.grad = None
        return loss.detach(), st.detach(), grads

    lf, sf, gf = run(True)
    lu, su, gu = run(False)
    torch.testing.assert_close(lf, lu, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(sf, su, rtol=1e-4, atol=5e-5)
    names = [n for n, q in policy.named_parameters() if q.requires_grad]
    for n, a, b in zip(names, gf, gu):
        assert _rel(a, b) < 2e-3, n


@pytest.mark.parametrize("rows", [2048, 32768])  # split-K weight gradients; the grouped launch
def test_store_grads_writes_every_gradient(rows):
    """fused_ppo_loss(store_grads=True) into a flat buffer pre-filled with NaN gives, bit for bit,
    the gradients of the zero-then-accumulate backward: every parameter has exactly one writer
    (clean_pufferl.core then skips the per-minibatch zeroing of the 68 MB buffer)."""
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(_Env())).to(DEV)
    pol = policy.policy
    cfg = TrainConfig()
    g = torch.Generator(device=DEV).manual_seed(5)
    obs = torch.randn((rows, 934), device=DEV, generator=g)
    atn = 0.1 * torch.randn((rows, 69), device=DEV, generator=g)
    old_lp = torch.randn(rows, device=DEV, generator=g) + 200.0  # ratios ~0: finite objective
    adv, val, ret = (torch.randn(rows, device=DEV, generator=g) for _ in range(3))
    ms = torch.tensor([0.0, 1.0], device=DEV)
    params = [q for q in policy.parameters() if q.requires_grad]
    fg = FlatGrads(params, order=pol.grad_ready_order())
    out = []
    for store in (False, True):
        if store:
            fg.fill_grads_(float("nan"))
        else:
            fg.zero()
        with torch.autocast("cuda", dtype=torch.float16):
            xh = pol.obs_half_input(obs)
            loss, _ = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, ppo_coefs(cfg, pol.soft_bound),
                                     store_grads=store)
        (loss * 64.0).backward()
        torch.cuda.synchronize()
        out.append(fg.flat.detach().clone())
    names = []
    for n_, q in policy.named_parameters():
        if q.requires_grad:
            names.append((n_, q))
    bad = []
    for n_, q in names:
        lo, hi = fg._range[id(q)]
        a, b = out[0][lo:hi], out[1][lo:hi]
        if not torch.equal(a, b):
            bad.append((n_, int((~torch.isfinite(b)).sum()), float((a - b).abs().nan_to_num(1e30).max())))
    assert torch.isfinite(out[0]).all()
    assert not bad, bad
