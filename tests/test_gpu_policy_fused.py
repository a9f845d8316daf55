"""Fused policy pieces around the trunk GEMMs (phc_policy.hip) vs plain PyTorch (needs an MI355X).

* phc_obs_half: RunningNorm + rounding into the padded f16 / bf16 GEMM operand, with and without
  a row gather — bit-equal to phc_rms_normalize followed by torch's cast (same fp32 expression,
  one rounding).
* phc_policy_act: LayerNorm+SiLU of both trunks, mu / value heads, Normal sample and log_prob
  vs torch fp32 modules evaluated with exact fp32 GEMMs (matmul precision "highest") and
  torch.distributions.Normal on the same noise: mu / actions / value within 2e-5 absolute,
  log_prob within 2e-3 absolute (a sum of 69 terms of magnitude ~1 whose (a - mu)^2 / 2 var part
  amplifies the 1-ulp differences of a - mu by 1 / var = e^5.8).
* PHCPolicy.act_rollout (the rollout step's fused path) vs the module path under fp16 autocast.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("gather", [False, True])
@pytest.mark.parametrize("n", [1000, 20001, 70001])  # 1, 4 and 8 rows per wave, ragged last block
def test_obs_half_matches_rms_normalize(dtype, gather, n):
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(0)
    d, ld = 934, 960
    obs = torch.randn((n, d), device=DEV, generator=g) * 4 + 1
    mean = torch.rand((1, d), device=DEV, generator=g) - 0.5
    var = torch.rand((1, d), device=DEV, generator=g) * 2 + 0.01
    m = n * 7 // 9 if gather else n
    rows = torch.randperm(n, device=DEV, generator=g)[:m] if gather else None
    out = torch.full((m, ld), 7.0, dtype=dtype, device=DEV)
    N.obs_half(obs, mean, var, 1e-5, 10.0, out, rows)
    ref = N.rms_normalize((obs[rows] if gather else obs).contiguous(), mean, var, 1e-5, 10.0)
    assert torch.equal(out[:, :d], ref.to(dtype))
    assert torch.equal(out[:, d:], torch.zeros_like(out[:, d:]))
    # empty input is a no-op
    N.obs_half(obs[:0], mean, var, 1e-5, 10.0, out[:0])


def _heads(H, A, g):
    ln_a = (torch.randn(H, device=DEV, generator=g) * 0.3 + 1, torch.randn(H, device=DEV, generator=g) * 0.1)
    ln_c = (torch.randn(H, device=DEV, generator=g) * 0.3 + 1, torch.randn(H, device=DEV, generator=g) * 0.1)
    w_mu = torch.randn((A, H), device=DEV, generator=g) * 0.05
    b_mu = torch.randn(A, device=DEV, generator=g) * 0.01
    w_v = torch.randn((1, H), device=DEV, generator=g) * 0.05
    b_v = torch.randn(1, device=DEV, generator=g)
    sigma = torch.full((A,), -2.9, device=DEV)
    return ln_a, ln_c, w_mu, b_mu, w_v, b_v, sigma


@pytest.mark.parametrize("rows,H", [(4096, 512), (37, 512), (50, 256), (33, 1024)])
@pytest.mark.parametrize("deterministic", [False, True])
@pytest.mark.parametrize("transposed", [False, True], ids=["w_mu", "w_mu_t"])
def test_policy_act_vs_torch(rows, H, deterministic, transposed):
    from puffer_phc_amd import _native as N

    A = 69
    g = torch.Generator(device=DEV).manual_seed(rows + H)
    y = torch.randn((2, rows, H), device=DEV, generator=g) * 2 + 0.3
    ln_a, ln_c, w_mu, b_mu, w_v, b_v, sigma = _heads(H, A, g)
    noise = torch.randn((rows, A), device=DEV, generator=g)
    actions = torch.empty((rows, A), device=DEV)
    mu = torch.empty((rows, A), device=DEV)
    logprob = torch.empty(rows, device=DEV)
    value = torch.empty(rows, device=DEV)
    std_max = 1e-6 if deterministic else float("inf")
    w_mu_t = None
    if transposed:  # the rollout's layout: W_mu^T in a [H, 72] buffer (coalesced reads across actions)
        w_mu_t = torch.zeros((H, 72), device=DEV)[:, :A]
        w_mu_t.copy_(w_mu.t())
    N.policy_act(y, ln_a, ln_c, 1e-5, w_mu, b_mu, w_v, b_v, sigma, noise, actions, logprob, value, mu=mu,
                 std_max=std_max, w_mu_t=w_mu_t)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        F = torch.nn.functional
        ha = F.silu(F.layer_norm(y[0], (H,), ln_a[0], ln_a[1], 1e-5))
        hc = F.silu(F.layer_norm(y[1], (H,), ln_c[0], ln_c[1], 1e-5))
        ref_mu = ha @ w_mu.t() + b_mu
        ref_v = (hc @ w_v.t() + b_v).view(-1)
    finally:
        torch.set_float32_matmul_precision(prev)
    std = torch.exp(sigma).expand_as(ref_mu)
    if deterministic:
        std = torch.clamp(std, max=1e-6)
    probs = torch.distributions.Normal(mu, std, validate_args=False)  # on the kernel's mu: isolates log_prob
    ref_a = mu + std * noise
    torch.testing.assert_close(mu, ref_mu, atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(value, ref_v, atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(actions, ref_a, atol=0, rtol=0)
    ref_lp = probs.log_prob(ref_a).sum(1)
    torch.testing.assert_close(logprob, ref_lp, atol=2e-3 if not deterministic else 5.0, rtol=1e-5)


def test_policy_act_is_deterministic():
    """Identical inputs give identical bits (the rollout graph vs eager equality relies on it)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(5)
    rows, H, A = 2048, 512, 69
    y = torch.randn((2, rows, H), device=DEV, generator=g)
    args = _heads(H, A, g)
    noise = torch.randn((rows, A), device=DEV, generator=g)
    w_mu_t = torch.zeros((H, 72), device=DEV)[:, :A]
    w_mu_t.copy_(args[2].t())
    for wt in (None, w_mu_t):
        outs = []
        for _ in range(2):
            o = (torch.empty((rows, A), device=DEV), torch.empty(rows, device=DEV), torch.empty(rows, device=DEV))
            N.policy_act(y, *args[:2], 1e-5, *args[2:], noise, *o, w_mu_t=wt)
            outs.append(o)
        for a, b in zip(*outs):
            assert torch.equal(a, b)


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


@pytest.mark.parametrize("precision", [torch.float16, torch.bfloat16])
def test_act_rollout_matches_module_path(precision):
    from puffer_phc_amd.policies import PHCPolicy, Policy

    torch.manual_seed(0)
    pol = Policy(PHCPolicy(_Env())).to(DEV)
    with torch.no_grad():
        pol.policy.obs_norm.running_mean.uniform_(-0.5, 0.5)
        pol.policy.obs_norm.running_var.uniform_(0.5, 2.0)
        for m in pol.modules():
            if isinstance(m, torch.nn.Linear):
                m.bias.uniform_(-0.1, 0.1)
    g = torch.Generator(device=DEV).manual_seed(2)
    n = 1024
    obs = torch.randn((n, 934), device=DEV, generator=g) * 2
    noise = torch.randn((n, 69), device=DEV, generator=g)
    act, lp, v = torch.empty((n, 69), device=DEV), torch.empty(n, device=DEV), torch.empty(n, device=DEV)
    with torch.no_grad(), torch.autocast("cuda", dtype=precision):
        assert pol.policy.act_rollout(obs, noise, act, lp, v)
        hidden, _ = pol.policy.encode_observations(obs)
        probs, value = pol.policy.decode_actions(hidden)
    ref_a = probs.loc + probs.scale * noise
    # same trunk GEMMs (bit-identical operands); the heads differ only in fp32 GEMM rounding
    torch.testing.assert_close(act, ref_a, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(v, value.view(-1), atol=1e-4, rtol=1e-4)
    ref_lp = probs.log_prob(act).sum(1)
    torch.testing.assert_close(lp, ref_lp, atol=0.5, rtol=1e-3)
    # the half input path of encode_observations agrees with the fp32 obs path bit for bit
    with torch.no_grad(), torch.autocast("cuda", dtype=precision):
        xh = pol.policy.obs_half_input(obs)
        h1, _ = pol.policy.encode_observations(xh)
        h2, _ = pol.policy.encode_observations(obs)
    assert torch.equal(h1, h2)
