"""Fused PPO objective (clean_pufferl/ppo_loss.py, phc_ppo.hip) vs the reference's eager
expression (clean_pufferl/core.py:298-352) on the same policy and minibatch (needs an MI355X).

Tolerance: loss and logged statistics within rel 1e-5 (float32 reductions in a different
order; the KL estimates, means of ~1e-2 terms, within 1e-4); parameter gradients within rel. L2
5e-5 (both paths share the same twin-trunk backward; d loss / d mu = ratio (a - mu) / sigma^2
with sigma^2 = 3e-3 is formed in a different association order than autograd's chain).  The test data keep every ratio >= 5e-3 away from the clip edges, so
float32 rounding cannot flip a row between the clipped and unclipped branches."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


def _eager(pol, policy, obs, atn, old_lp, adv, val, ret, cfg):
    # bound term: with cfg.bound_loss_grad a per-minibatch differentiable term; by default the
    # reference's no-grad constant, which train() adds outside the objective (core.py:349-350)
    _, newlogprob, entropy, newvalue = policy(obs, action=atn)
    logratio = newlogprob - old_lp
    ratio = logratio.exp()
    old_kl = (-logratio).mean()
    kl = ((ratio - 1) - logratio).mean()
    clipfrac = ((ratio - 1.0).abs() > cfg.clip_coef).float().mean()
    a = (adv - adv.mean()) / (adv.std() + 1e-8)
    pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)).mean()
    v = newvalue.view(-1)
    v_clipped = val + torch.clamp(v - val, -cfg.vf_clip_coef, cfg.vf_clip_coef)
    v_loss = torch.max((v - ret) ** 2, (v_clipped - ret) ** 2).mean()
    ent = entropy.mean()
    loss = pg - cfg.ent_coef * ent + v_loss * cfg.vf_coef
    if cfg.bound_loss_grad:
        loss = loss + pol.mean_bound_loss * cfg.bound_coef
    stats = torch.stack([pg, v_loss, ent, old_kl, kl, clipfrac, pol.mean_bound_loss])
    return loss, stats.detach()


@pytest.mark.parametrize("bound_grad", [False, True])
def test_fused_objective_matches_eager(bound_grad):
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_objective
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(_Env(), hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    pol = policy.policy
    with torch.no_grad():
        pol.mu[0].weight.mul_(100.0)  # push some |mu| past the 0.9 soft bound
    cfg = TrainConfig(ent_coef=0.01, bound_loss_grad=bound_grad)
    g = torch.Generator(device=DEV).manual_seed(1)
    M = 4096
    obs = torch.randn((M, 934), device=DEV, generator=g)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    with torch.no_grad():
        mu0, v0 = pol.forward_train(obs)  # the same mu both paths compute below
    torch.set_float32_matmul_precision(prev)
    atn = mu0 + 0.05 * torch.randn(mu0.shape, device=DEV, generator=g)
    sg = torch.exp(pol.sigma)
    lp0 = (-((atn - mu0) ** 2) / (2 * sg ** 2) - sg.log() - 0.5 * np.log(2 * np.pi)).sum(1)
    # log-ratios below, inside (the max() tie) and above [1 - clip, 1 + clip] (clip 0.01), each
    # >= 5e-3 away from the clip edges so float32 summation order cannot flip a row's branch
    pick = lambda vals: torch.tensor(vals, device=DEV)[torch.randint(len(vals), (M,), device=DEV, generator=g)]  # noqa
    old_lp = lp0 - pick([-0.05, -0.02, 0.0, 0.004, 0.02, 0.05])
    adv = torch.randn(M, device=DEV, generator=g)
    val = v0.view(-1) - pick([-0.5, -0.05, 0.05, 0.5])  # value clip 0.2: both branches
    ret = val + torch.randn(M, device=DEV, generator=g)

    torch.set_float32_matmul_precision("highest")
    try:
        policy.zero_grad(set_to_none=True)
        pol.fused = True
        loss_e, st_e = _eager(pol, policy, obs, atn, old_lp, adv, val, ret, cfg)
        loss_e.backward()
        ge = {n: p.grad.clone() for n, p in policy.named_parameters() if p.grad is not None}

        policy.zero_grad(set_to_none=True)
        mu, value = pol.forward_train(obs)
        loss_f, st_f = ppo_objective(mu, value, pol.sigma, atn, old_lp, adv, adv.mean(), adv.std(), val, ret, cfg,
                                     pol.soft_bound)
        loss_f.backward()
        gf = {n: p.grad.clone() for n, p in policy.named_parameters() if p.grad is not None}
    finally:
        torch.set_float32_matmul_precision(prev)

    clipped = ((st_e[5] > 0) & (st_e[5] < 1)).item()
    assert clipped, "test data must exercise both clipped and unclipped rows"
    assert st_e[6] > 0, "test data must exercise the bound loss"
    torch.testing.assert_close(loss_f, loss_e.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st_f[[0, 1, 2, 5, 6]], st_e[[0, 1, 2, 5, 6]], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st_f[3:5], st_e[3:5], rtol=1e-4, atol=2e-6)  # KL estimates: means of ~1e-2
    assert set(gf) == set(ge)
    for k in ge:
        err = float((gf[k] - ge[k]).norm() / ge[k].norm().clamp_min(1e-30))
        assert err < 5e-5, (k, err)
