"""The headline path at BASELINE configs[2] (C3) size, pinned to fp32 (needs an MI355X).

bench.py times, per PPO minibatch, exactly this: fused_ppo_loss (policies/fused_ppo.py) at the
reference's full PHCPolicy widths (934 -> 2048-1536-1024-1024-512-512, LayerNorm+SiLU, mu 512->69,
value 512->1) over 32768 rows, f16 MFMA trunk GEMMs with fp32 accumulation, the grouped
weight-gradient launch over all 32768 rows, the bf16-x3 mu-head kernels, the tail LayerNorm
kernels and the PPO objective kernels, gradients stored straight into the flat buffer, under the
fp16 loss scale the optimizer starts with (2^16).

Reference math: puffer_phc/policies/phc_policy.py:22-61 (the unfused nn.Sequential policy) and
puffer_phc/clean_pufferl/core.py:298-333 (ratio, per-minibatch advantage normalisation, clipped
policy loss, clipped value loss, entropy), evaluated two ways in torch:
  * exact fp32 (matmul precision "highest"): the truth;
  * an exact TF32 emulation of every nn.Linear (operands rounded to 10 stored mantissa bits, fp32
    products and sums): the arithmetic the reference itself runs on its GPUs
    (torch.set_float32_matmul_precision("high"), core.py:38).
Bound (the same rule as test_gpu_twin_mlp.test_fp16_operands_match_tf32_error, now at C3 size):
the headline path's error against exact fp32 is at most 1.5x the TF32 emulation's error for the
per-row outputs (mu, value) and every parameter gradient (+1e-7 absolute floor on the relative
error); the scalar loss and logged statistics (single sums, whose rounding errors cancel at random)
within 3x the TF32 error or 1e-6 relative.  Log-ratios are placed >= 0.19 from the clip edges (clip 0.01) and value deltas >= 0.15
from the value clip (0.2), so no row's branch depends on rounding: clipfrac must match exactly.

The second test runs one whole C3 iteration (4096 envs, 131072 rows, 16 minibatches, fp16 +
dynamic loss scaling) and asserts finiteness and that the loss scaler skipped no step.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LOG2PI = 0.5 * np.log(2 * np.pi)
ROWS = 32768
LOSS_SCALE = 2.0 ** 16


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


class _TF32Linear(torch.autograd.Function):
    @staticmethod
    def _r(t):
        i = t.contiguous().view(torch.int32)
        return ((i + 0x1000) & ~0x1FFF).view(torch.float32)

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _TF32Linear._r(x) @ _TF32Linear._r(w).t() + b

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        r = _TF32Linear._r
        g2 = gy.reshape(-1, gy.shape[-1])
        return (r(g2) @ r(w)).view(x.shape), r(g2).t() @ r(x.reshape(-1, x.shape[-1])), g2.sum(0)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _reference_loss(policy, obs, atn, old_lp, adv, ms, val, ret, cfg):
    """core.py:298-333 on the unfused policy (fp32 modules)."""
    _, newlp, entropy, newvalue = policy(obs, action=atn)
    logratio = newlp - old_lp
    ratio = logratio.exp()
    with torch.no_grad():
        old_kl = (-logratio).mean()
        kl = ((ratio - 1) - logratio).mean()
        clipfrac = ((ratio - 1.0).abs() > cfg.clip_coef).float().mean()
    a = (adv - ms[0]) / (ms[1] + 1e-8)
    pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)).mean()
    nv = newvalue.view(-1)
    v_unc = (nv - ret) ** 2
    v_clp = (val + torch.clamp(nv - val, -cfg.vf_clip_coef, cfg.vf_clip_coef) - ret) ** 2
    v = torch.max(v_unc, v_clp).mean()
    ent = entropy.mean()
    loss = pg - cfg.ent_coef * ent + v * cfg.vf_coef
    return loss, torch.stack([pg, v, ent, old_kl, kl, clipfrac]).detach()


def test_headline_minibatch_matches_fp32_within_tf32_error():
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss, fused_ppo_supported
    from puffer_phc_amd.policies.pufferl_policy import Linear

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(_Env())).to(DEV)  # the reference's full widths
    pol = policy.policy
    cfg = TrainConfig()
    g = torch.Generator(device=DEV).manual_seed(11)
    with torch.no_grad():
        pol.obs_norm.running_mean.uniform_(-0.5, 0.5, generator=g)
        pol.obs_norm.running_var.uniform_(0.5, 2.0, generator=g)
    obs = torch.randn((ROWS, 934), device=DEV, generator=g) * 2
    params = [(n, q) for n, q in policy.named_parameters() if q.requires_grad]
    prev = torch.get_float32_matmul_precision()
    orig = Linear.forward
    try:
        torch.set_float32_matmul_precision("highest")
        pol.fused = False
        with torch.no_grad():
            h, _ = pol.encode_observations(obs)
            mu0 = pol.mu(h).float()
            v0 = pol.critic_mlp(pol.obs_pointer).float().view(-1)
        atn = mu0 + 0.05 * torch.randn(mu0.shape, device=DEV, generator=g)
        sg = torch.exp(pol.sigma.detach())
        lp0 = (-((atn - mu0) ** 2) / (2 * sg ** 2) - sg.log() - LOG2PI).sum(1)
        pick = lambda vals: torch.tensor(vals, device=DEV)[torch.randint(len(vals), (ROWS,), device=DEV, generator=g)]  # noqa
        old_lp = lp0 - pick([-0.5, -0.2, 0.2, 0.5])  # log-ratio 0.19+ away from log(1 +- 0.01)
        adv = torch.randn(ROWS, device=DEV, generator=g)
        val = v0 - pick([-0.5, -0.05, 0.05, 0.5])  # 0.15 from the value clip edge (0.2)
        ret = val + torch.randn(ROWS, device=DEV, generator=g)
        ms = torch.stack([adv.mean(), adv.std()])

        def reference(tf32):
            policy.zero_grad(set_to_none=True)
            Linear.forward = (lambda self, x: _TF32Linear.apply(x, self.weight, self.bias)) if tf32 else orig
            loss, st = _reference_loss(policy, obs, atn, old_lp, adv, ms, val, ret, cfg)
            loss.backward()
            with torch.no_grad():
                h, _ = pol.encode_observations(obs)
                out = (pol.mu(h).float(), pol.critic_mlp(pol.obs_pointer).float().view(-1))
            Linear.forward = orig
            return loss.detach(), st, {n: q.grad.detach().clone() for n, q in params}, out

        exact = reference(False)
        tf32 = reference(True)
        rows = (exact[3], tf32[3])
    finally:
        Linear.forward = orig
        torch.set_float32_matmul_precision(prev)
        pol.fused = True
    assert _rel(tf32[0], exact[0]) > 0, "the TF32 emulation must be in effect"

    # the headline path: FlatGrads-bound gradients stored by the fused backward
    policy.zero_grad(set_to_none=True)
    fg = FlatGrads([q for _, q in params], order=pol.grad_ready_order())
    fg.fill_grads_(float("nan"))  # every gradient must be written
    with torch.autocast("cuda", dtype=torch.float16):
        xh = pol.obs_half_input(obs)
        assert fused_ppo_supported(pol, xh)
        loss, st = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, ppo_coefs(cfg, pol.soft_bound),
                                  store_grads=True)
    (loss * LOSS_SCALE).backward()
    torch.cuda.synchronize()
    got = {n: q.grad.detach() / LOSS_SCALE for n, q in params}
    # every gradient view of the flat buffer was written (the 64-B alignment gaps between them hold no
    # gradient and keep the fill)
    assert all(bool(torch.isfinite(q.grad).all()) for _, q in params)

    # per-row outputs (mu, value: 32768 x 69 and 32768 values) and every parameter gradient: the
    # 1.5x rule; the scalar losses / statistics are single sums whose errors cancel at random, so
    # one scalar's error ratio is noise: 3x the TF32 error, or fp32 rounding (1e-6 relative)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        mu_h, v_h = pol.forward_train(xh)
    vec = {"mu": (_rel(mu_h, rows[0][0]), _rel(rows[1][0], rows[0][0])),
           "value": (_rel(v_h.view(-1), rows[0][1]), _rel(rows[1][1], rows[0][1]))}
    for n in exact[2]:
        vec[n] = (_rel(got[n], exact[2][n]), _rel(tf32[2][n], exact[2][n]))
    bad = {k: v for k, v in vec.items() if v[0] > 1.5 * v[1] + 1e-7}
    assert not bad, bad
    sca = {"loss": (_rel(loss.detach(), exact[0]), _rel(tf32[0], exact[0]))}
    for i, name in enumerate(("pg", "v", "entropy", "old_kl", "kl")):
        sca[name] = (_rel(st[i], exact[1][i]), _rel(tf32[1][i], exact[1][i]))
    bad = {k: v for k, v in sca.items() if v[0] > max(3.0 * v[1], 1e-6)}
    assert not bad, bad
    assert float(st[5]) == float(exact[1][5]) == float(tf32[1][5])  # clipfrac: same branches


def test_c3_iteration_finite_no_skipped_steps():
    """One whole PPO iteration at C3 (4096 envs, batch 131072, minibatch 32768, 4 epochs, fp16
    with dynamic loss scaling) on the bench's workload: finite losses, no skipped optimizer step,
    every trained parameter finite and moved."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(4096, 60, 300, seed=1000, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    del q, t
    env = PHCPufferEnv(EnvConfig(num_envs=4096, seed=0), motion_data=packed)
    env.reset()
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env)).to(DEV)
    cfg = TrainConfig(checkpoint_interval=10 ** 9, total_timesteps=10 ** 15)
    assert (cfg.batch_size, cfg.minibatch_size, cfg.update_epochs, cfg.precision) == (131072, 32768, 4, "fp16")
    comps, info, util = clean_pufferl.create("c3", cfg, env.cfg, env, policy)
    before = {k: v.detach().clone() for k, v in policy.named_parameters() if v.requires_grad}
    for _ in range(2):
        clean_pufferl.evaluate(comps, info)
        policy.policy.update_obs_rms(comps.experience.obs)
        losses = clean_pufferl.train(comps, info, util)
        assert np.isfinite([losses.policy_loss, losses.value_loss, losses.approx_kl, losses.old_approx_kl,
                            losses.before_clip_grad_norm, losses.explained_variance]).all()
    assert info.global_step >= 2 * 131072
    assert int(comps.skipped_steps) == 0
    for k, v in policy.named_parameters():
        if v.requires_grad:
            assert torch.isfinite(v).all(), k
            assert not torch.equal(before[k], v.detach()), k
