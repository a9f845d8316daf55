"""The PPO minibatch objective (clean_pufferl/core.py:298-352) on the device: one forward and one
backward kernel (phc_ppo.hip) in place of the ~60 elementwise / reduction launches of the
eager expression, with the same math (see the kernel header for the formulas and tie rules).

`ppo_objective` returns the differentiable loss (pg - ent_coef ent + vf_coef v, plus
bound_coef bound only with TrainConfig.bound_loss_grad) and a detached [7] tensor of the logged
means (pg, v, entropy, old_approx_kl, approx_kl, clipfrac, bound loss).  Gradients flow to mu and value only, as in the reference (sigma is a
fixed parameter, the rollout tensors are data)."""

import torch

from .. import _native


class _PPOObjective(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, value, log_sigma, actions, old_logprob, adv, adv_mean_std, old_value, returns, coefs):
        stats, row_coef = _native.ppo_loss_fwd(mu, log_sigma, actions, old_logprob, adv, adv_mean_std, value,
                                               old_value, returns, coefs)
        ctx.save_for_backward(mu, log_sigma, actions, row_coef)
        ctx.coefs = coefs
        ctx.value_shape = value.shape
        tail = stats[1:]
        ctx.mark_non_differentiable(tail)
        return stats[0], tail

    @staticmethod
    def backward(ctx, g_loss, _g_stats):
        mu, log_sigma, actions, row_coef = ctx.saved_tensors
        gmu, gv = _native.ppo_loss_bwd(mu, log_sigma, actions, row_coef, g_loss.float().contiguous(), ctx.coefs)
        return gmu, gv.view(ctx.value_shape), None, None, None, None, None, None, None, None


def ppo_coefs(cfg, soft_bound):
    """phc_ppo_coefs of a TrainConfig.  The bound term enters the differentiable loss only with
    TrainConfig.bound_loss_grad (the reference's bound term is a no-grad constant, see config.py);
    the kernel still reports the minibatch's bound loss in stats[6]."""
    bound = cfg.bound_coef if (cfg.bound_coef > 0 and getattr(cfg, "bound_loss_grad", False)) else 0.0
    return _native.ppo_coefs(cfg.clip_coef, cfg.vf_clip_coef, cfg.vf_coef, cfg.ent_coef, bound, soft_bound,
                             cfg.clip_vloss)


def ppo_objective(mu, value, log_sigma, actions, old_logprob, adv, adv_mean, adv_std, old_value, returns, cfg,
                  soft_bound):
    coefs = ppo_coefs(cfg, soft_bound)
    if adv_std is None:  # adv_mean is already the device [2] (mean, std) pair
        ms = adv_mean
    else:
        ms = torch.stack([torch.as_tensor(adv_mean, dtype=torch.float32, device=mu.device).reshape(()),
                          torch.as_tensor(adv_std, dtype=torch.float32, device=mu.device).reshape(())])
    f = lambda t: t.detach().float().contiguous().reshape(-1)  # noqa: E731
    return _PPOObjective.apply(mu.float().contiguous(), value.float().reshape(-1), log_sigma.detach().float(),
                               actions.detach().float().contiguous(), f(old_logprob), f(adv), ms, f(old_value),
                               f(returns), coefs)
