"""The PPO minibatch as one autograd node on the device (R19 + R21).

forward: MFMA twin trunks (twin_mlp.mfma_trunk_forward) -> phc_tail_ln_fwd (LayerNorm + SiLU of
both trunks, the critic's value head) -> the fp32 mu head (phc_mu_head_fwd) -> the PPO objective
kernels (phc_ppo_loss_fwd).  backward: phc_ppo_loss_bwd (d mu, d value) -> d h_a = dmu W_mu and the
split-K W_mu gradient (phc_mu_head_dgrad / _wgrad, fp32-input MFMA) -> phc_tail_ln_bwd (LayerNorm +
SiLU backward of both trunks; dy in the trunk's operand type; every remaining tail gradient as
per-block column sums) -> the trunk backward.  Same math as PHCPolicy.forward_train + ppo_objective (reference:
policies/phc_policy.py:16-61, clean_pufferl/core.py:298-352) without the ~30 elementwise, fill,
copy and reduction launches autograd runs between those pieces; the unfused path stays for fp32
storage and other shapes."""

import os

import torch

from .. import _native as N
from . import twin_mlp
from .twin_mlp import _compute_dtype, _use_mfma, direct_grads_bound, mfma_trunk_backward, mfma_trunk_forward


MU_WGRAD_SPLITS = int(os.environ.get("PHC_MU_WGRAD_SPLITS", "128"))  # row chunks of the mu-head weight gradient
# forward / input gradient of the mu head on phc_mu_head_fwd / _dgrad (1, default) or the library
# GEMMs (0): the bf16-x3 MFMA kernels (three-way bf16 operand splits, fp32-class products; see
# phc_head.hip) against the library's fp32 GEMMs, per 32768-row minibatch (tools/mu_head_probe.py);
# the weight gradient runs on phc_mu_head_wgrad either way (39 us + its partial sum riding in
# phc_reduce_into, library 140 us)
MU_HEAD_KERNELS = os.environ.get("PHC_MU_HEAD_KERNELS", "1") == "1"


def _aligned(w):
    """w, or a 16-byte aligned copy (phc_mu_head_fwd reads w with 16-B loads; a parameter may be a
    view into a flat buffer at any 4-byte offset)."""
    w = w.contiguous()
    return w if w.data_ptr() % 16 == 0 else w.clone(memory_format=torch.contiguous_format)


class FusedPPOLossFn(torch.autograd.Function):
    """apply(x, weights, (ln_eps, log_sigma, coefs), data, n_trunk, *trunk_params, *tail_params)
    -> (loss, stats [7]); tail_params = actor LN (w, b), critic LN (w, b), mu head (w, b), value
    head (w, b); data = (actions, old_logprob, adv, adv_mean_std, old_value, returns)."""

    @staticmethod
    def forward(ctx, x, weights, cfg, data, n_trunk, *params):
        eps, log_sigma, coefs, ctx.store_grads, stats_acc = cfg
        y, saved = mfma_trunk_forward(x, weights, True)
        la_w, la_b, lc_w, lc_b, mu_w, mu_b, v_w, v_b = [p.detach() for p in params[n_trunk:]]
        actions, old_logprob, adv, adv_ms, old_value, returns = data
        with torch.no_grad(), torch.autocast("cuda", enabled=False):
            tail = N.TailLN(y, (la_w, la_b), (lc_w, lc_b), eps, v_w, v_b)
            h_a, value = tail.forward()
            if MU_HEAD_KERNELS:
                mu = N.mu_head_fwd(h_a, _aligned(mu_w), mu_b)  # fp32 head, as HeadLinearFn
            else:
                mu = torch.addmm(mu_b, h_a, mu_w.t())
            stats, row_coef = N.ppo_loss_fwd(mu, log_sigma, actions, old_logprob, adv, adv_ms, value, old_value,
                                             returns, coefs, stats_acc=stats_acc)
        ctx.saved, ctx.tail, ctx.params, ctx.n_trunk = saved, tail, params, n_trunk
        ctx.ppo = (mu, log_sigma, actions, row_coef, coefs)
        st = stats[1:]
        ctx.mark_non_differentiable(st)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        return stats[0], st

    @staticmethod
    def backward(ctx, g_loss, _g_stats):
        saved, tail, params, n = ctx.saved, ctx.tail, ctx.params, ctx.n_trunk
        mu, log_sigma, actions, row_coef, coefs = ctx.ppo
        la_w, la_b, lc_w, lc_b, mu_w, mu_b, v_w, v_b = params[n:]
        direct = direct_grads_bound(params)
        with torch.no_grad(), torch.autocast("cuda", enabled=False):
            gmu, gv = N.ppo_loss_bwd(mu, log_sigma, actions, row_coef, g_loss.float().contiguous(), coefs)
            if MU_HEAD_KERNELS:
                dh_a = N.mu_head_dgrad(gmu, mu_w.detach().contiguous())
            else:
                dh_a = torch.mm(gmu, mu_w.detach())
            dy, part, lay = tail.backward(dh_a, gmu, gv, saved.xc.dtype)
            A, H = gmu.shape[1], tail.H
            # direct mode: the tail's per-block partial rows go to phc_reduce_into as [parts, 1, w]
            # sources (summed in the same launch that writes them into .grad); otherwise summed here
            sums = None if direct else part.sum(0)

            def seg(key, width):
                o = lay[key]
                return part[:, None, o:o + width] if direct else sums[o:o + width]

            tail_srcs = [(seg("gamma", 2 * H), (la_w, lc_w)), (seg("beta", 2 * H), (la_b, lc_b)),
                         (seg("b_mu", A), (mu_b,)), (seg("w_value", H), (v_w,)), (seg("b_value", 1), (v_b,))]
            tail_srcs = [(src[..., k * p.numel():(k + 1) * p.numel()], p) for src, ps in tail_srcs
                         for k, p in enumerate(ps)]
            db6 = part[:, lay["b6"]:lay["b6"] + 2 * H] if direct else sums[lay["b6"]:lay["b6"] + 2 * H]
            if direct:
                jobs = [(N.mu_head_wgrad_parts(gmu, tail.h_actor, MU_WGRAD_SPLITS), mu_w.grad)]
                jobs += [(s, p.grad) for s, p in tail_srcs]
                store = ctx.store_grads
                if twin_mlp.GRAD_READY is not None:  # data parallel: the tail's all-reduce starts now
                    N.reduce_into(jobs, accumulate=not store)
                    twin_mlp.GRAD_READY(params[n:])
                    jobs = None
                # single-GPU: the tail's sums ride along with the trunk's final reduce launch
                mfma_trunk_backward(saved, dy, db6, params[:n], True, extra_jobs=jobs, store=store)
                grads = [None] * len(params)
            else:
                g_mu_w = N.mu_head_wgrad_parts(gmu, tail.h_actor, MU_WGRAD_SPLITS).sum(0)
                tg = {id(p): s.reshape(p.shape).clone() for s, p in tail_srcs}
                tg[id(mu_w)] = g_mu_w
                trunk = mfma_trunk_backward(saved, dy, db6.clone(), params[:n], False)
                grads = list(trunk) + [tg[id(p)] for p in params[n:]]
        ctx.saved = ctx.tail = ctx.ppo = None
        return (None, None, None, None, None, *grads)


def fused_ppo_supported(policy, obs):
    """The fused minibatch needs the MFMA trunks (f16 / bf16 autocast), the half-precision GEMM
    operand as input, hidden 512 and at most 72 actions."""
    if not (getattr(policy, "fused", False) and getattr(policy, "fused_ln", False) and obs.is_cuda):
        return False
    dt = _compute_dtype()
    if dt == torch.float32 or obs.dtype != dt or not _use_mfma(policy._twin, dt):
        return False
    h = policy._head
    return (policy.actor_mlp[h].weight.shape[0] == N.TAIL_HIDDEN
            and policy.mu[0].weight.shape[0] <= N.TAIL_MAX_ACTIONS)


def fused_ppo_loss(policy, obs, actions, old_logprob, adv, adv_mean_std, old_value, returns, coefs,
                   store_grads=False, stats_acc=None):
    """(loss, stats [7]: pg, v, entropy, old_approx_kl, approx_kl, clipfrac, bound) of one
    minibatch; the backward writes every policy gradient.  store_grads: with the gradients bound
    to a flat buffer (direct mode), the backward stores them instead of adding to them, so the
    buffer need not be zeroed first (every parameter of the policy has exactly one writer).  stats_acc
    (device float64 [7], optional) += the stats in the objective's own reduce launch."""
    h = policy._head
    la, lc = policy.actor_mlp[h], policy.critic_mlp[h]
    vh, mh = policy.critic_mlp[h + 2], policy.mu[0]
    tail = [la.weight, la.bias, lc.weight, lc.bias, mh.weight, mh.bias, vh.weight, vh.bias]
    trunk = policy._twin.params()
    f = lambda t: t.detach().float().contiguous().reshape(-1)  # noqa: E731
    data = (actions.detach().float().contiguous(), f(old_logprob), f(adv), adv_mean_std.detach().float().contiguous(),
            f(old_value), f(returns))
    cfg = (la.eps, policy.sigma.detach().float().contiguous().reshape(-1), coefs, bool(store_grads), stats_acc)
    return FusedPPOLossFn.apply(obs, policy._twin, cfg, data, len(trunk), *trunk, *tail)
