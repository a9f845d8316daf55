"""AMP discriminator (R22) on the hand-written MFMA GEMM.

DiscriminatorPolicy.discriminate (puffer_phc/policies/discriminator_policy.py:72-79) is
RunningNorm(1960) -> Linear(1960, 1024) + ReLU -> Linear(1024, H) + ReLU -> Linear(H, 1), used
twice per PPO iteration by clean_pufferl (core.py:229-242: the adversarial reward
-log(max(1 - sigmoid(logit), 1e-4)) of every collected row, no grad; core.py:336-347: the BCE
loss of agent / replay rows against demo rows, with gradients).  Here, in the f16 / bf16 modes:

  input   RunningNorm + rounding into the first GEMM's operand, the rows gathered straight from
          the experience buffers through their minibatch index (phc_obs_half, one launch per
          source), K zero-padded 1960 -> 1984
  layers  phc_twin_gemm with the BIAS_RELU epilogue (fp32 accumulate, the ReLU output rounded once
          into the next operand), backward with RELU_GRAD (relu' read from the ReLU output, as
          torch's threshold_backward) + fused bias-gradient column sums, weight gradients on the
          transposed-read MFMA kernel (phc_weight_grad, split-K) summed by phc_reduce_into
  head    phc_disc_head_fwd / _bwd: the H -> 1 dot product per row in fp32 (+ the adversarial
          reward in the same launch), its backward producing the second layer's input gradient

Parameters stay the reference's nn.Linear modules (state-dict keys _disc_mlp.0 / .2,
_disc_logits); the half-precision weight copies are a cache keyed on parameter versions and the
optimizer generation (weight_cache.py), refreshed by one phc_pack_weights launch.
"""

import torch

from .. import _native as N
from .twin_mlp import _compute_dtype, _pad64, _wgrad_splits, _wgrad_tiles
from . import weight_cache
from .weight_cache import cache_key, layout_key


class DiscOperands:
    def __init__(self):
        self.key = self.plan_key = self.plan = None
        self.w1 = self.w2 = self.w2t = None
        self.b1 = self.b2 = None


def _linears(pol):
    return pol._disc_mlp[0], pol._disc_mlp[2], pol._disc_logits


def disc_params(pol):
    l1, l2, l3 = _linears(pol)
    return [l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias]


def mfma_disc_supported(pol, dtype):
    """The MFMA path serves f16 / bf16 with hidden widths % 64 == 0 and a head width <= 1024."""
    if dtype not in (torch.float16, torch.bfloat16) or not getattr(pol, "use_amp_obs", False):
        return False
    l1, l2, l3 = _linears(pol)
    return l1.weight.shape[0] % 64 == 0 and l2.weight.shape[0] % 64 == 0 and l2.weight.shape[0] <= 1024 \
        and l3.weight.shape[0] == 1 and l1.weight.is_cuda


def disc_operands(pol, dtype):
    l1, l2, _ = _linears(pol)
    ps = disc_params(pol)
    key = cache_key(dtype, ps)
    ops = pol.__dict__.setdefault("_disc_ops", DiscOperands())
    if ops.key == key:
        return ops
    with torch.no_grad():
        n1, k1 = l1.weight.shape
        fresh = ops.w1 is None or ops.w1.dtype != dtype
        if fresh:
            dev = l1.weight.device
            ops.w1 = torch.zeros((n1, _pad64(k1)), dtype=dtype, device=dev)
            ops.w2 = torch.empty(l2.weight.shape, dtype=dtype, device=dev)
            ops.w2t = torch.empty((l2.weight.shape[1], l2.weight.shape[0]), dtype=dtype, device=dev)
        lk = layout_key(dtype, ps)
        if fresh or ops.plan_key != lk:
            ops.plan_jobs = [(l1.weight.detach(), ops.w1[:, :k1], None), (l2.weight.detach(), ops.w2, ops.w2t)]
            ops.plan = N.PackPlan(ops.plan_jobs)
            ops.plan_key = lk
            # key of the copies: the two weights (the biases are read in place)
            ops.fresh_dtype, ops.fresh_params = dtype, ps
            weight_cache.register_plan(ops)
        ops.plan.run()
        ops.b1 = l1.bias.detach().float().contiguous()
        ops.b2 = l2.bias.detach().float().contiguous()
    ops.key = key
    return ops


def disc_input(pol, sources, dtype):
    """[R, pad64(1960)] operand of the first layer: RunningNorm of every source's rows (a source is
    (amp_obs [*, 1960] fp32, row index int64 [n] or None = all rows)), concatenated in order."""
    norm = pol.amp_obs_norm
    K0 = norm.running_mean.shape[1]
    Kp = _pad64(K0)
    counts = [(idx.numel() if idx is not None else src.shape[0]) for src, idx in sources]
    x = torch.empty((sum(counts), Kp), dtype=dtype, device=norm.running_mean.device)
    r0 = 0
    for (src, idx), n in zip(sources, counts):
        if n:
            N.obs_half(src, norm.running_mean, norm.running_var, norm.epsilon, norm.clip, x[r0:r0 + n],
                       idx.contiguous() if idx is not None else None)
        r0 += n
    return x


def _forward(ops, l3, x):
    """(h1, h2) of the two ReLU layers on the MFMA GEMM."""
    R = x.shape[0]
    n1, n2 = ops.w1.shape[0], ops.w2.shape[0]
    h1 = torch.empty((R, n1), dtype=x.dtype, device=x.device)
    N.twin_gemm(x, ops.w1, N.EPI_BIAS_RELU, h1, (1, n1), bias=ops.b1)
    h2 = torch.empty((R, n2), dtype=x.dtype, device=x.device)
    N.twin_gemm(h1, ops.w2, N.EPI_BIAS_RELU, h2, (1, n2), bias=ops.b2)
    return h1, h2


def _weight_grad_sum(g, z, n_valid=None):
    """dW = g^T z [m, n_valid] fp32 over all rows (split-K MFMA partials + one reduce)."""
    R = g.shape[0]
    if R % 64:
        # phc_weight_grad reduces whole 64-row chunks: zero rows (which add nothing to g^T z) pad
        # a ragged row count, e.g. AMP training with num_envs not a multiple of 64
        Rp = -(-R // 64) * 64
        gp = torch.zeros((Rp, g.shape[1]), dtype=g.dtype, device=g.device)
        zp = torch.zeros((Rp, z.shape[1]), dtype=z.dtype, device=z.device)
        gp[:R].copy_(g)
        zp[:R].copy_(z)
        g, z, R = gp, zp, Rp
    S = _wgrad_splits(_wgrad_tiles(g[None], z[None]), R, g.device)
    part = N.weight_grad(g, z, S)  # [S, 1, m, n]
    nv = n_valid or part.shape[3]
    out = torch.empty((part.shape[2], nv), dtype=torch.float32, device=g.device)
    N.reduce_into([(part[:, 0, :, :nv], out)], accumulate=False)
    return out


class DiscMlpFn(torch.autograd.Function):
    """logits [R] fp32 of the discriminator on the operand x [R, Kp] (disc_input)."""

    @staticmethod
    def forward(ctx, x, ops, l3, *params):
        with torch.autocast("cuda", enabled=False):
            h1, h2 = _forward(ops, l3, x)
            logits = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
            N.disc_head_fwd(h2, l3.weight.detach(), l3.bias.detach(), logits=logits)
        ctx.save_for_backward(x, h1, h2)
        ctx.ops, ctx.l3 = ops, l3
        ctx.k0 = params[0].shape[1]
        return logits

    @staticmethod
    def backward(ctx, gl):
        x, h1, h2 = ctx.saved_tensors
        ops, l3 = ctx.ops, ctx.l3
        with torch.autocast("cuda", enabled=False):
            gl = gl.float().contiguous()
            n1, n2 = h1.shape[1], h2.shape[1]
            g2 = torch.empty_like(h2)
            parts = N.disc_head_bwd(h2, l3.weight.detach(), gl, g2)  # [blocks, 2 n2 + 4]
            dw3 = torch.empty((1, n2), dtype=torch.float32, device=x.device)
            db2 = torch.empty(n2, dtype=torch.float32, device=x.device)
            db3 = torch.empty(1, dtype=torch.float32, device=x.device)
            N.reduce_into([(parts[:, None, :n2], dw3), (parts[:, None, n2:2 * n2], db2),
                           (parts[:, None, 2 * n2:2 * n2 + 1], db3)], accumulate=False)
            dw2 = _weight_grad_sum(g2, h1)
            g1 = torch.empty_like(h1)
            db1 = torch.empty(n1, dtype=torch.float32, device=x.device)
            N.twin_gemm(g2, ops.w2t, N.EPI_RELU_GRAD, g1, (1, n1), aux=h1, bias_grad=db1)
            dw1 = _weight_grad_sum(g1, x, ctx.k0)
        return None, None, None, dw1, db1, dw2, db2, dw3, db3


def discriminate_rows(pol, sources):
    """Discriminator logits [R, 1] of the concatenated row sources (see disc_input) on the MFMA
    path, differentiable w.r.t. the discriminator parameters."""
    dt = _compute_dtype()
    ops = disc_operands(pol, dt)
    x = disc_input(pol, sources, dt)
    return DiscMlpFn.apply(x, ops, pol._disc_logits, *disc_params(pol)).unsqueeze(1)


@torch.no_grad()
def adversarial_reward(pol, sources, out=None):
    """-log(max(1 - sigmoid(disc(rows)), 1e-4)) [R] fp32 (clean_pufferl/core.py:229-242) in one
    pass: input, two GEMMs, head + reward."""
    dt = _compute_dtype()
    ops = disc_operands(pol, dt)
    x = disc_input(pol, sources, dt)
    with torch.autocast("cuda", enabled=False):
        _, h2 = _forward(ops, pol._disc_logits, x)
        if out is None:
            out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        l3 = pol._disc_logits
        N.disc_head_fwd(h2, l3.weight.detach(), l3.bias.detach(), reward=out)
    return out
