"""Twin actor/critic trunks of PHCPolicy on MI355X (R19/R21).

PHCPolicy (puffer_phc/policies/phc_policy.py:10-61) runs two 6-layer SiLU MLPs of identical
shape over the same normalised observation.  Here they run side by side: the shared input
goes through ONE GEMM against the stacked first-layer weights ([2*2048, 934]), layers 2-6 are
batched GEMMs over the two trunks ([2, M, K] x [2, K, N]), and every bias-add / SiLU /
SiLU-backward / bias-gradient between the GEMMs is one fused HIP kernel (phc_bias_act_fwd,
phc_act_bwd).  Parameters stay the reference's nn.Linear modules (same state-dict keys); the
stacked weights are a cache in the GEMM dtype, rebuilt when a parameter's version or the
optimizer generation changes (weight_cache.py: after each optimizer step).

GEMM arithmetic follows the autocast context: fp32 storage with torch's "high" matmul
precision (hipBLASLt xf32) outside autocast, fp16 / bf16 operands inside.  In the half-precision
modes only the GEMM OPERANDS are rounded: every GEMM accumulates and writes fp32, the epilogues
compute in fp32 from those outputs and round once, when they write the next GEMM's operand
(activations forward, activation gradients backward), and bias / weight gradients are fp32.
The pre-activations saved for the SiLU backward are kept in the operand type on the MFMA path,
as torch.autocast keeps them (PRE_HALF).
With fp16 operands this is TF32's arithmetic (an 11-bit significand per operand, fp32 products
and sums; the reference sets torch.set_float32_matmul_precision("high"),
clean_pufferl/core.py:38) with fp16's exponent range, which dynamic loss scaling covers for the
gradients.  The reference's unfused path (nn.Sequential of Linear/SiLU) is what the tests
compare against.
"""

import os

import torch

from .. import _native as N
from . import weight_cache
from .weight_cache import cache_key, layout_key


def _compute_dtype():
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return torch.float32


def _bmm(a, b, out_fp32=False):
    """Batched GEMM over the two trunks.  bf16 runs as one GEMM per trunk: hipBLASLt's batched
    bf16 solution for [2, 32768, 2048] x [2, 2048, 1536] (ROCm 7.0 torch wheel) faults the GPU
    (illegal address; tools/bf16_probe.py), the per-trunk 2-D GEMMs do not."""
    out_dt = torch.float32 if (out_fp32 and a.dtype != torch.float32) else None
    if a.dtype == torch.bfloat16:
        out = torch.empty((a.shape[0], a.shape[1], b.shape[2]), dtype=out_dt or a.dtype, device=a.device)
        for g in range(a.shape[0]):
            if out_dt is None:
                torch.mm(a[g], b[g], out=out[g])
            else:
                torch.mm(a[g], b[g], out_dtype=out_dt, out=out[g])
        return out
    if out_dt is not None:
        return torch.bmm(a, b, out_dtype=out_dt)
    return torch.bmm(a, b)


def _split_k(m, n, k, groups):
    """Row chunks for a weight-gradient GEMM (a [n, m] x [m, k] reduction over m rows): the output
    has only ceil(n/256) * ceil(k/256) * groups tiles, too few for 256 CUs, so the rows are cut
    into S chunks run as one batched GEMM (S * tiles >= ~256 workgroups, >= 1024 rows per chunk)
    and the fp32 partials summed (measured: tools/gemm_shapes.py)."""
    tiles = max(1, -(-n // 256) * -(-k // 256) * groups)
    s = 1
    # at most 8 chunks: past that the fp32 partials' round trip costs more than the extra
    # workgroups gain (tools/wgrad_probe.py: 512x512 layer 82 us at S=32, 61 us at S=8)
    while s * 2 * tiles <= 256 and s < 8 and m % (s * 2) == 0 and m // (s * 2) >= 1024:
        s *= 2
    return s


def _weight_grad_parts(g, z):
    """The split-K partials of dW[b] = g[b]^T z[b]: [B, S, n, k] fp32 (S = 1: no split), summed
    by the caller (phc_reduce_into, straight into the gradient views)."""
    B, M, n = g.shape
    k = z.shape[2]
    S = 1 if g.dtype == torch.bfloat16 else _split_k(M, n, k, B)
    if S == 1:
        return _bmm(g.transpose(1, 2), z, True).view(B, 1, n, k)
    part = _bmm(g.reshape(B * S, M // S, n).transpose(1, 2), z.reshape(B * S, M // S, k), True)
    return part.view(B, S, n, k)


def _weight_grad(g, z):
    """dW[b] = g[b]^T z[b] in fp32 for g [B, M, n], z [B, M, k] (split-K over M)."""
    B, M, n = g.shape
    k = z.shape[2]
    S = 1 if g.dtype == torch.bfloat16 else _split_k(M, n, k, B)
    if S == 1:
        return _bmm(g.transpose(1, 2), z, True)
    part = _bmm(g.reshape(B * S, M // S, n).transpose(1, 2), z.reshape(B * S, M // S, k), True)
    return part.view(B, S, n, k).sum(1)


class TwinWeights:
    """Stacked [actor; critic] weights in the GEMM dtype + fp32 biases, keyed on parameter
    versions (in-place optimizer updates and load_state_dict bump them)."""

    def __init__(self, actor_linears, critic_linears):
        assert len(actor_linears) == len(critic_linears)
        self.pairs = list(zip(actor_linears, critic_linears))
        self._key = None
        self.w, self.b = [], []
        # fp32 parameters copied alongside the MFMA operands into 16-B aligned buffers (a view into
        # the flat optimizer buffer is only 4-B aligned): (parameter, destination, transposed
        # destination) — the rollout tail reads the mu head's weight transposed, [hidden, ld]
        self.extras = []

    def add_extra(self, param, transpose_ld=None):
        """Register a 2-D fp32 parameter [rows, cols] for an aligned copy refreshed with the MFMA
        operands; returns the destination (valid after the next mfma_operands / refresh_twin):
        [rows, cols], or with transpose_ld the transposed [cols, rows] view of a [cols,
        transpose_ld] buffer."""
        if transpose_ld is None:
            dst = torch.empty(param.shape, dtype=torch.float32, device=param.device)
            self.extras.append((param, dst, None))
            return dst
        rows, cols = param.shape
        buf = torch.zeros((cols, transpose_ld), dtype=torch.float32, device=param.device)
        dst_t = buf[:, :rows]
        self.extras.append((param, None, dst_t))
        return dst_t

    def params(self):
        out = []
        for a, c in self.pairs:
            out += [a.weight, a.bias, c.weight, c.bias]
        return out + [e[0] for e in self.extras]

    def get(self, dtype):
        """Stacked weights for `dtype`; refreshed IN PLACE when a parameter changed, so a captured
        rollout graph that reads these buffers sees every optimizer update."""
        key = cache_key(dtype, self.params())
        if key == self._key:
            return self.w, self.b
        with torch.no_grad():
            same = bool(self.w) and self.w[0].dtype == dtype
            for i, (a, c) in enumerate(self.pairs):
                if same:
                    if i == 0:
                        n = a.weight.shape[0]
                        self.w[0][:n].copy_(a.weight)
                        self.w[0][n:].copy_(c.weight)
                    else:
                        self.w[i][0].copy_(a.weight)
                        self.w[i][1].copy_(c.weight)
                    self.b[i][:a.bias.shape[0]].copy_(a.bias)
                    self.b[i][a.bias.shape[0]:].copy_(c.bias)
                else:
                    if i == 0:
                        w = torch.cat([a.weight, c.weight]).to(dtype).contiguous()
                    else:
                        w = torch.stack([a.weight, c.weight]).to(dtype).contiguous()
                    b = torch.cat([a.bias, c.bias]).float().contiguous()
                    if i == 0:
                        self.w, self.b = [], []
                    self.w.append(w)
                    self.b.append(b)
        self._key = key
        return self.w, self.b


def _pad64(k):
    return -(-k // 64) * 64


class MfmaOperands:
    """Operands of the hand-written MFMA GEMM path (phc_twin_gemm) in a half-precision dtype:
    the first layer's stacked weight zero-padded to K % 64 == 0, the stacked [2, N, K] weights
    of layers 2..L (forward B operands) and their transposes [2, K, N] (input-gradient B
    operands), the stacked fp32 biases.  Refreshed in place (a captured rollout graph reads
    these buffers) by one phc_pack_weights launch."""

    def __init__(self):
        self.key = None
        self.plan_key = None
        self.plan = None
        self.w0 = None
        self.w, self.wt, self.b = [], [], []


def mfma_supported(weights):
    """The MFMA path needs every reduction and output width (but the input's) % 64 == 0."""
    for i, (a, _) in enumerate(weights.pairs):
        n, k = a.weight.shape
        if n % 64 or (i > 0 and k % 64):
            return False
    return True


def _pack_jobs(weights, ops):
    a0, c0 = weights.pairs[0]
    n0, k0 = a0.weight.shape
    jobs = [(a0.weight.detach(), ops.w0[:n0, :k0], None), (c0.weight.detach(), ops.w0[n0:, :k0], None)]
    for i, (a, c) in enumerate(weights.pairs):
        na = a.bias.shape[0]
        jobs += [(a.bias.detach(), ops.b[i][:na], None), (c.bias.detach(), ops.b[i][na:], None)]
    for i, (a, c) in enumerate(weights.pairs[1:]):
        jobs += [(a.weight.detach(), ops.w[i][0], ops.wt[i][0]), (c.weight.detach(), ops.w[i][1], ops.wt[i][1])]
    jobs += [(p.detach(), dst, dst_t) for p, dst, dst_t in weights.extras]
    return jobs


def mfma_operands(weights, dtype):
    ps = weights.params()
    key = cache_key(dtype, ps)
    ops = weights.__dict__.setdefault("_mfma", MfmaOperands())
    if ops.key == key:
        return ops
    with torch.no_grad():
        a0, c0 = weights.pairs[0]
        n0, k0 = a0.weight.shape
        fresh = ops.w0 is None or ops.w0.dtype != dtype
        if fresh:
            ops.w0 = torch.zeros((2 * n0, _pad64(k0)), dtype=dtype, device=a0.weight.device)
            ops.w = [torch.empty((2,) + a.weight.shape, dtype=dtype, device=a.weight.device)
                     for a, _ in weights.pairs[1:]]
            ops.wt = [torch.empty((2, a.weight.shape[1], a.weight.shape[0]), dtype=dtype, device=a.weight.device)
                      for a, _ in weights.pairs[1:]]
            ops.b = [torch.empty(2 * a.bias.shape[0], dtype=torch.float32, device=a.bias.device)
                     for a, _ in weights.pairs]
        lk = layout_key(dtype, ps)
        if fresh or ops.plan_key != lk:
            ops.plan_jobs = _pack_jobs(weights, ops)
            ops.plan, ops.plan_key = N.PackPlan(ops.plan_jobs), lk
            ops.fresh_dtype, ops.fresh_params = dtype, ps
            weight_cache.register_plan(ops)  # FlatAdam's step may write these copies itself
        ops.plan.run()
    ops.key = key
    return ops


class MfmaTrunkSaved:
    """What the MFMA trunk backward needs from its forward: the padded input, the transposed
    weights, the pre-activations and the post-activations (layer inputs) of every layer."""

    def __init__(self, xc, wt, pres, zs, K0):
        self.xc, self.wt, self.pres, self.zs, self.K0 = xc, wt, pres, zs, K0
        self.deriv = False  # pres are the pre-activations (True: their silu', PHC_EPI_BIAS_SILU_D)
        self.L = len(wt) + 1


# the forward GEMMs keep silu'(pre-activation) for the backward instead of the pre-activation itself
# (PHC_EPI_BIAS_SILU_D / PHC_EPI_DSILU_GRAD: the same bytes, and the input-gradient epilogues multiply
# instead of evaluating the sigmoid, which made them VALU-bound); PHC_SILU_DERIV=0 keeps the pre-activation
SILU_DERIV = os.environ.get("PHC_SILU_DERIV", "1") == "1"


def mfma_trunk_forward(x, weights, need_grad):
    """Both trunks on the hand-written MFMA GEMM (phc_gemm.hip) for f16 / bf16 operands: every
    forward GEMM carries its bias + SiLU epilogue (pre-activation kept for backward in the operand
    type, see PRE_HALF), the last layer its bias (fp32 out).  Returns (y [2, M, n] fp32,
    MfmaTrunkSaved or None)."""
    dt = _compute_dtype()
    with torch.autocast("cuda", enabled=False):
        ops = mfma_operands(weights, dt)
        B = ops.b
        M = x.shape[0]
        K0 = weights.pairs[0][0].weight.shape[1]
        Kp = ops.w0.shape[1]
        if x.dtype == dt and x.shape[1] == Kp and x.is_contiguous():
            xc = x  # already the padded GEMM operand (obs_half_input)
        else:
            xc = torch.empty((M, Kp), dtype=dt, device=x.device)
            xc[:, :K0].copy_(x)
            if Kp != K0:
                xc[:, K0:].zero_()  # K padding (the padded weight columns are zero too)
        n1 = ops.w0.shape[0] // 2
        z = torch.empty((2, M, n1), dtype=dt, device=x.device)
        pdt = dt if PRE_HALF else torch.float32
        pre = torch.empty((M, 2 * n1), dtype=pdt, device=x.device) if need_grad else None
        epi_fwd = N.EPI_BIAS_SILU_D if (need_grad and SILU_DERIV) else N.EPI_BIAS_SILU
        N.twin_gemm(xc, ops.w0, epi_fwd, z, (2, n1), bias=B[0], aux=pre, aux_layout=N.SPLIT,
                    out_layout=N.GROUPED, k_valid=K0)
        pres, zs = [pre], [z]
        L = len(ops.w) + 1
        for l in range(1, L):
            n = ops.w[l - 1].shape[1]
            if l < L - 1:
                z = torch.empty((2, M, n), dtype=dt, device=x.device)
                pre = torch.empty((2, M, n), dtype=pdt, device=x.device) if need_grad else None
                N.twin_gemm(zs[-1], ops.w[l - 1], epi_fwd, z, (2, n), bias=B[l], aux=pre)
                pres.append(pre)
                zs.append(z)
            else:
                y = torch.empty((2, M, n), dtype=torch.float32, device=x.device)
                N.twin_gemm(zs[-1], ops.w[l - 1], N.EPI_BIAS, y, (2, n), bias=B[l])
    saved = MfmaTrunkSaved(xc, list(ops.wt), pres, zs, K0) if need_grad else None
    if saved is not None:
        saved.deriv = epi_fwd == N.EPI_BIAS_SILU_D  # pres hold silu'(pre-activation)
    return y, saved


_CU_COUNT = {}


def _wgrad_tiles(g, z):
    m, n = g.shape[-1], z.shape[-1]
    return -(-m // 256) * -(-n // 256) * (g.shape[0] if g.dim() == 3 else 1)


def _wgrad_splits(tiles, rows, device):
    """Row chunks for a split-K phc_weight_grad launch: the largest power of two <= 32 that keeps
    tiles * S within one wave of the CUs and >= 1024 rows (a multiple of 64) per chunk."""
    cus = _cu_count(device)
    S = 1
    while S < 32 and tiles * S * 2 <= cus and rows % (S * 2 * 64) == 0 and rows // (S * 2) >= 1024:
        S *= 2
    return S


def _cu_count(device):
    key = torch.device(device).index or 0
    cus = _CU_COUNT.get(key)
    if cus is None:
        cus = _CU_COUNT[key] = torch.cuda.get_device_properties(device).multi_processor_count
    return cus


def _grouped_subset(problems, device, rest=False):
    """Layers of the grouped weight-gradient launch: all of them when their 256 x 256 tiles fill
    whole waves of the CUs (or fit one), else without the smallest layers that would open
    another wave for a handful of tiles (each tile runs over all rows, so a partial wave costs a
    whole one).  rest=True: the layers left out."""
    cus = _cu_count(device)
    order = sorted(problems, key=lambda l: _wgrad_tiles(problems[l][1], problems[l][2]))
    tiles = {l: _wgrad_tiles(problems[l][1], problems[l][2]) for l in problems}
    total = sum(tiles.values())
    keep = set(problems)
    if total > cus and total % cus:
        target = (total // cus) * cus
        for l in order:  # smallest first
            if total <= target or len(keep) == 1:
                break
            keep.discard(l)
            total -= tiles[l]
        if total % cus and total > cus:  # could not trim to whole waves: group everything
            keep = set(problems)
    sel = sorted(set(problems) - keep) if rest else sorted(keep, reverse=True)
    return sel


def _mfma_wgrad_parts(g, z):
    """Split-K partials [B, S, n, k] of dW[b] = g[b]^T z[b] for the MFMA path's per-layer weight
    gradients: the transposed-read kernel (phc_weight_grad) when the rows split into 64-row
    chunks, else the library GEMMs (_weight_grad_parts: ragged row counts, e.g. 1000-row tests)."""
    B, M, n = g.shape
    if M % 64 or n % 8 or z.shape[2] % 8:
        return _weight_grad_parts(g, z)
    S = _wgrad_splits(_wgrad_tiles(g, z), M, g.device)
    gg = g if B > 1 else g[0]
    zz = z if z.shape[0] > 1 else z[0]
    part = N.weight_grad(gg, zz, S)  # [S, B, n, k]
    return part.transpose(0, 1)


def mfma_trunk_backward(saved, g, db, params, direct, extra_jobs=None, store=False):
    """Backward of mfma_trunk_forward from g = d loss / d (last layer output) [2, M, n] in the
    operand dtype and db = its fp32 column sums [2n] (the last layer's bias gradient; in direct
    mode also [parts, 2n] partial rows, summed into the bias gradients).  Every
    input-gradient GEMM carries its SiLU-backward + bias-gradient epilogue.  Weight gradients:
    all layers in ONE grouped launch after the input-gradient chain (phc_weight_grad_group: one
    workgroup per output tile over all M rows, no split, no partials), or — when a data-parallel
    hook is set (GRAD_READY) — per layer as soon as the layer's output gradient exists (split-K
    library GEMMs summed by phc_reduce_into), so each layer's all-reduce can start while the
    backward continues.  direct: the gradients are summed straight into the parameters' bound
    .grad views and None is returned; otherwise the per-parameter gradient list (trunk params
    order).  extra_jobs: (src, dst) accumulate jobs of the caller, flushed with the trunk's own
    bias-gradient sums in one phc_reduce_into launch (direct mode).  store (direct mode): every
    gradient is written, not added — each parameter has exactly one writer (its job or its
    grouped tile), so the caller need not zero the gradient buffer first."""
    L, K0 = saved.L, saved.K0
    xc, WT, pres, zs = saved.xc, saved.wt, saved.pres, saved.zs
    epi_bwd = N.EPI_DSILU_GRAD if saved.deriv else N.EPI_SILU_GRAD
    dt = xc.dtype
    M = xc.shape[0]
    grads = [None] * (2 * L)
    jobs = list(extra_jobs) if (direct and extra_jobs) else []
    grouped = (GRAD_READY is None or not DP_PER_LAYER) and GROUPED_WGRAD and M % 64 == 0 and L <= N.WGRAD_GROUP_MAX
    problems = {}

    def put_bias(l, db):
        wa, ba, wc, bc = params[4 * l:4 * l + 4]
        n = wa.shape[0]
        if db.dim() == 2:  # [parts, 2n] partial rows (the fused PPO tail)
            jobs.extend([(db[:, :n].unsqueeze(1), ba.grad), (db[:, n:].unsqueeze(1), bc.grad)])
        else:
            jobs.extend([(db[:n].view(1, n), ba.grad), (db[n:].view(1, n), bc.grad)])

    def put(l, dW_parts, db):
        """dW_parts: ([parts, 2n, k] or [2, parts, n, k] partials, layer-1 flag), db [2n]
        (per-layer path: without data parallelism, or with DP_PER_LAYER)."""
        if not direct:
            grads[2 * l], grads[2 * l + 1] = dW_parts, db
            return
        wa, ba, wc, bc = params[4 * l:4 * l + 4]
        n, k = wa.shape
        if l == 0:
            jobs.extend([(dW_parts[:, :n, :k], wa.grad), (dW_parts[:, n:, :k], wc.grad)])
        else:
            jobs.extend([(dW_parts[0], wa.grad), (dW_parts[1], wc.grad)])
        put_bias(l, db)
        if GRAD_READY is not None:  # data parallel: this layer's gradients now, then its all-reduce
            N.reduce_into(jobs, accumulate=not store)
            jobs.clear()
            GRAD_READY(params[4 * l:4 * l + 4])

    def wdst(l):
        """Destinations of layer l's weight gradient: the bound .grad views (direct), or views of a
        new [2, n, k] (layer 0: [2n, k]) tensor, returned as well."""
        wa, _, wc, _ = params[4 * l:4 * l + 4]
        if direct:
            return [wa.grad, wc.grad], None
        n = wa.shape[0]
        W = torch.empty((2 * n, wa.shape[1]) if l == 0 else (2,) + tuple(wa.shape), dtype=torch.float32,
                        device=xc.device)
        return [W[:n], W[n:]] if l == 0 else [W[0], W[1]], W

    with torch.autocast("cuda", enabled=False):
        for l in range(L - 1, 0, -1):
            if grouped:
                d, W = wdst(l)
                problems[l] = (l, g, zs[l - 1], (g, zs[l - 1], d, g.shape[2], zs[l - 1].shape[2]))
                if direct:
                    put_bias(l, db)
                else:
                    grads[2 * l], grads[2 * l + 1] = W, db
            else:
                put(l, _mfma_wgrad_parts(g, zs[l - 1]) if direct else _mfma_wgrad_parts(g, zs[l - 1]).sum(1), db)
            k = WT[l - 1].shape[1]
            # direct mode: the bias gradient stays as the epilogue's per-m-tile partial rows
            # [tiles, 2k], summed by the final phc_reduce_into launch (no column-sum launch per layer)
            if direct:
                db = torch.empty((N.twin_gemm_m_tiles(M, k, 2), 2 * k), dtype=torch.float32, device=g.device)
                bias_out = dict(bias_partial=db)
            else:
                db = torch.empty(2 * k, dtype=torch.float32, device=g.device)
                bias_out = dict(bias_grad=db)
            if l > 1:
                gp = torch.empty((2, M, k), dtype=dt, device=g.device)
                N.twin_gemm(g, WT[l - 1], epi_bwd, gp, (2, k), aux=pres[l - 1], **bias_out)
            else:  # into the first layer's SPLIT [M, 2k] layout, the operand of its weight gradient
                gp = torch.empty((M, 2 * k), dtype=dt, device=g.device)
                N.twin_gemm(g, WT[0], epi_bwd, gp, (2, k), aux=pres[0], aux_layout=N.SPLIT,
                            out_layout=N.SPLIT, **bias_out)
                if grouped:
                    d, W = wdst(0)
                    problems[0] = (0, gp, xc, (gp, xc, d, k, K0))
                    if direct:
                        put_bias(0, db)
                    else:
                        grads[0], grads[1] = W, db
                elif direct:
                    put(0, _mfma_wgrad_parts(gp[None], xc[None])[0], db)
                else:
                    put(0, _mfma_wgrad_parts(gp[None], xc[None])[0].sum(0)[:, :K0], db)
            g = gp
        if grouped:
            for l in _grouped_subset(problems, xc.device, rest=True):
                # layers left out of the grouped launch (they would start another whole wave): the
                # split-K form of the same kernel, enough row chunks to give every CU a workgroup
                _, gg, zz, (_, _, d, _, _) = problems[l]
                S = _wgrad_splits(_wgrad_tiles(gg, zz), M, xc.device)
                part = N.weight_grad(gg, zz, S)  # [S, B, m, n]
                if l == 0:
                    n = d[0].shape[0]
                    pairs = [(part[:, 0, :n, :K0], d[0]), (part[:, 0, n:, :K0], d[1])]
                else:
                    pairs = [(part[:, 0], d[0]), (part[:, 1], d[1])]
                if direct:
                    jobs.extend(pairs)  # summed with the bias jobs below
                else:
                    N.reduce_into(pairs, accumulate=False)
            sel = _grouped_subset(problems, xc.device)
            if direct and GRAD_READY is not None and DP_SPLIT_GROUP:
                # data parallel, split mode: the bias sums and left-out layers first, then the last
                # three trunk layers' tiles in one launch and their span's all-reduce, which overlaps
                # the launch of the remaining layers (the same tiles: bit-equal to one launch)
                if jobs:
                    N.reduce_into(jobs, accumulate=not store)
                    jobs.clear()
                for lo in (max(L - 3, 0), 0):
                    part = [l for l in sel if l >= lo]
                    sel = [l for l in sel if l < lo]
                    if part:
                        N.weight_grad_group([problems[l][3] for l in part], accumulate=not store)
                    GRAD_READY([p for l in range(L - 1, lo - 1, -1) for p in params[4 * l:4 * l + 4]])
                return None
            N.weight_grad_group([problems[l][3] for l in sel], accumulate=direct and not store)
        if direct:
            if jobs:
                N.reduce_into(jobs, accumulate=not store)
            if grouped and GRAD_READY is not None:
                # data parallel on the grouped path: every trunk gradient is final now; their
                # all-reduce (one contiguous span of the flat buffer, last layer first) starts
                GRAD_READY([p for l in range(L - 1, -1, -1) for p in params[4 * l:4 * l + 4]])
            return None
    out = []
    for l in range(L):
        dW, db = grads[2 * l], grads[2 * l + 1]
        n = db.shape[0] // 2
        dWa, dWc = (dW[:n], dW[n:]) if l == 0 else (dW[0], dW[1])
        out += [dWa, db[:n], dWc, db[n:]]
    return out


def direct_grads_bound(params):
    """True when every parameter's .grad is a bound dense fp32 view (FlatGrads): the backward
    then writes gradients in place instead of returning them to autograd."""
    return DIRECT_GRADS and all(p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
                                for p in params)


class TwinTrunkMfmaFn(torch.autograd.Function):
    """TwinTrunkFn on the hand-written MFMA GEMM (mfma_trunk_forward / mfma_trunk_backward)."""

    @staticmethod
    def forward(ctx, x, weights, need_grad, *params):
        y, saved = mfma_trunk_forward(x, weights, need_grad)
        if need_grad:
            ctx.saved = saved
            ctx.params = params
        return y

    @staticmethod
    def backward(ctx, gy):
        saved, params = ctx.saved, ctx.params
        direct = direct_grads_bound(params)
        with torch.autocast("cuda", enabled=False):
            gy = gy.float().contiguous()
            M, n = gy.shape[1], gy.shape[2]
            db = torch.empty(2 * n, dtype=torch.float32, device=gy.device)
            g = torch.empty(gy.shape, dtype=saved.xc.dtype, device=gy.device)
            N.act_bwd(gy, N.GROUPED, None, N.GROUPED, g, N.GROUPED, db, M, 2, n, N.ACT_NONE)
        out = mfma_trunk_backward(saved, g, db, params, direct)
        ctx.saved = None
        if direct:
            return (None, None, None) + (None,) * len(params)
        return (None, None, None, *out)


class TwinTrunkFn(torch.autograd.Function):
    """y[2, M, H] = the two trunks' last Linear outputs (before LayerNorm)."""

    @staticmethod
    def forward(ctx, x, weights, need_grad, *params):
        dt = _compute_dtype()
        with torch.autocast("cuda", enabled=False):
            W, B = weights.get(dt)
            M = x.shape[0]
            xc = x.to(dt).contiguous()
            n1 = W[0].shape[0] // 2
            # GEMM outputs are fp32 in every mode (see the module docstring)
            y = torch.mm(xc, W[0].t()) if dt == torch.float32 else torch.mm(xc, W[0].t(), out_dtype=torch.float32)
            z = torch.empty((2, M, n1), dtype=dt, device=x.device)  # [M, 2*n1] SPLIT -> GROUPED
            # the raw GEMM output y is kept for backward (pre-activation = y + b recomputed there)
            N.bias_act_fwd(y, N.SPLIT, B[0], None, z, N.GROUPED, M, 2, n1, N.ACT_SILU)
            pres, zs = [y], [z]
            L = len(W)
            for l in range(1, L):
                n = W[l].shape[1]
                y = _bmm(zs[-1], W[l].transpose(1, 2), True)  # [2, M, n] fp32
                if l < L - 1:
                    z = torch.empty(y.shape, dtype=dt, device=y.device)
                    N.bias_act_fwd(y, N.GROUPED, B[l], None, z, N.GROUPED, M, 2, n, N.ACT_SILU)
                    pres.append(y)
                    zs.append(z)
                else:
                    N.bias_act_fwd(y, N.GROUPED, B[l], None, y, N.GROUPED, M, 2, n, N.ACT_NONE)
        if need_grad:
            ctx.save_for_backward(xc, *W, *B, *pres, *zs)
            ctx.L = L
        return y

    @staticmethod
    def backward(ctx, gy):
        L = ctx.L
        saved = ctx.saved_tensors
        xc, W, B = saved[0], saved[1:1 + L], saved[1 + L:1 + 2 * L]
        pres, zs = saved[1 + 2 * L:3 * L], saved[3 * L:4 * L - 1]
        dt = xc.dtype
        M = xc.shape[0]
        grads = [None] * (2 * L)  # (dW, db) per layer, stacked over the two trunks
        with torch.autocast("cuda", enabled=False):
            gy = gy.float().contiguous()
            n = gy.shape[2]
            db = torch.empty(2 * n, dtype=torch.float32, device=gy.device)
            if dt == torch.float32:
                g = gy
                N.act_bwd(g, N.GROUPED, None, N.GROUPED, None, N.GROUPED, db, M, 2, n, N.ACT_NONE)
            else:  # the fp32 gradient rounded once into the next GEMMs' operand; bias grad from fp32
                g = torch.empty(gy.shape, dtype=dt, device=gy.device)
                N.act_bwd(gy, N.GROUPED, None, N.GROUPED, g, N.GROUPED, db, M, 2, n, N.ACT_NONE)
            for l in range(L - 1, 0, -1):
                dW = _weight_grad(g, zs[l - 1])  # [2, n_out, n_in] fp32
                grads[2 * l], grads[2 * l + 1] = dW, db
                dz = _bmm(g, W[l], True)  # [2, M, n_in] fp32
                n = dz.shape[2]
                db = torch.empty(2 * n, dtype=torch.float32, device=g.device)
                if l > 1:
                    g = dz if dt == torch.float32 else torch.empty(dz.shape, dtype=dt, device=dz.device)
                    N.act_bwd(dz, N.GROUPED, pres[l - 1], N.GROUPED, g, N.GROUPED, db, M, 2, n, N.ACT_SILU,
                              pre_bias=B[l - 1])
                else:
                    # SPLIT [M, 2n]; fp32: the layer-1 GEMM output buffer is reused for its grad
                    g1 = pres[0] if dt == torch.float32 else torch.empty(pres[0].shape, dtype=dt, device=dz.device)
                    N.act_bwd(dz, N.GROUPED, pres[0], N.SPLIT, g1, N.SPLIT, db, M, 2, n, N.ACT_SILU, pre_bias=B[0])
                    grads[0] = _weight_grad(g1[None], xc[None])[0]  # [2n, K]
                    grads[1] = db
        out = []
        for l in range(L):
            dW, db = grads[2 * l], grads[2 * l + 1]
            n = db.shape[0] // 2
            if l == 0:
                dWa, dWc = dW[:n], dW[n:]
            else:
                dWa, dWc = dW[0], dW[1]
            out += [dWa.float(), db[:n], dWc.float(), db[n:]]
        return (None, None, None, *out)


# half-precision trunks on phc_twin_gemm (PHC_MFMA_GEMM=0: hipBLASLt GEMMs + epilogue kernels)
USE_MFMA_GEMM = os.environ.get("PHC_MFMA_GEMM", "1") == "1"
# trunk weight / bias gradients written straight into bound gradient views (FlatGrads) by one
# phc_reduce_into launch per backward (PHC_DIRECT_GRADS=0: returned to autograd)
DIRECT_GRADS = os.environ.get("PHC_DIRECT_GRADS", "1") == "1"
# the pre-activations saved for backward in the operand type (what torch.autocast keeps: its
# Linear returns f16 / bf16 and SiLU saves that input), not fp32: a third less epilogue traffic
# (PHC_PRE_HALF=0: fp32)
PRE_HALF = os.environ.get("PHC_PRE_HALF", "1") == "1"
# data-parallel hook (distributed.FlatGrads.overlap_begin): called with the parameters whose
# gradients a direct-mode backward has just finished, so their all-reduce can start early
GRAD_READY = None
# one grouped weight-gradient launch per backward (False: per-layer split-K library GEMMs)
GROUPED_WGRAD = True
# data parallel: per-layer split-K weight gradients, each layer's all-reduce started as soon as
# its gradient lands (1), or the single-GPU grouped launch with every trunk span's all-reduce
# started after it (0, default: the grouped launch fills the 256 CUs exactly once and RCCL's
# kernels do not take CUs from the backward's GEMMs)
DP_PER_LAYER = os.environ.get("PHC_DP_PER_LAYER", "0") == "1"
# data parallel on the grouped path: two grouped weight-gradient launches, the last three trunk
# layers first, so that span's all-reduce overlaps the second launch (PHC_DP_SPLIT_GROUP=1)
DP_SPLIT_GROUP = os.environ.get("PHC_DP_SPLIT_GROUP", "0") == "1"
DP_MODES = ("grouped", "per_layer", "split")


def set_dp_mode(mode):
    """grouped (default): one grouped weight-gradient launch, then the trunk span's all-reduce;
    per_layer: per-layer split-K weight gradients, each layer's all-reduce started as it lands;
    split: two grouped launches (last three layers first), the first span's all-reduce overlapping
    the second launch.  Only the data-parallel backward reads this (GRAD_READY set)."""
    global DP_PER_LAYER, DP_SPLIT_GROUP
    if mode not in DP_MODES:
        raise ValueError(f"dp mode {mode!r} not in {DP_MODES}")
    DP_PER_LAYER, DP_SPLIT_GROUP = mode == "per_layer", mode == "split"


def dp_mode():
    return "per_layer" if DP_PER_LAYER else ("split" if DP_SPLIT_GROUP else "grouped")


def _use_mfma(weights, dtype):
    return USE_MFMA_GEMM and dtype != torch.float32 and mfma_supported(weights)


def refresh_twin(weights, dtype):
    """Refresh, in place, the weight copies the trunk path for `dtype` reads (a captured
    rollout graph replays on these buffers)."""
    if _use_mfma(weights, dtype):
        mfma_operands(weights, dtype)
    else:
        weights.get(dtype)


def half_input_width(weights, dtype):
    """Width of the first trunk GEMM's padded operand for `dtype` on the MFMA path (None when
    that path does not serve `dtype`)."""
    if not _use_mfma(weights, dtype):
        return None
    return _pad64(weights.pairs[0][0].weight.shape[1])


def twin_trunks(x, weights):
    """Both trunks' pre-LayerNorm outputs, [2, M, H] (index 0 = actor, 1 = critic).  x is the
    normalised observation (fp32), or on the MFMA path already its padded half operand."""
    if not x.is_cuda:
        raise RuntimeError("twin_trunks runs on the HIP path only (no CPU fallback)")
    need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in weights.params())
    if _use_mfma(weights, _compute_dtype()):
        return TwinTrunkMfmaFn.apply(x, weights, need_grad, *weights.params())
    return TwinTrunkFn.apply(x, weights, need_grad, *weights.params())


def _row_sum(g):
    """sum over rows of g [M, N] in fp32 as a two-level reduction: torch's dim-0 sum of a
    [32768, 69] tensor runs on 128 threads (0.33 ms, rocprofv3), the chunked form on thousands."""
    M = g.shape[0]
    S = 1
    while S < 256 and M % (S * 2) == 0:
        S *= 2
    return g.float().reshape(S, M // S, -1).sum(1).sum(0)


def _head_kernels(x, w):
    """phc_mu_head_* serve an fp32 device head with at most 80 outputs and width % 16 == 0."""
    return x.is_cuda and w.shape[0] <= N.MU_HEAD_MAX_ACTIONS and w.shape[1] % 16 == 0 and x.dtype == torch.float32


class HeadLinearFn(torch.autograd.Function):
    """nn.Linear with few outputs (the actor's mu head 512 -> 69, the critic's value head 512 -> 1)
    with a split-K weight gradient and a chunked bias gradient: torch's backward for these shapes
    picks 32x16/32x64-tile GEMMs and a 128-thread bias reduction (~0.8 ms per minibatch)."""
    # (fp32 head: see forward)

    @staticmethod
    def forward(ctx, x, w, b):
        # float32 storage in every precision mode: the heads are < 1 % of the FLOPs; on the device
        # the three GEMMs run on the fp32-input MFMA kernels of phc_head.hip (phc_mu_head_*)
        with torch.autocast("cuda", enabled=False):
            xc = x.float().contiguous()
            wc = w.detach().float().contiguous()
            if _head_kernels(xc, wc):
                y = N.mu_head_fwd(xc, wc if wc.data_ptr() % 16 == 0 else wc.clone(), b.detach().float().contiguous())
            else:
                y = torch.mm(xc, w.t()) + b
        ctx.save_for_backward(xc, w)
        ctx.x_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        with torch.autocast("cuda", enabled=False):
            g = gy.to(xc.dtype).contiguous()
            wd = wc.detach().float().contiguous()
            if _head_kernels(xc, wd):
                gx = N.mu_head_dgrad(g, wd).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
                gw = N.mu_head_wgrad_parts(g, xc, 128).sum(0)
            else:
                gx = torch.mm(g, wc).to(ctx.x_dtype) if ctx.needs_input_grad[0] else None
                gw = _weight_grad(g[None], xc[None])[0]
            gb = _row_sum(g)
        return gx, gw, gb


def head_linear(x, lin):
    return HeadLinearFn.apply(x, lin.weight, lin.bias)


class TwinLNSiLUFn(torch.autograd.Function):
    """silu(LayerNorm_g(y[g])) for the two trunks (actor g = 0, critic g = 1) in one HIP kernel each
    way (phc_ln_silu_fwd / _bwd); float32 output as torch's LayerNorm under autocast."""

    @staticmethod
    def forward(ctx, y, g_a, b_a, g_c, b_c, eps):
        gamma = torch.cat([g_a, g_c]).float().contiguous()
        beta = torch.cat([b_a, b_c]).float().contiguous()
        yc = y.contiguous()
        z, mr = N.ln_silu_fwd(yc, gamma, beta, eps)
        ctx.save_for_backward(yc, gamma, beta, mr)
        return z

    @staticmethod
    def backward(ctx, dz):
        y, gamma, beta, mr = ctx.saved_tensors
        dy, dg, db = N.ln_silu_bwd(y, gamma, beta, mr, dz.float().contiguous())
        n = y.shape[2]
        return dy, dg[:n], db[:n], dg[n:], db[n:], None


def twin_ln_silu_supported(width):
    """phc_ln_silu_* handle row widths that are multiples of 256 up to 1024 (the reference's 512)."""
    return width % 256 == 0 and width <= 1024


def twin_ln_silu(y, ln_a, ln_c):
    """[2, M, H] trunk outputs -> [2, M, H] float32 silu(LayerNorm(.)) with the actor's / critic's
    nn.LayerNorm parameters (same eps)."""
    return TwinLNSiLUFn.apply(y, ln_a.weight, ln_a.bias, ln_c.weight, ln_c.bias, ln_a.eps)
