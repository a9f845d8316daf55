"""Twin actor/critic trunks (policies/twin_mlp.py + phc_mlp.hip) vs plain PyTorch fp32
(needs an MI355X).

Tolerances: the epilogue kernels against torch fp32 elementwise ops within 2e-6 relative
(fp32 arithmetic; exp may differ by an ulp).  The whole policy forward/backward against the
unfused nn.Sequential path evaluated with exact fp32 GEMMs (matmul precision "highest"):
relative L2 error <= 1e-4 for the xf32 GEMM path (the reference's own TF32 setting is looser),
<= 3e-3 for fp16 operands and <= 3e-2 for bf16 operands (fp32 accumulation throughout).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("layouts", [(0, 1), (1, 1), (0, 0)])
def test_bias_act_kernels_vs_torch(layouts):
    from puffer_phc_amd import _native as N

    yl, ol = layouts
    g = torch.Generator(device=DEV).manual_seed(0)
    M, G, C = 300, 2, 260  # ragged rows and a partial 256-column tile
    y = torch.randn((M, G * C) if yl == N.SPLIT else (G, M, C), device=DEV, generator=g) * 3
    b = torch.randn(G * C, device=DEV, generator=g)

    def logical(t, layout):  # -> [M, G*C]
        return t if layout == N.SPLIT else t.permute(1, 0, 2).reshape(M, G * C)

    ref_pre = logical(y, yl) + b
    ref_out = torch.nn.functional.silu(ref_pre)
    pre = torch.empty_like(y)
    out = torch.empty((M, G * C) if ol == N.SPLIT else (G, M, C), device=DEV)
    N.bias_act_fwd(y, yl, b, pre, out, ol, M, G, C, N.ACT_SILU)
    torch.testing.assert_close(logical(pre, yl), ref_pre, atol=0, rtol=0)
    torch.testing.assert_close(logical(out, ol), ref_out, atol=1e-6, rtol=2e-6)
    # backward: grad_pre = dout * silu'(pre) and the bias gradient
    dout = torch.randn_like(out)
    p = ref_pre.clone().requires_grad_(True)
    torch.nn.functional.silu(p).backward(logical(dout, ol))
    gp = torch.empty_like(pre)
    db = torch.empty(G * C, device=DEV)
    N.act_bwd(dout, ol, pre, yl, gp, yl, db, M, G, C, N.ACT_SILU)
    torch.testing.assert_close(logical(gp, yl), p.grad, atol=1e-6, rtol=2e-6)
    torch.testing.assert_close(db, p.grad.sum(0), atol=1e-4, rtol=1e-5)
    # identity act: bias add only / column sums only
    if yl == ol:
        out2 = torch.empty_like(out)
        N.bias_act_fwd(y, yl, b, None, out2, ol, M, G, C, N.ACT_NONE)
        torch.testing.assert_close(logical(out2, ol), ref_pre, atol=0, rtol=0)
    N.act_bwd(dout, ol, None, ol, None, ol, db, M, G, C, N.ACT_NONE)
    torch.testing.assert_close(db, logical(dout, ol).sum(0), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_bias_act_half_types(dtype):
    from puffer_phc_amd import _native as N

    M, G, C = 128, 2, 512
    y = (torch.randn((G, M, C), device=DEV) * 2).to(dtype)
    b = torch.randn(G * C, device=DEV)
    out = torch.empty_like(y)
    N.bias_act_fwd(y, N.GROUPED, b, None, out, N.GROUPED, M, G, C, N.ACT_SILU)
    ref = torch.nn.functional.silu(y.float() + b.view(G, 1, C))
    tol = 1e-3 if dtype == torch.float16 else 8e-3
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_bias_act_f32_to_half(dtype):
    """fp32 GEMM output -> half-precision operand of the next GEMM: fp32 math, one rounding on the
    write; the bias gradient sums the fp32 values (before that rounding)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(5)
    M, G, C = 200, 2, 512
    y = torch.randn((M, G * C), device=DEV, generator=g) * 2
    b = torch.randn(G * C, device=DEV, generator=g)
    out = torch.empty((G, M, C), dtype=dtype, device=DEV)
    N.bias_act_fwd(y, N.SPLIT, b, None, out, N.GROUPED, M, G, C, N.ACT_SILU)
    ref = torch.nn.functional.silu(y + b).view(M, G, C).permute(1, 0, 2)
    ulp = 2.0 ** -10 if dtype == torch.float16 else 2.0 ** -7
    torch.testing.assert_close(out.float(), ref, atol=1e-6, rtol=ulp)  # one rounding of the fp32 value
    dz = torch.randn((G, M, C), device=DEV, generator=g)
    gp = torch.empty((M, G * C), dtype=dtype, device=DEV)
    db = torch.empty(G * C, device=DEV)
    N.act_bwd(dz, N.GROUPED, y, N.SPLIT, gp, N.SPLIT, db, M, G, C, N.ACT_SILU, pre_bias=b)
    p = (y + b).requires_grad_(True)
    torch.nn.functional.silu(p).backward(dz.permute(1, 0, 2).reshape(M, G * C))
    torch.testing.assert_close(gp.float(), p.grad, atol=1e-6, rtol=ulp)
    torch.testing.assert_close(db, p.grad.sum(0), atol=1e-4, rtol=1e-5)


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


def _policy():
    from puffer_phc_amd.policies import PHCPolicy, Policy

    torch.manual_seed(0)
    pol = Policy(PHCPolicy(_Env())).to(DEV)
    with torch.no_grad():  # non-trivial normaliser and biases
        pol.policy.obs_norm.running_mean.uniform_(-0.5, 0.5)
        pol.policy.obs_norm.running_var.uniform_(0.5, 2.0)
        for m in pol.modules():
            if isinstance(m, torch.nn.Linear):
                m.bias.uniform_(-0.1, 0.1)
    return pol


def _run(pol, obs, act, fused, precision, loss_scale=1.0):
    pol.policy.fused = fused
    pol.zero_grad(set_to_none=True)
    ctx = torch.autocast("cuda", dtype=precision) if precision is not None else torch.autocast("cuda", enabled=False)
    with ctx:
        _, logp, _, value = pol(obs, action=act)
    loss = logp.sum() * 1e-3 + (value.float() ** 2).sum()
    (loss * loss_scale).backward()  # fp16 training scales the loss (GradScaler) the same way
    grads = {n: p.grad.detach() / loss_scale for n, p in pol.named_parameters() if p.grad is not None}
    return logp.detach(), value.detach().float(), grads


@pytest.mark.parametrize("precision,tol,rows", [(None, 1e-4, 1000), (torch.float16, 3e-3, 1000),
                                                (torch.bfloat16, 3e-2, 1000), (torch.float16, 3e-3, 2048),
                                                (torch.bfloat16, 3e-2, 2048)])
def test_twin_policy_matches_unfused_fp32(precision, tol, rows):
    """rows = 1000: per-layer split-K weight gradients; rows = 2048 (a multiple of 64): the grouped
    weight-gradient launch (phc_weight_grad_group) plus the split-K form for the layer it leaves out,
    all against exact fp32 torch autograd."""
    pol = _policy()
    g = torch.Generator(device=DEV).manual_seed(1)
    obs = torch.randn((rows, 934), device=DEV, generator=g) * 2
    act = torch.randn((rows, 69), device=DEV, generator=g) * 0.3
    prev = torch.get_float32_matmul_precision()
    try:
        torch.set_float32_matmul_precision("highest")
        ref_lp, ref_v, ref_g = _run(pol, obs, act, fused=False, precision=None)
        torch.set_float32_matmul_precision("high")
        lp, v, gr = _run(pol, obs, act, fused=True, precision=precision)
    finally:
        torch.set_float32_matmul_precision(prev)
    # logprob of a near-deterministic Normal (sigma = e^-2.9) amplifies mu errors; compare mu via logp
    assert rel(v, ref_v) <= tol
    assert rel(lp, ref_lp) <= tol * 10
    assert set(gr) == set(ref_g)
    worst = max(rel(gr[k], ref_g[k]) for k in ref_g)
    assert worst <= tol * 10, worst
    # fused path keeps reference state-dict keys and fp32 grads
    assert all(t.dtype == torch.float32 for t in gr.values())


def test_twin_cache_follows_optimizer_updates():
    """The stacked-weight cache is rebuilt after in-place parameter updates."""
    pol = _policy()
    obs = torch.randn((64, 934), device=DEV)
    with torch.no_grad():
        a0 = pol(obs)[3].clone()
        for p in pol.policy.critic_mlp.parameters():
            p.add_(0.01)
        a1 = pol(obs)[3]
        pol.policy.fused = False
        a2 = pol(obs)[3]
    assert not torch.equal(a0, a1)
    assert rel(a1, a2) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_ln_silu_kernels_vs_torch(dtype):
    """phc_ln_silu_fwd / _bwd vs torch LayerNorm + SiLU per group (fp32 math; inputs in dtype)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(3)
    G, M, H = 2, 777, 512  # ragged rows: partial last wave of the backward
    y = (torch.randn((G, M, H), device=DEV, generator=g) * 2 + 0.5).to(dtype)
    gamma = torch.randn(G * H, device=DEV, generator=g)
    beta = torch.randn(G * H, device=DEV, generator=g)
    z, mr = N.ln_silu_fwd(y.contiguous(), gamma, beta, 1e-5)
    yr = y.float().clone().requires_grad_(True)
    gr = gamma.view(G, 1, H).clone().requires_grad_(True)
    br = beta.view(G, 1, H).clone().requires_grad_(True)
    ref = torch.nn.functional.silu(torch.nn.functional.layer_norm(yr, (H,), eps=1e-5) * gr + br)
    torch.testing.assert_close(z, ref.detach(), atol=2e-5, rtol=2e-5)
    dz = torch.randn((G, M, H), device=DEV, generator=g)
    ref.backward(dz)
    dy, dg, db = N.ln_silu_bwd(y.contiguous(), gamma, beta, mr, dz)
    tol = 2e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(dy.float(), yr.grad, atol=tol, rtol=tol)
    torch.testing.assert_close(dg, gr.grad.view(-1), atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(db, br.grad.view(-1), atol=1e-3, rtol=1e-4)


class _TF32Linear(torch.autograd.Function):
    """nn.Linear under TF32 (the reference's matmul precision "high" on its GPUs): every GEMM
    operand rounded to a 10-bit mantissa, exact fp32 products and sums, forward and backward."""

    @staticmethod
    def _r(t):
        i = t.contiguous().view(torch.int32)
        return ((i + 0x1000) & ~0x1FFF).view(torch.float32)  # round-to-nearest on the 13 dropped bits

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _TF32Linear._r(x) @ _TF32Linear._r(w).t() + b

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        r = _TF32Linear._r
        gx = r(gy.reshape(-1, gy.shape[-1])) @ r(w)
        gw = r(gy.reshape(-1, gy.shape[-1])).t() @ r(x.reshape(-1, x.shape[-1]))
        return gx.view(x.shape), gw, gy.reshape(-1, gy.shape[-1]).sum(0)


def test_fp16_operands_match_tf32_error():
    """The fp16 mode (fp16 GEMM operands, fp32 GEMM outputs and epilogues) is as precise as the
    reference's TF32 GEMMs: its error against exact fp32 stays within 1.5x the error of an exact
    TF32 emulation of the unfused policy (values, log-probs and every parameter gradient; both
    are a few 1e-4 here, bf16 operands are ~8x worse).  The backward runs on a loss scaled by
    2^12, as fp16 training does (GradScaler), so the deepest activation gradients stay fp16
    normals: fp16's exponent range is the one difference from TF32."""
    pol = _policy()
    g = torch.Generator(device=DEV).manual_seed(2)
    obs = torch.randn((1000, 934), device=DEV, generator=g) * 2
    act = torch.randn((1000, 69), device=DEV, generator=g) * 0.3
    from puffer_phc_amd.policies.pufferl_policy import Linear

    prev = torch.get_float32_matmul_precision()
    orig = Linear.forward
    try:
        torch.set_float32_matmul_precision("highest")
        ref = _run(pol, obs, act, fused=False, precision=None)
        Linear.forward = lambda self, x: _TF32Linear.apply(x, self.weight, self.bias)
        tf32 = _run(pol, obs, act, fused=False, precision=None)
        Linear.forward = orig
        f16 = _run(pol, obs, act, fused=True, precision=torch.float16, loss_scale=2.0 ** 12)
    finally:
        Linear.forward = orig
        torch.set_float32_matmul_precision(prev)
    assert rel(tf32[1], ref[1]) > 0, "the TF32 emulation must be in effect"
    errs = {}
    for name, i in (("logp", 0), ("value", 1)):
        errs[name] = (rel(f16[i], ref[i]), rel(tf32[i], ref[i]))
    for k in ref[2]:
        errs[k] = (rel(f16[2][k], ref[2][k]), rel(tf32[2][k], ref[2][k]))
    bad = {k: v for k, v in errs.items() if v[0] > 1.5 * v[1] + 1e-7}
    assert not bad, bad


@pytest.mark.parametrize("precision", [torch.float16, torch.bfloat16])
def test_mfma_trunks_match_library_path(precision):
    """The hand-written MFMA GEMM path (phc_twin_gemm with fused epilogues) against the
    hipBLASLt + epilogue-kernel path on the same half-precision operands: the same rounding
    points, so only fp32 summation order differs (rel. L2 <= 1e-3 f16 / 1e-2 bf16 incl. the
    log-prob's amplification of mu)."""
    from puffer_phc_amd.policies import twin_mlp

    pol = _policy()
    g = torch.Generator(device=DEV).manual_seed(6)
    obs = torch.randn((1000, 934), device=DEV, generator=g) * 2
    act = torch.randn((1000, 69), device=DEV, generator=g) * 0.3
    assert twin_mlp.mfma_supported(pol.policy._twin)
    try:
        twin_mlp.USE_MFMA_GEMM = False
        lib = _run(pol, obs, act, fused=True, precision=precision, loss_scale=2.0 ** 12)
        twin_mlp.USE_MFMA_GEMM = True
        mf = _run(pol, obs, act, fused=True, precision=precision, loss_scale=2.0 ** 12)
    finally:
        twin_mlp.USE_MFMA_GEMM = True
    tol = 1e-3 if precision == torch.float16 else 1e-2
    assert rel(mf[1], lib[1]) <= tol
    assert rel(mf[0], lib[0]) <= tol
    worst = max(rel(mf[2][k], lib[2][k]) for k in lib[2])
    assert worst <= tol, worst


def test_direct_gradient_writes_match_autograd():
    """With gradient views bound (FlatGrads), the MFMA trunk writes its weight / bias gradients
    straight into them (phc_reduce_into) and accumulates onto what is there; without, autograd
    receives them.  Same values up to the split-K partial summation order (rel 1e-6)."""
    from puffer_phc_amd.distributed import FlatGrads

    pol = _policy()
    g = torch.Generator(device=DEV).manual_seed(7)
    obs = torch.randn((2048, 934), device=DEV, generator=g)
    act = torch.randn((2048, 69), device=DEV, generator=g) * 0.3
    _, _, ref = _run(pol, obs, act, fused=True, precision=torch.float16)
    fg = FlatGrads(pol.parameters())
    for p in fg.params:
        p.grad.fill_(0.25)  # accumulate semantics: the bound values are added to
    with torch.autocast("cuda", dtype=torch.float16):
        _, logp, _, value = pol(obs, action=act)
    (logp.sum() * 1e-3 + (value.float() ** 2).sum()).backward()
    for n, p in pol.named_parameters():
        if n in ref:
            torch.testing.assert_close(p.grad - 0.25, ref[n], rtol=1e-5, atol=1e-6)
