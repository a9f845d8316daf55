"""GEMM-operand weight caches vs the parameters they copy (needs an MI355X).

The MFMA GEMMs of the twin trunks and the AMP discriminator read f16 / bf16 copies of the fp32
parameters (twin_mlp.mfma_operands, disc_mlp.disc_operands).  FlatAdam updates the parameters
through a raw pointer (phc_opt_step), which torch's version counters do not see; the caches are
keyed on a generation FlatAdam advances (policies/weight_cache.py).  These tests pin that every
cached operand equals `param.to(dtype)` bit for bit after optimizer steps, a load_state_dict and a
rollout-style in-place refresh, and that the refresh kernel (phc_pack_weights) rounds exactly as
torch's copy_ does.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class _Env:
    def __init__(self, amp=True):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = Box(np.full(1960, -np.inf), np.full(1960, np.inf)) if amp else None


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_pack_weights_matches_torch_copy(dtype):
    """phc_pack_weights: ragged tiles, a destination leading dimension wider than the columns
    (the K padding must stay untouched), transposes, 1-D biases, several jobs per launch."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(0)
    jobs, checks = [], []
    for rows, cols, pad in [(300, 934, 26), (64, 64, 0), (1, 1000, 0), (77, 5, 3), (2048, 1536, 0)]:
        src = torch.randn((rows, cols), device=DEV, generator=g) * 3
        src[0, 0] = 65504.0 * 1.5  # f16 overflow -> inf, as torch's copy_
        dst = torch.full((rows, cols + pad), 7.0, device=DEV).to(dtype)
        dst_t = torch.empty((cols, rows), dtype=dtype, device=DEV)
        jobs.append((src, dst[:, :cols], dst_t))
        checks.append((src, dst, dst_t, cols))
    bias = torch.randn(513, device=DEV, generator=g)
    bdst = torch.empty(1026, dtype=dtype, device=DEV)
    jobs.append((bias, bdst[513:], None))
    N.PackPlan(jobs).run()
    torch.cuda.synchronize()
    for src, dst, dst_t, cols in checks:
        ref = src.to(dtype)
        assert torch.equal(dst[:, :cols], ref)
        assert torch.equal(dst_t, ref.t())
        if dst.shape[1] > cols:
            assert bool((dst[:, cols:] == 7.0).all())
    assert torch.equal(bdst[513:], bias.to(dtype))


def _check_trunk_operands(pol, dtype):
    from puffer_phc_amd.policies import twin_mlp

    ops = twin_mlp.mfma_operands(pol._twin, dtype)
    a0, c0 = pol._twin.pairs[0]
    n0, k0 = a0.weight.shape
    assert torch.equal(ops.w0[:n0, :k0], a0.weight.detach().to(dtype))
    assert torch.equal(ops.w0[n0:, :k0], c0.weight.detach().to(dtype))
    assert bool((ops.w0[:, k0:] == 0).all())
    for i, (a, c) in enumerate(pol._twin.pairs):
        na = a.bias.shape[0]
        assert torch.equal(ops.b[i][:na], a.bias.detach()) and torch.equal(ops.b[i][na:], c.bias.detach())
    for i, (a, c) in enumerate(pol._twin.pairs[1:]):
        assert torch.equal(ops.w[i][0], a.weight.detach().to(dtype))
        assert torch.equal(ops.w[i][1], c.weight.detach().to(dtype))
        assert torch.equal(ops.wt[i][0], a.weight.detach().t().to(dtype))
        assert torch.equal(ops.wt[i][1], c.weight.detach().t().to(dtype))
    return ops


def _check_disc_operands(pol, dtype):
    from puffer_phc_amd.policies import disc_mlp

    ops = disc_mlp.disc_operands(pol, dtype)
    l1, l2 = pol._disc_mlp[0], pol._disc_mlp[2]
    k1 = l1.weight.shape[1]
    assert torch.equal(ops.w1[:, :k1], l1.weight.detach().to(dtype))
    assert torch.equal(ops.w2, l2.weight.detach().to(dtype))
    assert torch.equal(ops.w2t, l2.weight.detach().t().to(dtype))
    assert torch.equal(ops.b1, l1.bias.detach()) and torch.equal(ops.b2, l2.bias.detach())


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_caches_follow_flat_adam_steps(dtype):
    """Two FlatAdam steps (raw-pointer updates), then a load_state_dict: the trunk and
    discriminator operands follow every change, and the fused fp16 trunk forward agrees with the
    unfused fp32 modules reading the updated parameters."""
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.optim import FlatAdam
    from puffer_phc_amd.policies import PHCPolicy, Policy

    torch.manual_seed(0)
    pol = Policy(PHCPolicy(_Env())).to(DEV)
    inner = pol.policy
    fg = FlatGrads(pol.parameters(), order=inner.grad_ready_order())
    opt = FlatAdam(fg, lr=1e-2)
    obs = torch.randn((256, 934), device=DEV)
    _check_trunk_operands(inner, dtype)
    _check_disc_operands(inner, dtype)
    g = torch.Generator(device=DEV).manual_seed(1)
    outs = []
    for step in range(2):
        w0 = inner._twin.pairs[0][0].weight
        before = w0.detach().clone()
        fg.flat.copy_(torch.randn(fg.flat.shape, device=DEV, generator=g))
        opt.fused_step(1e9)
        assert not torch.equal(w0.detach(), before)  # the trunk's first layer moved
        _check_trunk_operands(inner, dtype)
        _check_disc_operands(inner, dtype)
        with torch.no_grad(), torch.autocast("cuda", dtype=dtype):
            inner.fused = True
            v_fused = pol(obs)[3].float()
        with torch.no_grad():
            inner.fused = False
            v_ref = pol(obs)[3].float()
        inner.fused = True
        rel = float((v_fused - v_ref).norm() / v_ref.norm())
        assert rel < (3e-3 if dtype == torch.float16 else 3e-2), rel
        outs.append(v_fused)
    assert not torch.equal(outs[0], outs[1])
    # load_state_dict of the optimizer (moments only) and of the module (parameters): the module
    # load goes through copy_, the optimizer one through the flat buffers
    sd = {k: v.clone() for k, v in pol.state_dict().items()}
    with torch.no_grad():
        opt.param_flat.mul_(0.5)  # a raw write of every parameter ...
    opt.load_state_dict(opt.state_dict())  # ... made visible by the optimizer's generation bump
    _check_trunk_operands(inner, dtype)
    pol.load_state_dict(sd)
    _check_trunk_operands(inner, dtype)
    _check_disc_operands(inner, dtype)


def test_rollout_graph_sees_optimizer_updates():
    """The captured rollout graph reads the operand buffers refreshed in place: after an optimizer
    step, a replay computes with the new weights (its value equals an eager forward's)."""
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.optim import FlatAdam
    from puffer_phc_amd.policies import PHCPolicy, Policy, twin_mlp

    torch.manual_seed(0)
    pol = Policy(PHCPolicy(_Env(amp=False))).to(DEV)
    inner = pol.policy
    fg = FlatGrads(pol.parameters(), order=inner.grad_ready_order())
    opt = FlatAdam(fg, lr=1e-2)
    n = 512
    obs = torch.randn((n, 934), device=DEV)
    noise = torch.zeros((n, 69), device=DEV)
    act, lp, val = torch.empty((n, 69), device=DEV), torch.empty(n, device=DEV), torch.empty(n, device=DEV)

    def body():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            assert inner.act_rollout(obs, noise, act, lp, val)

    body()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body()
    graph.replay()
    v0, a0 = val.clone(), act.clone()
    fg.flat.copy_(torch.randn(fg.flat.shape, device=DEV))
    opt.fused_step(1e9)
    twin_mlp.refresh_twin(inner._twin, torch.float16)  # what RolloutStep.run does before a replay
    graph.replay()
    v1, a1 = val.clone(), act.clone()
    body()
    assert not torch.equal(v0, v1) and not torch.equal(a0, a1)
    assert torch.equal(v1, val) and torch.equal(a1, act)
    # the mu head reads its 16-B aligned copy (float4 loads), refreshed with the trunk operands
    # (the transposed [hidden, actions] copy with a 16-B aligned row stride: the rollout tail's
    # weight loads coalesce across the actions)
    assert inner._w_mu_aligned.data_ptr() % 16 == 0 and inner._w_mu_aligned.stride(0) % 4 == 0
    assert torch.equal(inner._w_mu_aligned, inner.mu[0].weight.detach().t())


def test_step_writes_operand_copies_bit_exact(monkeypatch):
    """FlatAdam's step writes the registered operand copies itself (phc_opt_step_operands): the
    caches stay current with no refresh launch, every copy equals param.to(dtype), and the
    parameters / moments are bit-identical to the plain step followed by the caches' own refresh
    (PHC_OPERANDS_IN_STEP=0)."""
    from puffer_phc_amd import optim
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.optim import FlatAdam
    from puffer_phc_amd.policies import PHCPolicy, Policy, disc_mlp, twin_mlp, weight_cache

    runs = []
    for in_step in (True, False):
        monkeypatch.setattr(optim, "OPERANDS_IN_STEP", in_step)
        torch.manual_seed(0)
        pol = Policy(PHCPolicy(_Env())).to(DEV)
        inner = pol.policy
        fg = FlatGrads(pol.parameters(), order=inner.grad_ready_order())
        opt = FlatAdam(fg, lr=1e-2, use_loss_scale=True)
        ops = twin_mlp.mfma_operands(inner._twin, torch.float16)
        dops = disc_mlp.disc_operands(inner, torch.float16)
        g = torch.Generator(device=DEV).manual_seed(1)
        for _ in range(3):
            fg.flat.copy_(torch.randn(fg.flat.shape, device=DEV, generator=g) * 1e3)
            opt.fused_step(10.0)
            if in_step:
                assert weight_cache.is_fresh(ops) and weight_cache.is_fresh(dops)
                assert opt._ops is not None and len(opt._ops_owners) == 2
            else:
                assert not weight_cache.is_fresh(ops)
            _check_trunk_operands(inner, torch.float16)
            _check_disc_operands(inner, torch.float16)
        torch.cuda.synchronize()
        runs.append((opt.param_flat.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt._state.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
