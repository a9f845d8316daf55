"""optim.FlatAdam (phc_opt_step, phc_optim.hip) vs the reference's update tail
(clean_pufferl/core.py:360-372: clip_grad_norm_ + torch.optim.Adam(eps=1e-5), and
torch.amp.GradScaler for the fp16 path) on the same parameters and gradients (needs an MI355X).

Tolerance: parameters within rel 2e-6 / abs 1e-8 after several steps (Adam's update is
lr * m / (sqrt(v) + eps) in fp32 in both; torch's moment updates use lerp / addcmul, a different
rounding order; the clip coefficient here comes from a double-precision norm).  The logged norm
(sum of per-parameter norms) within rel 1e-5, the logged L2-init distance within rel 1e-4
(double accumulation here, fp32 per-parameter means in torch).  Skip / scale decisions are exact.
"""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SHAPES = [(256, 96), (256,), (69, 256), (69,), (1, 256), (1,), (3000,)]


def _params(seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(s, device=DEV, generator=g) * 0.1) for s in SHAPES]


def _grads(step, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(100 + step)
    return [torch.randn(s, device=DEV, generator=g) * (0.5 + step) * scale for s in SHAPES]


def _flat(params, **kw):
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.optim import FlatAdam

    fg = FlatGrads(params)
    return fg, FlatAdam(fg, lr=3e-4, eps=1e-5, **kw)


@pytest.mark.parametrize("max_norm", [1.0, 1e9])
def test_clip_adam_matches_torch(max_norm):
    ref = _params(0)
    ours = _params(0)
    opt_ref = torch.optim.Adam(ref, lr=3e-4, eps=1e-5)
    fg, opt = _flat(ours)
    opt.track_init_distance()
    init = [p.detach().clone() for p in ref]
    for step in range(4):
        for p, g in zip(ref, _grads(step)):
            p.grad = g.clone()
        norms = torch.stack([p.grad.norm() for p in ref])
        # the L2-init regulariser of the parameters before this step (core.py:352-359)
        l2 = sum(((p.detach() - p0) ** 2).mean() for p, p0 in zip(ref, init))
        torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_ref.step()
        fg.zero()
        for p, g in zip(ours, _grads(step)):
            p.grad.copy_(g)
        out = opt.fused_step(max_norm)
        torch.testing.assert_close(out[0], norms.sum(), rtol=1e-5, atol=0)
        torch.testing.assert_close(out[2], l2, rtol=1e-4, atol=1e-12)
        for a, b in zip(ours, ref):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-6, atol=1e-8)
    # the module parameters are views of the flat buffer, each slice starting 64-B aligned
    from puffer_phc_amd.distributed import PARAM_ALIGN

    for p in ours:
        off = fg._range[id(p)][0]
        assert off % PARAM_ALIGN == 0 and p.data_ptr() == opt.param_flat[off:].data_ptr()
    assert int(opt._i[2]) == 4


def test_loss_scale_skip_and_growth():
    """GradScaler semantics: gradients of a scaled loss are unscaled; an inf gradient skips the
    step (parameters and moments untouched) and halves the scale; growth after the interval."""
    ref = _params(1)
    ours = _params(1)
    opt_ref = torch.optim.Adam(ref, lr=3e-4, eps=1e-5)
    fg, opt = _flat(ours, use_loss_scale=True, init_scale=1024.0, growth_interval=2)
    scales = []
    for step in range(5):
        S = float(opt.loss_scale)
        scales.append(S)
        grads = _grads(step)
        fg.zero()
        for p, g in zip(ours, grads):
            p.grad.copy_(g * S)
        if step == 2:
            ours[3].grad[0] = float("inf")
        before = [p.detach().clone() for p in ours]
        opt.fused_step(1.0)
        if step == 2:
            for a, b in zip(ours, before):
                assert torch.equal(a.detach(), b)
            continue
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt_ref.step()
        for a, b in zip(ours, ref):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-6, atol=1e-8)
    # 1024 -> (2 clean steps) 2048 -> inf: 1024 -> 1024 -> (2 clean) 2048
    assert scales == [1024.0, 1024.0, 2048.0, 1024.0, 1024.0]
    assert float(opt.loss_scale) == 2048.0
    assert int(opt.skipped_steps) == 1
    assert int(opt._i[2]) == 4


def test_state_dict_round_trip():
    a = _params(2)
    fg, opt = _flat(a, use_loss_scale=True)
    for step in range(3):
        fg.zero()
        for p, g in zip(a, _grads(step, float(opt.loss_scale))):
            p.grad.copy_(g)
        opt.fused_step(5.0)
    sd = opt.state_dict()
    assert all(float(st["step"]) == 3.0 for st in sd["state"].values())
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    fg2, opt2 = _flat(b, use_loss_scale=True)
    opt2.load_state_dict(sd)
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
    assert float(opt2.loss_scale) == float(opt.loss_scale)
    assert sd["flat_adam"]["index_space"] == "module"
    # a FlatAdam state dict of the earlier, flat grad-ready index order (no marker) is refused, not
    # loaded into whichever parameters happen to share the count
    old = copy.deepcopy(sd)
    del old["flat_adam"]["index_space"]
    with pytest.raises(ValueError, match="older FlatAdam"):
        opt2.load_state_dict(old)
    bad = copy.deepcopy(sd)
    k0 = next(iter(bad["state"]))
    bad["state"][k0]["exp_avg"] = bad["state"][k0]["exp_avg"].reshape(-1)[:1].clone()
    with pytest.raises(ValueError, match="moments of shape"):
        opt2.load_state_dict(bad)
    for o, f, P in ((opt, fg, a), (opt2, fg2, b)):
        f.zero()
        for p, g in zip(P, _grads(7, float(o.loss_scale))):
            p.grad.copy_(g)
        o.fused_step(5.0)
    for x, y in zip(a, b):
        assert torch.equal(x.detach(), y.detach())


@pytest.mark.parametrize("parts", [1, 2, 8, 9, 16, 17, 32, 128, 131])
@pytest.mark.parametrize("accumulate", [False, True])
def test_reduce_into_many_parts(parts, accumulate):
    """phc_reduce_into (phc_optim.hip k_reduce_into) over many parts: the 8-running-sum branch
    with its remainder loop (> 8 parts), a row stride wider than the columns and a part stride
    wider than rows * row stride, several jobs of different shapes in one launch.  dst (+)=
    src.sum(0) within rel 1e-6 of a float64 sum (the kernel sums in a fixed fp32 order)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(parts)
    jobs, refs = [], []
    for rows, cols, pad_c, pad_p in [(37, 96, 8, 64), (1, 1000, 0, 24), (256, 69, 3, 0)]:
        big = torch.randn((parts, rows * (cols + pad_c) + pad_p), device=DEV, generator=g)
        src = big[:, :rows * (cols + pad_c)].reshape(parts, rows, cols + pad_c)[:, :, :cols]
        dst = torch.randn((rows, cols), device=DEV, generator=g)
        ref = src.double().sum(0) + (dst.double() if accumulate else 0.0)
        jobs.append((src, dst))
        refs.append(ref)
    N.reduce_into(jobs, accumulate=accumulate)
    torch.cuda.synchronize()
    for (_, dst), ref in zip(jobs, refs):
        torch.testing.assert_close(dst.double(), ref, rtol=1e-6, atol=1e-5)


def test_checkpoint_optimizer_state_loads_into_torch_adam(tmp_path):
    """trainer_state.pt's optimizer_state_dict is in the reference's layout
    (clean_pufferl/utils.py:18-42: torch.optim.Adam(policy.parameters()).state_dict()): a plain
    torch.optim.Adam over a copy of the policy loads it and takes the same next step as FlatAdam
    (state indices follow policy.parameters(), frozen sigma included; FlatAdam's flat buffer is
    laid out in backward-ready order instead)."""
    import copy

    import numpy as np

    from puffer_phc_amd.clean_pufferl.utils import save_checkpoint
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.distributed import FlatGrads
    from puffer_phc_amd.envs.humanoid_phc import Box
    from puffer_phc_amd.optim import FlatAdam
    from puffer_phc_amd.policies import PHCPolicy, Policy

    class E:
        single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        single_action_space = Box(-np.ones(69), np.ones(69))
        amp_observation_space = None

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(E(), hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    fg = FlatGrads(policy.parameters(), order=policy.policy.grad_ready_order())
    opt = FlatAdam(fg, lr=3e-4, eps=1e-5)
    assert fg.params[0] is not list(policy.parameters())[0]  # the flat layout is NOT module order
    g = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(3):
        fg.flat.copy_(torch.randn(fg.flat.shape, device=DEV, generator=g))
        opt.step()
    cfg = TrainConfig(data_dir=str(tmp_path))
    save_checkpoint(policy, opt, cfg, "ck", 3, 123)
    st = torch.load(tmp_path / "ck" / "trainer_state.pt", weights_only=True)
    sd = st["optimizer_state_dict"]
    names = [n for n, _ in policy.named_parameters()]
    assert sd["param_groups"][0]["params"] == list(range(len(names)))
    frozen = [i for i, p in enumerate(policy.parameters()) if not p.requires_grad]
    assert frozen and all(i not in sd["state"] for i in frozen)  # sigma: no state, as torch's Adam
    twin = copy.deepcopy(policy)
    ref = torch.optim.Adam(twin.parameters(), lr=3e-4, eps=1e-5)
    ref.load_state_dict(sd)
    grads = torch.randn(fg.flat.shape, device=DEV, generator=g)
    fg.flat.copy_(grads)
    for p, q in zip(policy.parameters(), twin.parameters()):
        if p.requires_grad:
            q.grad = p.grad.detach().clone()
    opt.step()
    ref.step()
    for (n, p), q in zip(policy.named_parameters(), twin.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-6, atol=1e-8, msg=n)
    # and back: FlatAdam loads torch's own state dict
    fg2 = FlatGrads(twin.parameters(), order=twin.policy.grad_ready_order())
    opt2 = FlatAdam(fg2, lr=3e-4, eps=1e-5)
    opt2.load_state_dict(ref.state_dict())
    assert int(opt2._i[2]) == 4
    torch.testing.assert_close(opt2.exp_avg_sq[fg2._range[id(fg2.params[0])][0]:][:5],
                               ref.state[fg2.params[0]]["exp_avg_sq"].reshape(-1)[:5])
