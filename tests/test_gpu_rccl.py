"""RCCL executed on the leased GPU (needs an MI355X): a 1-rank torch.distributed process group on
backend "nccl" (RCCL on ROCm), brought up by distributed.init_from_env exactly as bench.py /
scripts/train.py bring up each rank of a node (device_id bound, one process per GPU).  With the
group up, every data-parallel code path runs for real: the gradient spans' async all-reduces
started from inside the fused backward (twin_mlp.GRAD_READY -> FlatGrads._on_ready) on RCCL's
stream, in the grouped and the per-layer modes; the global advantage statistics; the RunningNorm
moments exchange (phc_rms_moments / all_gather / phc_rms_apply); the rank-agreed step count.

A 1-rank all-reduce is the identity and the division by the world size is exact, so the DP
gradients must equal the single-GPU path's BIT FOR BIT, and so must the RunningNorm update (one
part merged = phc_rms_update).  A whole PPO iteration under the group is compared with the same
iteration with the data-parallel helpers switched off (the advantage statistics differ in the
last bits: float64 sums vs torch's fp32 mean / std).
"""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl():
    import torch.distributed as dist

    from puffer_phc_amd import distributed as D

    keys = ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    try:
        rank, world = D.init_from_env("nccl", force=True)
        assert (rank, world) == (0, 1) and D.is_dist() and dist.get_backend() == "nccl"
        yield D
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


def test_rccl_collectives(rccl):
    D = rccl
    from puffer_phc_amd.clean_pufferl import core as C

    x = torch.randn((4, 32768), device=DEV)
    ms = D.global_mean_std_rows(x)
    torch.testing.assert_close(ms[:, 0], x.mean(1), rtol=0, atol=1e-6)
    torch.testing.assert_close(ms[:, 1], x.std(1), rtol=1e-6, atol=1e-7)
    assert C._global_count(131072 - 5, DEV) == 131072 - 5
    t = torch.arange(1 << 20, device=DEV, dtype=torch.float32)
    ref = t.clone()
    D.allreduce_sum_(t)
    assert torch.equal(t, ref)


@pytest.mark.parametrize("mode", ["grouped", "per_layer", "split"])
def test_rccl_overlapped_backward_bit_equal(rccl, mode):
    """The trainer's DP minibatch backward (full widths, 32768 rows, gradients stored into a
    NaN-filled flat buffer, all-reduces started during the backward) vs the single-GPU backward."""
    D = rccl
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy, twin_mlp
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss

    torch.manual_seed(0)
    policy = Policy(PHCPolicy(_Env())).to(DEV)
    pol = policy.policy
    fg = D.FlatGrads(policy.parameters(), order=pol.grad_ready_order())
    M = 32768
    g = torch.Generator(device=DEV).manual_seed(3)
    obs = torch.randn((M, 934), device=DEV, generator=g)
    atn = 0.1 * torch.randn((M, 69), device=DEV, generator=g)
    old_lp = torch.randn(M, device=DEV, generator=g) + 200.0
    adv, val, ret = (torch.randn(M, device=DEV, generator=g) for _ in range(3))
    ms = torch.tensor([0.0, 1.0], device=DEV)
    coefs = ppo_coefs(TrainConfig(), pol.soft_bound)

    def backward(dp):
        fg.fill_grads_(float("nan"))
        with torch.autocast("cuda", dtype=torch.float16):
            xh = pol.obs_half_input(obs)
            loss, _ = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, coefs, store_grads=True)
        if dp:
            fg.overlap_begin()
            assert twin_mlp.GRAD_READY is not None
        (loss * 1024.0).backward()
        if dp:
            fg.overlap_finish()
        torch.cuda.synchronize()
        return fg.flat.detach().clone()

    prev = (twin_mlp.dp_mode(), twin_mlp.GROUPED_WGRAD)
    ready = []
    try:
        twin_mlp.set_dp_mode(mode)
        orig = fg._on_ready
        fg._on_ready = lambda ps: (ready.append(len(ps)), orig(ps))  # noqa: E731 (spy)
        dp = backward(True)
        fg._on_ready = orig
        # the single-GPU path with the same weight-gradient kernels: grouped launch (grouped and
        # split modes: the same tiles), or (per-layer mode) the split-K per-layer launches
        twin_mlp.GROUPED_WGRAD = mode != "per_layer"
        single = backward(False)
    finally:
        twin_mlp.set_dp_mode(prev[0])
        twin_mlp.GROUPED_WGRAD = prev[1]
    if mode == "split":  # ... the last three trunk layers' span (12 params), then the whole trunk
        assert ready[-2:] == [12, 24], ready
    assert torch.isfinite(dp).all()
    assert torch.equal(dp, single)


def test_rccl_running_norm_bit_equal(rccl):
    from puffer_phc_amd import _native as N
    from puffer_phc_amd.policies.running_norm import RunningNorm

    g = torch.Generator(device=DEV).manual_seed(9)
    a, b = RunningNorm(934).to(DEV), RunningNorm(934).to(DEV)
    for k in range(2):
        x = torch.randn((131072 + 77, 934), device=DEV, generator=g) * (1 + k) + 0.3
        a.update(x)  # the group is up: moments -> all_gather -> apply
        b._ws = N.rms_update(x, b.running_mean, b.running_var, b.count, b._ws)  # the single-GPU kernel
    torch.cuda.synchronize()
    assert torch.equal(a.running_mean, b.running_mean) and torch.equal(a.running_var, b.running_var)
    assert float(a.count) == float(b.count) == 3.0


def test_rccl_ppo_iteration_matches_single_gpu(rccl, monkeypatch):
    D = rccl
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    def run():
        q, t, c, fps = synthetic_clips(256, 40, 120, seed=3, device=DEV)
        env = PHCPufferEnv(EnvConfig(num_envs=256, seed=2), motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        env.reset()
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env)).to(DEV)
        # one minibatch of the whole batch, one epoch: the logged losses are those of the parameters
        # both runs start from; one Adam step follows
        cfg = TrainConfig(batch_size=256 * 64, minibatch_size=256 * 64, update_epochs=1, checkpoint_interval=10 ** 9)
        comps, info, util = clean_pufferl.create("r", cfg, env.cfg, env, policy)
        clean_pufferl.evaluate(comps, info)
        policy.policy.update_obs_rms(comps.experience.obs)
        losses = clean_pufferl.train(comps, info, util)
        params = torch.cat([p.detach().reshape(-1) for p in policy.parameters() if p.requires_grad])
        return info.global_step, losses, params, policy.policy.obs_norm.running_var.clone()

    steps_dp, l_dp, p_dp, var_dp = run()
    monkeypatch.setattr(D, "is_dist", lambda: False)
    steps_1, l_1, p_1, var_1 = run()
    assert steps_dp == steps_1
    assert torch.equal(var_dp, var_1)
    for k in ("policy_loss", "value_loss", "approx_kl"):
        a, b = getattr(l_dp, k), getattr(l_1, k)
        assert abs(a - b) <= 1e-5 * max(abs(b), 1e-3), (k, a, b)
    # one Adam step of lr 1e-4 (|update| ~ lr): a coordinate whose tiny gradient changes sign on
    # last-bit differences moves by up to 2 lr; the rest agree to fp32 rounding
    diff = (p_dp - p_1).abs()
    assert float(diff.max()) <= 2.5e-4
    assert float((diff > 1e-6).float().mean()) < 1e-3


@pytest.mark.parametrize("mode", ["grouped", "split"])
def test_rccl_graphed_dp_train_matches_eager_dp(rccl, monkeypatch, mode):
    """train()'s minibatch loop captured WITH its RCCL collectives (the per-train()
    advantage-statistics all-reduce, every minibatch's gradient-span all-reduces forked onto RCCL's
    stream by the backward and joined before the optimizer step) replays bit for bit like the eager
    data-parallel loop of the same launches, over several iterations (eager, capture, replays) — at
    world size 1 over RCCL, the data-parallel path of every rank of a node.  The graph is really
    used (the train graph state records a captured graph, not a fallback)."""
    from puffer_phc_amd.clean_pufferl import core
    from puffer_phc_amd.policies import twin_mlp

    from test_gpu_train_graph import _iterate, _trainer

    old = twin_mlp.dp_mode()
    twin_mlp.set_dp_mode(mode)
    try:
        eager = _trainer()
        graphed = _trainer()
        for it in range(5):
            monkeypatch.setattr(core, "TRAIN_GRAPH", False)
            la = _iterate(*eager, seed=300 + it)
            monkeypatch.setattr(core, "TRAIN_GRAPH", True)
            lb = _iterate(*graphed, seed=300 + it)
            for k in la:
                assert (la[k] == lb[k]) or (la[k] != la[k] and lb[k] != lb[k]), (it, k, la[k], lb[k])
            pa = dict(eager[3].named_parameters())
            for n, p in graphed[3].named_parameters():
                assert torch.equal(p, pa[n]), (it, n)
            oa, ob = eager[1].optimizer, graphed[1].optimizer
            assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq), it
        st = graphed[1].__dict__.get("_train_graph")
        assert st is not None and st["graph"] is not None and not st["failed"], "the DP train graph was not captured"
    finally:
        twin_mlp.set_dp_mode(old)
