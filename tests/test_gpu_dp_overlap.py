"""Data-parallel fused minibatch (policies/fused_ppo.py + distributed.FlatGrads overlap): two
ranks on one GPU over gloo (needs an MI355X).  Each rank runs the fused PPO minibatch on its
own data; with the per-layer all-reduces started during the backward (twin_mlp.GRAD_READY) the
final flat gradient must equal the mean of the two ranks' local gradients (fp32 a + b summed in
either order is the same number: exact up to the final division, tolerance 1e-6)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = None


def _worker(rank, world, port, out_dir):
    import sys

    sys.path.insert(0, ROOT)
    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd import distributed as D
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = "cuda:0"
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(_Env(), hidden_size=512, layer_sizes=(256, 128))).to(dev)
        pol = policy.policy
        fg = D.FlatGrads(policy.parameters(), order=pol.grad_ready_order())
        g = torch.Generator(device=dev).manual_seed(10 + rank)
        M = 1024
        obs = torch.randn((M, 934), device=dev, generator=g)
        atn = 0.1 * torch.randn((M, 69), device=dev, generator=g)
        old_lp = torch.randn(M, device=dev, generator=g) + 200.0
        adv = torch.randn(M, device=dev, generator=g)
        val = torch.randn(M, device=dev, generator=g)
        ret = torch.randn(M, device=dev, generator=g)
        ms = torch.tensor([0.0, 1.0], device=dev)
        coefs = ppo_coefs(TrainConfig(), pol.soft_bound)

        def backward(overlap):
            fg.zero()
            with torch.autocast("cuda", dtype=torch.float16):
                xh = pol.obs_half_input(obs)
                loss, _ = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, coefs)
            if overlap:
                fg.overlap_begin()
            (loss * 64.0).backward()
            if overlap:
                fg.overlap_finish()
            torch.cuda.synchronize()
            return fg.flat.detach().clone()

        local = backward(False)
        dp = backward(True)
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        ref = (gathered[0] + gathered[1]) / world
        err = float((dp - ref).abs().max())
        scale = float(ref.abs().max())
        torch.save({"err": err, "scale": scale, "nonzero": int((local != 0).sum())},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_matches_mean_of_local_gradients(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["nonzero"] > 1000
        assert res["err"] <= 1e-6 * max(res["scale"], 1.0), res
