"""Data-parallel fused minibatch (policies/fused_ppo.py + distributed.FlatGrads overlap): two
ranks on one GPU over gloo (needs an MI355X), full PHCPolicy widths, 32768-row minibatches per
rank.  Each rank runs the fused PPO minibatch on its own data with the all-reduces started from
the backward (twin_mlp.GRAD_READY) and the gradients stored into a NaN-filled buffer (store_grads,
as the trainer runs it) — on the grouped weight-gradient path (default: every trunk
span after the grouped launch) and on the per-layer path (PHC_DP_PER_LAYER).  Checks:
  * the reduced flat gradient equals the mean of the two ranks' local gradients (fp32 a + b
    summed in either order is the same number: exact up to the final division, tol 1e-6);
  * it matches ONE rank's gradient over the union of both ranks' rows (65536): the per-row
    math is identical and 1/65536 = (1/32768) / 2 exactly, so only the fp32 summation order
    of the row reductions (weight / bias gradients, 32768 vs 65536 fp32 terms) differs:
    |diff| <= 1e-4 * max |grad| (measured 2.3e-5)."""

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


def _worker(rank, world, port, out_dir, mode):
    import sys

    sys.path.insert(0, ROOT)
    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd import distributed as D
    from puffer_phc_amd.clean_pufferl.ppo_loss import ppo_coefs
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy, twin_mlp
    from puffer_phc_amd.policies.fused_ppo import fused_ppo_loss

    twin_mlp.set_dp_mode(mode)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = "cuda:0"
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(_Env())).to(dev)  # the reference's full widths
        pol = policy.policy
        fg = D.FlatGrads(policy.parameters(), order=pol.grad_ready_order())
        M = 32768

        def data(r):
            g = torch.Generator(device=dev).manual_seed(10 + r)
            return (torch.randn((M, 934), device=dev, generator=g), 0.1 * torch.randn((M, 69), device=dev, generator=g),
                    torch.randn(M, device=dev, generator=g) + 200.0, torch.randn(M, device=dev, generator=g),
                    torch.randn(M, device=dev, generator=g), torch.randn(M, device=dev, generator=g))

        ms = torch.tensor([0.0, 1.0], device=dev)
        coefs = ppo_coefs(TrainConfig(), pol.soft_bound)

        def backward(batch, overlap):
            obs, atn, old_lp, adv, val, ret = batch
            if overlap:  # as clean_pufferl.core.train runs it: gradients stored, the buffer not zeroed
                fg.fill_grads_(float("nan"))
            else:
                fg.zero()
            with torch.autocast("cuda", dtype=torch.float16):
                xh = pol.obs_half_input(obs)
                loss, _ = fused_ppo_loss(pol, xh, atn, old_lp, adv, ms, val, ret, coefs, store_grads=overlap)
            if overlap:
                fg.overlap_begin()
            (loss * 64.0).backward()
            if overlap:
                fg.overlap_finish()
            torch.cuda.synchronize()
            return fg.flat.detach().clone()

        mine = data(rank)
        local = backward(mine, False)
        dp = backward(mine, True)
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        ref = (gathered[0] + gathered[1]) / world
        res = {"err": float((dp - ref).abs().max()), "scale": float(ref.abs().max()),
               "nonzero": int((local != 0).sum())}
        if rank == 0:
            both = [data(0), data(1)]
            union = backward(tuple(torch.cat([a, b]) for a, b in zip(*both)), False)
            res["union_err"] = float((dp - union).abs().max())
            res["union_scale"] = float(union.abs().max())
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["grouped", "per_layer", "split"])
def test_dp_gradient_matches_mean_and_union(tmp_path, mode):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), mode), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["nonzero"] > 1000
        assert res["err"] <= 1e-6 * max(res["scale"], 1.0), res
        if r == 0:
            assert res["union_err"] <= 1e-4 * res["union_scale"], res
