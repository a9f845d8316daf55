"""Data-parallel collectives (distributed.py) on CPU with gloo, world_size 2 (the RunningNorm
moments exchange runs on the device: tests/test_gpu_rccl.py).

Each check compares the 2-rank result with the single-process computation over the union of
both ranks' data (what one GPU would have computed on the whole global batch)."""

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data(rank, n=64, f=12):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, f, generator=g) * (1 + rank) + rank, torch.randn(n, 1, generator=g)


def _worker(rank, world, port, root):
    import sys

    sys.path.insert(0, root)
    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # (5) parameter broadcast: rank 1 starts from a different init
        torch.manual_seed(rank)
        net = torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.SiLU(), torch.nn.Linear(16, 1))
        D.broadcast_params(net)
        torch.manual_seed(0)
        ref_net = torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.SiLU(), torch.nn.Linear(16, 1))
        for a, b in zip(net.parameters(), ref_net.parameters()):
            assert torch.equal(a, b)
        # (1) flat-bucket gradient all-reduce == gradient of the mean loss over both ranks
        fg = D.FlatGrads(net.parameters(), bucket_bytes=256)  # force several buckets
        x, y = _data(rank)
        fg.zero()
        ((net(x) - y) ** 2).mean().backward()
        fg.allreduce_mean()
        xs = torch.cat([_data(r)[0] for r in range(world)])
        ys = torch.cat([_data(r)[1] for r in range(world)])
        ref_net.zero_grad()
        ((ref_net(xs) - ys) ** 2).mean().backward()
        for p, q in zip(net.parameters(), ref_net.parameters()):
            torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-5)
        # (1b) overlapped all-reduce: FlatGrads laid out in a given order, groups reported
        # ready during the "backward" (twin_mlp.GRAD_READY), the rest at overlap_finish
        from puffer_phc_amd.policies import twin_mlp

        ps = list(net.parameters())
        fo = D.FlatGrads(ps, order=[ps[2], ps[3], ps[0]])  # layer 2 (w, b), then layer 1's weight
        assert fo.params[:3] == [ps[2], ps[3], ps[0]] and fo.params[3] is ps[1]
        fo.zero()
        ((net(x) - y) ** 2).mean().backward()
        fo.overlap_begin()
        assert twin_mlp.GRAD_READY is not None
        twin_mlp.GRAD_READY([ps[2], ps[3]])
        fo.overlap_finish()
        assert twin_mlp.GRAD_READY is None
        for p, q in zip(net.parameters(), ref_net.parameters()):
            torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-5)
        # (2) global advantage statistics
        adv = x[:, 0].contiguous()
        m, s = D.global_mean_std(adv)
        allv = xs[:, 0]
        torch.testing.assert_close(m, allv.mean(), atol=1e-6, rtol=1e-6)
        torch.testing.assert_close(s, allv.std(), atol=1e-6, rtol=1e-6)
        # (4) scalar reductions
        t = torch.tensor([float(rank + 1)])
        D.allreduce_max_(t)
        assert float(t) == world
        # (6) loop-control values agree across ranks: ranks with different
        # truncation patterns store different mask-true row counts, and their minibatches give
        # different approx_kl; the trainer's global_step and target_kl test use these reductions
        from puffer_phc_amd.clean_pufferl import core as C

        counts = [131072 - 17, 131072 - 905]
        assert C._global_count(counts[rank], "cpu") == sum(counts)
        kls = [0.004, 0.03]
        kl = C._global_mean(torch.tensor(kls[rank]))
        assert abs(kl - sum(kls) / world) < 1e-8
        # target_kl = 0.02: rank 0 alone would continue and rank 1 alone would stop; both stop
        # together or continue together on the shared mean
        decision = torch.tensor([float(kl > 0.02)])
        both = decision.clone()
        D.allreduce_sum_(both)
        assert float(both) in (0.0, float(world))
        # (7) the train graph's capture outcome is agreed over the ranks (core._all_ranks_agree): a rank
        # whose capture failed makes every rank stay eager (a lone eager rank would issue the graph's
        # collectives alone)
        assert C._all_ranks_agree(True, "cpu") is True
        assert C._all_ranks_agree(rank == 0, "cpu") is False
    finally:
        dist.destroy_process_group()


def test_collectives_world2():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mp.spawn(_worker, args=(2, _free_port(), root), nprocs=2, join=True)


L_TRUNK = 5  # twin trunk depth of the test model (PHCPolicy: 6)


def _twin_model(seed):
    """A twin-trunk stand-in with PHCPolicy's parameter grouping: layer l of the trunk owns
    [actor W, actor b, critic W, critic b]; a tail (value / mu heads) follows."""
    torch.manual_seed(seed)
    dims = [12, 24, 20, 16, 16, 8]
    actor = torch.nn.ModuleList([torch.nn.Linear(dims[i], dims[i + 1]) for i in range(L_TRUNK)])
    critic = torch.nn.ModuleList([torch.nn.Linear(dims[i], dims[i + 1]) for i in range(L_TRUNK)])
    mu, value = torch.nn.Linear(dims[-1], 3), torch.nn.Linear(dims[-1], 1)
    trunk = [p for l in range(L_TRUNK) for p in (actor[l].weight, actor[l].bias, critic[l].weight, critic[l].bias)]
    tail = [mu.weight, mu.bias, value.weight, value.bias]

    def loss(x, y):
        a = c = x
        for l in range(L_TRUNK):
            a, c = torch.nn.functional.silu(actor[l](a)), torch.nn.functional.silu(critic[l](c))
        return ((mu(a) - y) ** 2).mean() + ((value(c) - y[:, :1]) ** 2).mean()

    return trunk, tail, loss


def _ready_sequence(mode, trunk, tail):
    """The GRAD_READY calls the fused backward makes in each data-parallel mode (fused_ppo.py:95-98 for
    the tail; twin_mlp.py mfma_trunk_backward for the trunk): grouped = one call with every trunk
    layer, last first; per_layer = one call per layer as its gradient lands; split = the last three
    layers, then (cumulatively) all of them."""
    L = len(trunk) // 4
    layers = lambda lo: [p for l in range(L - 1, lo - 1, -1) for p in trunk[4 * l:4 * l + 4]]  # noqa: E731
    seq = [tail]
    if mode == "grouped":
        seq.append(layers(0))
    elif mode == "per_layer":
        seq += [trunk[4 * l:4 * l + 4] for l in range(L - 1, -1, -1)]
    else:
        seq += [layers(max(L - 3, 0)), layers(0)]
    return seq


def _dp_modes_worker(rank, world, port, root):
    import sys

    sys.path.insert(0, root)
    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd import distributed as D
    from puffer_phc_amd.policies import twin_mlp

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7 + rank)
        x, y = torch.randn(32, 12, generator=g), torch.randn(32, 3, generator=g)
        xs = [torch.empty_like(x) for _ in range(world)]
        ys = [torch.empty_like(y) for _ in range(world)]
        dist.all_gather(xs, x)
        dist.all_gather(ys, y)
        rt, rtail, rloss = _twin_model(0)
        rloss(torch.cat(xs), torch.cat(ys)).backward()  # the mean loss over the union, one process
        want = [p.grad.clone() for p in rtail + rt]
        for mode in twin_mlp.DP_MODES:
            twin_mlp.set_dp_mode(mode)
            assert twin_mlp.dp_mode() == mode
            trunk, tail, loss = _twin_model(0)
            order = tail + [p for l in range(L_TRUNK - 1, -1, -1) for p in trunk[4 * l:4 * l + 4]]
            fg = D.FlatGrads(trunk + tail, order=order)
            fg.zero()
            loss(x, y).backward()  # the per-rank gradient (the mean over this rank's rows)
            fg.overlap_begin()
            seq = _ready_sequence(mode, trunk, tail)
            for group in seq:
                twin_mlp.GRAD_READY(group)
            # every group is one contiguous span of the flat buffer (alignment gaps bridged): one
            # all-reduce per call, none for parameters an earlier call already reduced
            assert len(fg._works) == len(seq), (mode, len(fg._works))
            fg.overlap_finish()
            for p, w in zip(tail + trunk, want):
                torch.testing.assert_close(p.grad, w, atol=1e-6, rtol=1e-5, msg=mode)
        twin_mlp.set_dp_mode("grouped")
    finally:
        dist.destroy_process_group()


def test_dp_modes_world2():
    """grouped / per_layer / split: each mode's readiness calls all-reduce every gradient exactly once
    and leave every rank with the gradient of the mean loss over both ranks' rows."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mp.spawn(_dp_modes_worker, args=(2, _free_port(), root), nprocs=2, join=True)
