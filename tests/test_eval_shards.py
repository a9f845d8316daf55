"""Sharded evaluation merge (eval_stats.merge_eval_shards / summarize_eval / sync_sampling_state) on
CPU with gloo, world_size 2.

Each rank holds per-motion rows of a disjoint motion subset with different failures; after the
merge both ranks must see the whole-set result a single process would compute (success rate,
failed keys, frame-weighted metric means), and after the PMCP soft update
(motion_lib.py:472-500) identical sampling weights, even when one rank's weights had drifted.
"""

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_MOTIONS, N_ENVS = 10, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _motion_rows(ids, failed):
    """Per-motion rows as EvalStats.local_rows builds them, with deterministic fake metrics."""
    from puffer_phc_amd.eval_stats import COLS, METRICS

    rows = torch.zeros((N_MOTIONS, COLS), dtype=torch.float64)
    for m in ids:
        frames = 5 + m
        rows[m, 0] = 1
        rows[m, 1] = float(m in failed)
        rows[m, 2] = frames + 1
        rows[m, 3] = frames - (2 if m in failed else 0)
        for k in range(len(METRICS)):
            rows[m, 4 + 2 * k] = (m + 1) * (k + 1) * frames  # sum over frames
            rows[m, 5 + 2 * k] = frames  # frame count
    return rows


def _shard_ids(rank, world):
    """Batches of N_ENVS motions dealt round-robin (batch b on rank b % world), the last one cut
    at the set's end, as HumanoidPHC.toggle_eval_mode(shard=...) deals them."""
    ids = []
    for b in range(rank, -(-N_MOTIONS // N_ENVS), world):
        ids += list(range(b * N_ENVS, min((b + 1) * N_ENVS, N_MOTIONS)))
    return ids


FAILED = {0: {1, 7}, 1: {4}}


def _sampling_lib():
    from puffer_phc_amd.motion_lib import MotionLibBase

    ml = MotionLibBase.__new__(MotionLibBase)
    ml._device = "cpu"
    ml._motion_data_keys = np.array([f"m{i}" for i in range(N_MOTIONS)])
    ml._num_unique_motions = N_MOTIONS
    ml.setup_constants()
    return ml


def _worker(rank, world, port, root):
    import sys

    sys.path.insert(0, root)
    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd.eval_stats import merge_eval_shards, summarize_eval, sync_sampling_state

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _shard_ids(rank, world)
        assert set(mine).isdisjoint(_shard_ids(1 - rank, world))
        merged = merge_eval_shards(_motion_rows(mine, FAILED[rank]))
        res, terminated, lengths, played = summarize_eval(merged)
        # the single-process result over every motion
        every = _motion_rows(range(N_MOTIONS), FAILED[0] | FAILED[1])
        ref, ref_term, ref_len, ref_played = summarize_eval(every)
        assert res == ref
        assert np.array_equal(terminated, ref_term) and np.flatnonzero(terminated).tolist() == [1, 4, 7]
        assert np.array_equal(lengths, ref_len) and np.array_equal(played, ref_played)
        assert res["eval/success_rate"] == 0.7
        # overlapping shards are rejected
        try:
            merge_eval_shards(_motion_rows(range(N_MOTIONS), set()))
            raise AssertionError("overlap not detected")
        except RuntimeError:
            pass
        # PMCP soft weights from the merged failures, then rank 0's broadcast
        ml = _sampling_lib()
        keys = ml._motion_data_keys[terminated]
        ml.update_soft_sampling_weight(keys)
        if rank == 1:
            ml._sampling_prob[0] += 0.25  # a drifted replica
        sync_sampling_state(ml)
        expect = torch.zeros(N_MOTIONS)
        expect[[1, 4, 7]] = 1 / 3
        torch.testing.assert_close(ml._sampling_prob, expect)
        assert ml._termination_history.tolist() == [0, 1, 0, 0, 1, 0, 0, 1, 0, 0]
    finally:
        dist.destroy_process_group()


def test_eval_shards_merge_world2():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mp.spawn(_worker, args=(2, _free_port(), root), nprocs=2, join=True)


def test_shard_dealing_covers_every_motion_once():
    for world in (1, 2, 3, 5):
        ids = sorted(i for r in range(world) for i in _shard_ids(r, world))
        assert ids == list(range(N_MOTIONS)), world
