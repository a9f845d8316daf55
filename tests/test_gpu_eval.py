"""Eval path: EvalStats + eval_rollout over a motion set loaded through the
reference-style loader, on the HIP env (needs an MI355X).  compute_metrics_lite's own numbers are
parity-unpinned (smpl_sim is un-vendored); this checks the bookkeeping: every motion is played
exactly once in sequential batches, success / failed keys agree, MPJPE is the replay noise."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _clips(golden):
    g = golden("motion_lib")
    out = {}
    for i in range(int(g["num_input_motions"])):
        q, t = g[f"in_quat_{i}"], g[f"in_trans_{i}"]
        out[f"synth_{i:02d}"] = {"pose_quat_global": q, "root_trans_offset": torch.from_numpy(t),
                                 "pose_aa": np.zeros((q.shape[0], 72)), "fps": 30}
    return out


def _run(golden, sigma):
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.eval_stats import EvalStats, eval_rollout
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env = PHCPufferEnv(EnvConfig(num_envs=4, seed=2, replay_pos_sigma=sigma, min_motion_len=-1),
                       motion_data=_clips(golden))
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    stats = EvalStats(env, progress=False)
    n_motions = stats.num_unique_motions
    steps = eval_rollout(env, policy, stats, max_steps=5000)
    assert stats.results is not None, "eval did not finish"
    res = stats.update_env_and_close()
    assert not env.env.flag_im_eval and not env.env.flag_test  # back in training mode
    return env, stats, res, n_motions, steps


def test_eval_low_noise_all_succeed(golden):
    env, stats, res, n, steps = _run(golden, 0.02)
    rbm = stats.results_by_motion
    assert len(rbm["motion_length"]) == n == len(rbm["success"]) == len(rbm["played_steps"])
    assert res["eval/success_rate"] == 1.0 and len(stats.failed_keys) == 0
    # positions differ from the reference only by the replay noise (N(0, 0.02^2) per axis)
    assert 10.0 < res["eval/mpjpe_all"] < 60.0
    assert res["eval/mpjpel_all"] > 0 and res["eval/mpjpe_pa"] <= res["eval/mpjpel_all"] + 1e-6
    assert np.all(rbm["played_steps"] >= 1) and np.all(rbm["played_steps"] <= rbm["motion_length"])


def test_eval_metrics_recomputed_from_recorded_positions(golden):
    """The eval metrics are compute_metrics_lite over exactly the frames the reference keeps
    (scripts/train.py:150-201: per motion the first motion_num_steps - 1 steps of body_pos /
    body_pos_gt), and the per-step MPJPE extra is the mean joint distance of those two arrays
    (humanoid_phc.py:159-169).  Recomputed here with independent loops."""
    env, stats, res, n, steps = _run(golden, 0.02)
    pred, gt = stats.pred_pos_all[:n], stats.gt_pos_all[:n]
    lens = stats.results_by_motion["motion_length"]
    assert [p.shape[0] for p in pred] == [int(x) - 1 for x in lens]
    frames = []
    for p, g in zip(pred, gt):
        for t in range(p.shape[0]):
            frames.append(np.mean([np.linalg.norm(p[t, j] - g[t, j]) for j in range(p.shape[1])]) * 1000.0)
    np.testing.assert_allclose(res["eval/mpjpe_all"], np.mean(frames), rtol=1e-6)
    # the per-step MPJPE means of the batches (mpjpe_all, reported live) come from the same arrays
    means = [float(x) for b in stats.mpjpe_all for x in b][:n]
    np.testing.assert_allclose(means, [np.mean(np.linalg.norm(p - g, axis=2)) for p, g in zip(pred, gt)],
                               rtol=1e-5)


def test_eval_high_noise_reports_failures(golden):
    env, stats, res, n, steps = _run(golden, 0.6)
    succ = stats.results_by_motion["success"]
    assert res["eval/success_rate"] == pytest.approx(succ.mean())
    assert (~succ).sum() == len(stats.failed_keys) > 0


def _eval_shard_worker(rank, world, port, out_dir):
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import phc_amd_path

    phc_amd_path.register()
    import torch.distributed as dist

    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.eval_stats import EvalStats, eval_rollout
    from puffer_phc_amd.policies import PHCPolicy, Policy

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dict(np.load(os.path.join(root, "tests", "golden", "motion_lib.npz")))
        clips = {}
        for i in range(int(g["num_input_motions"])):
            q, t = g[f"in_quat_{i}"], g[f"in_trans_{i}"]
            clips[f"synth_{i:02d}"] = {"pose_quat_global": q, "root_trans_offset": torch.from_numpy(t),
                                       "pose_aa": np.zeros((q.shape[0], 72)), "fps": 30}

        def run(shard, seed):
            env = PHCPufferEnv(EnvConfig(num_envs=2, seed=seed, replay_pos_sigma=0.02, min_motion_len=-1),
                               motion_data=clips)
            torch.manual_seed(0)
            policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
            stats = EvalStats(env, progress=False, shard=shard)
            eval_rollout(env, policy, stats, max_steps=5000)
            assert stats.results is not None
            res = stats.update_env_and_close()
            lib = env.env._motion_lib
            return stats, res, lib

        stats, res, lib = run(None, 10 + rank)  # the DP shard of this rank
        out = {"ids": np.concatenate(stats.batch_ids).tolist(), "res": res,
               "len": stats.results_by_motion["motion_length"].tolist(),
               "played": stats.results_by_motion["played_steps"].tolist(),
               "succ": stats.results_by_motion["success"].tolist(),
               "prob": lib._sampling_prob.cpu().tolist(), "hist": lib._termination_history.cpu().tolist()}
        if rank == 0:  # the reference's single sequential pass over every motion, same process
            s1, r1, _ = run((0, 1), 10)
            out["single_len"] = s1.results_by_motion["motion_length"].tolist()
            out["single_succ"] = s1.results_by_motion["success"].tolist()
            out["single_ids"] = np.concatenate(s1.batch_ids).tolist()
        torch.save(out, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_eval_sharded_over_two_ranks(tmp_path):
    """§8e(5): two data-parallel ranks (gloo, one GPU) play disjoint motion batches (rank 0:
    batches 0 and 2, rank 1: batch 1 of 2 motions each), merge the per-motion results, and end
    with the same results, failed keys and PMCP sampling weights; the merged per-motion lengths
    and successes equal one rank's sequential pass over all 6 motions (low replay noise)."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_eval_shard_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["ids"] == [0, 1, 4, 5] and r1["ids"] == [2, 3]
    assert r0["single_ids"] == list(range(6))
    assert r0["res"] == r1["res"] and r0["len"] == r1["len"] and r0["succ"] == r1["succ"]
    assert r0["prob"] == r1["prob"] and r0["hist"] == r1["hist"]
    assert r0["len"] == r0["single_len"] and r0["succ"] == r0["single_succ"]
    assert r0["res"]["eval/success_rate"] == 1.0
