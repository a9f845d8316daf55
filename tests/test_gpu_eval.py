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
