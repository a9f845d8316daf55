"""train()'s advantage / minibatch-layout pass replayed from a captured hipGraph
(clean_pufferl.core._compute_advantages_train) against the eager compute_advantages on the same
buffers, over several rollouts: the first call runs eagerly, the second captures, later ones replay.
Every output the minibatch loop reads must be bit-identical (reference: core.py:212-260)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FIELDS = ("b_obs_half", "b_actions", "b_logprobs", "b_values", "b_advantages", "b_returns", "returns",
          "sorted_values", "b_dones", "b_truncated", "b_idxs_flat", "b_adv_ms", "ev_pair")


@pytest.fixture(scope="module")
def trainer():
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 90, seed=7, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=4), motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    return clean_pufferl, comps, info, policy


def _snapshot(exp):
    out = {}
    for k in FIELDS:
        v = getattr(exp, k, None)
        out[k] = None if v is None else v.detach().clone()
    return out


def test_graphed_advantages_match_eager(trainer):
    cp, comps, info, policy = trainer
    core = cp.core
    assert core.ADV_GRAPH
    exp = comps.experience
    for it in range(4):
        cp.evaluate(comps, info)
        policy.policy.update_obs_rms(exp.obs)
        got_adv = core._compute_advantages_train(comps, info).clone()
        got = _snapshot(exp)
        ref_adv = core.compute_advantages(comps, info)  # eager on the same buffers
        ref = _snapshot(exp)
        torch.cuda.synchronize()
        assert torch.equal(got_adv, ref_adv), it
        for k in FIELDS:
            if ref[k] is None:
                assert got[k] is None, (it, k)
            else:
                assert torch.equal(got[k], ref[k]), (it, k)
        # the eager call above re-pointed the experience attributes; the graphed path must
        # restore its own outputs on the next call (re-captured when the attributes moved)
    st = getattr(comps, "_adv_graph", None)
    assert st is not None and not st["failed"]
