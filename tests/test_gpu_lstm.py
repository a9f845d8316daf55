"""N4 on the device: clean_pufferl with an LSTM policy under the Recurrent wrapper — the rollout
carries each env's (h, c) in the experience buffers and zeroes it for envs that reset (core.py:
149-160); the update runs [minibatch_rows, bptt] segments through the LSTM with the state carried
from minibatch to minibatch within an epoch (core.py:268-289); the eval rollout carries and resets
the state (scripts/train.py:392-429)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("name", ["LSTMCriticPolicy", "LSTMActorPolicy"])
def test_ppo_iteration_with_recurrent_policy(name):
    from puffer_phc_amd import clean_pufferl, policies
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 60, seed=5, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=3), motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    torch.manual_seed(0)
    inner = getattr(policies, name)(env)
    policy = policies.RecurrentPolicy(policies.Recurrent(env, inner)).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("lstm", cfg, env.cfg, env, policy)
    exp = comps.experience
    assert exp.lstm_h is not None and exp.lstm_h.shape == (1, 64, 512)
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    clean_pufferl.evaluate(comps, info)
    assert info.global_step >= cfg.batch_size
    assert torch.isfinite(exp.lstm_h).all() and float(exp.lstm_h.abs().sum()) > 0
    assert torch.isfinite(exp.obs).all() and torch.isfinite(exp.logprobs).all()
    inner.update_obs_rms(exp.obs)
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.approx_kl, losses.entropy]).all()
    moved = [k for k, v in policy.named_parameters() if v.requires_grad and not torch.equal(before[k], v)]
    assert any("recurrent" in k for k in moved) and any("actor_mlp" in k for k in moved)


def test_lstm_state_resets_for_done_envs():
    """The rollout zeroes (h, c) of envs that terminated or truncated before their next forward."""
    from puffer_phc_amd import clean_pufferl, policies
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(32, 8, 12, seed=6, device=DEV)  # short clips: resets within the rollout
    env = PHCPufferEnv(EnvConfig(num_envs=32, seed=4), motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    torch.manual_seed(1)
    policy = policies.RecurrentPolicy(policies.Recurrent(env, policies.LSTMCriticPolicy(env))).to(DEV)
    cfg = TrainConfig(batch_size=32 * 16, minibatch_size=128, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("lstm2", cfg, env.cfg, env, policy)
    exp = comps.experience
    seen = []
    orig = policy.forward

    def spy(x, state=None, action=None, info=None):
        if state is not None:
            seen.append((state[0].detach().clone(), env.terminals.clone() | env.truncations.clone()))
        return orig(x, state, action, info)

    policy.forward = spy
    clean_pufferl.evaluate(comps, info)
    policy.forward = orig
    resets = [(h, d) for h, d in seen[1:] if bool(d.any())]
    assert resets, "no env reset during the rollout"
    for h, d in resets:
        assert float(h[:, d].abs().max()) == 0.0  # the state handed to the policy was zeroed
        assert float(h[:, ~d].abs().max()) > 0.0
