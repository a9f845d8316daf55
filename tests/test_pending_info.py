"""PendingInfo (clean_pufferl/env.py): mean_and_log()'s statistics arrive by a non-blocking copy; any
read of the info waits on the copy's event once and builds the same dict the blocking read built
(the reference's PHCPufferEnv.mean_and_log, clean_pufferl/env.py:145-188), updating the env's episode
count once.  The rollout loop reads the step infos after its loop (clean_pufferl/core.py)."""

import types

import numpy as np
import torch

from puffer_phc_amd.clean_pufferl.env import PendingInfo, PHCPufferEnv


class _Event:
    def __init__(self):
        self.waits = 0

    def synchronize(self):
        self.waits += 1


def _env(log_interval=32, n=4096):
    e = types.SimpleNamespace(cfg=types.SimpleNamespace(log_interval=log_interval), num_agents=n, episode_count=0)
    e._resolve_info = types.MethodType(PHCPufferEnv._resolve_info, e)
    return e


def _sums(n_ep):
    s = torch.zeros(16, dtype=torch.float64)
    s[:5] = torch.tensor([1000.0, 2000.0, 3000.0, 4000.0, 5000.0], dtype=torch.float64)
    s[5:9] = torch.tensor([50.0, 600.0, n_ep, 2.0], dtype=torch.float64)
    return s


def test_pending_info_resolves_once_to_the_blocking_dict():
    env, ev = _env(), _Event()
    info = PendingInfo(env, _sums(10.0), ev)
    assert ev.waits == 0 and env.episode_count == 0  # nothing read yet
    assert "rew_body_pos" in info
    d = dict(info)
    denom = 32 * 4096
    np.testing.assert_allclose([d["rew_body_pos"], d["rew_power"]], [1000.0 / denom, 5000.0 / denom])
    np.testing.assert_allclose([d["episode_return"], d["episode_length"], d["truncated_rate"]], [5.0, 60.0, 0.2])
    assert ev.waits == 1 and env.episode_count == 10
    list(info.items()), len(info), repr(info), info["rew_body_rot"]
    assert ev.waits == 1 and env.episode_count == 10  # resolved once


def test_pending_info_without_episodes_has_no_episode_keys():
    env = _env()
    info = PendingInfo(env, _sums(0.0), _Event())
    assert set(info) == {"rew_body_pos", "rew_body_rot", "rew_lin_vel", "rew_ang_vel", "rew_power"}
    assert env.episode_count == 0


def test_pending_info_reads_a_snapshot_of_the_buffer():
    """The pinned buffer is reused round-robin: the resolved values must not follow later writes."""
    env, buf = _env(), _sums(4.0)
    info = PendingInfo(env, buf, _Event())
    first = dict(info)
    buf.zero_()
    assert dict(info) == first


def test_flush_counts_unread_infos_once():
    """PHCPufferEnv.flush resolves every outstanding ring slot: episodes of infos nobody read are
    counted, each once; a second flush (or a later read) adds nothing."""
    env = _env()
    env._info_ring = [[None, None] for _ in range(4)]
    evs = [_Event() for _ in range(3)]
    infos = [PendingInfo(env, _sums(float(k + 1)), evs[k]) for k in range(3)]
    for k, info in enumerate(infos):
        env._info_ring[k][1] = info
    dict(infos[1])  # one read already
    assert env.episode_count == 2
    PHCPufferEnv.flush(env)
    assert env.episode_count == 1 + 2 + 3 and [e.waits for e in evs] == [1, 1, 1]
    PHCPufferEnv.flush(env)
    dict(infos[0])
    assert env.episode_count == 6 and [e.waits for e in evs] == [1, 1, 1]
