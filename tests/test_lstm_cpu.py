"""N4: the LSTM policies and the restated pufferlib recurrent wrappers (CPU; no kernel calls).
pufferlib is absent, so parity with its LSTMWrapper / RecurrentPolicy is unpinned; these checks pin
the properties the trainer relies on: a [B, T] segment through the LSTM equals stepping it T times
with the carried (h, c); log-probabilities are those of the Normal head; both call spellings of the
reference (policy(obs, (h, c)) and policy(obs, info=state, action=atn)) agree; the parameter count
of LSTMActorPolicy matches the reference's own note (lstm_policy.py:90, "13.5M params")."""

from types import SimpleNamespace

import numpy as np
import pytest
import torch
from torch import nn

from puffer_phc_amd.policies import LSTMActorPolicy, LSTMCriticPolicy, Recurrent, RecurrentPolicy


class Box:
    def __init__(self, n, high=1.0):
        self.shape = (n,)
        self.high = np.full(n, high, np.float32)


def _env():
    return SimpleNamespace(single_observation_space=Box(934, np.inf), single_action_space=Box(69),
                           amp_observation_space=None)


def _policy(cls, seed=0):
    torch.manual_seed(seed)
    inner = cls(_env())
    inner.obs_norm = nn.Identity()  # the HIP RunningNorm needs a device; the statistics are not under test
    return RecurrentPolicy(Recurrent(_env(), inner))


@pytest.mark.parametrize("cls", [LSTMCriticPolicy, LSTMActorPolicy])
def test_segment_equals_stepping(cls):
    pol = _policy(cls)
    B, T = 3, 5
    x = torch.randn(B, T, 934)
    atn = torch.randn(B, T, 69) * 0.1
    with torch.no_grad():
        _, lp_seq, ent_seq, v_seq, (h, c) = pol(x, None, action=atn)
        state = None
        lps, vs = [], []
        for t in range(T):
            _, lp, _, v, state = pol(x[:, t], state, action=atn[:, t])
            lps.append(lp)
            vs.append(v)
    lp_step = torch.stack(lps, 1).reshape(-1)  # rows in (b, t) order, as the segment's
    v_step = torch.stack(vs, 1).reshape(-1)
    torch.testing.assert_close(lp_seq, lp_step, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(v_seq.reshape(-1), v_step, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(h, state[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(c, state[1], rtol=1e-5, atol=1e-6)
    assert h.shape == (1, B, 512) and lp_seq.shape == (B * T,) and ent_seq.shape == (B * T,)


def test_logprob_is_the_normal_heads_and_call_spellings_agree():
    pol = _policy(LSTMCriticPolicy, seed=1)
    x = torch.randn(4, 934)
    state = (torch.randn(1, 4, 512) * 0.1, torch.randn(1, 4, 512) * 0.1)
    with torch.no_grad():
        a, lp, ent, v, st = pol(x, state)
        a2, lp2, ent2, v2, st2 = pol(x, info=state, action=a)
        probs, _, _ = pol.policy(x, state)
    torch.testing.assert_close(lp, probs.log_prob(a).sum(1))
    torch.testing.assert_close(lp2, lp)
    torch.testing.assert_close(v2, v)
    torch.testing.assert_close(ent, probs.entropy().sum(1))
    assert torch.equal(st[0], st2[0]) and isinstance(pol.lstm, nn.LSTM) and pol.lstm.hidden_size == 512
    # deterministic action: std clamped to 1e-6 (lstm_policy.py:74-75)
    pol.policy.set_deterministic_action(True)
    with torch.no_grad():
        a3, _, _, _, _ = pol(x, state)
    assert float((a3 - probs.loc).abs().max()) < 1e-4


def test_lstm_init_and_parameter_count():
    pol = _policy(LSTMActorPolicy)
    lstm = pol.lstm
    assert float(lstm.bias_ih_l0.detach().abs().max()) == 0.0 and float(lstm.bias_hh_l0.detach().abs().max()) == 0.0
    for w in (lstm.weight_ih_l0, lstm.weight_hh_l0):  # orthogonal, gain 1: rows orthonormal (4H x H)
        g = w.detach().t() @ w.detach()
        torch.testing.assert_close(g, torch.eye(512), atol=1e-4, rtol=0)
    n = sum(p.numel() for p in pol.parameters() if p.requires_grad)
    assert abs(n - 13.5e6) < 0.1e6, n  # "13.5M params" (lstm_policy.py:90)
    assert pol.policy.mean_bound_loss is None and pol.policy.soft_bound == pytest.approx(0.9)
