"""N4 parity: the LSTM policies (puffer-phc_amd/policies/lstm_policy.py) against the reference's own
modules (puffer_phc/policies/lstm_policy.py:25-148), pinned by tests/golden/lstm_policy.npz and
lstm_state_dict_keys.tsv (tests/golden/make_golden.py `gen_lstm`: the reference's classes imported
with pufferlib.models.LSTMWrapper stubbed, weights set by `lstm_fill`, fixed inputs).

Checked: state-dict keys, shapes, dtypes and the trainable parameter count; encode_observations and
decode_actions (Normal mean / std, value; the mean bound loss in training mode) on the same weights
and inputs, in eval and training mode.  CPU: the HIP RunningNorm is replaced by the oracle's
restatement of the reference's RunningNorm.forward (oracle/phc_oracle.py rms_normalize) over the
same buffers; GPU: the shipped HIP RunningNorm.  Tolerance 1e-5 (fp32 GEMM reassociation).
The pufferlib LSTMWrapper / RecurrentPolicy wrappers themselves stay unpinned (pufferlib absent)."""

import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import phc_oracle as O
from puffer_phc_amd.policies import LSTMActorPolicy, LSTMCriticPolicy

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CLASSES = {"critic": LSTMCriticPolicy, "actor": LSTMActorPolicy}


class Box:
    def __init__(self, n, high=1.0):
        self.shape = (n,)
        self.high = np.full(n, high, np.float32)


def _env():
    return SimpleNamespace(single_observation_space=Box(934, np.inf), single_action_space=Box(69),
                           amp_observation_space=None)


def lstm_fill(module):
    """The rule of make_golden.lstm_fill (restated: the generator imports the reference)."""
    with torch.no_grad():
        for i, (k, v) in enumerate(module.state_dict().items()):
            g = torch.Generator().manual_seed(1000 + i)
            x = torch.randn(v.shape, generator=g, dtype=torch.float64)
            if k.endswith("running_var"):
                x = x.abs() + 0.5
            elif k.endswith("count"):
                x = torch.full(v.shape, 10.0, dtype=torch.float64)
            elif k.endswith("sigma"):
                x = x * 0.1 - 1.0
            else:
                x = x * (0.5 / max(1, v.shape[-1]) ** 0.5)
            v.copy_(x.to(v.dtype))


class _OracleNorm(torch.nn.Module):
    """RunningNorm.forward of the reference (running_norm.py:15-20) via the oracle, on the port's
    own buffers."""

    def __init__(self, rn):
        super().__init__()
        self.rn = rn

    def forward(self, x):
        y = O.rms_normalize(x.numpy(), self.rn.running_mean.numpy(), self.rn.running_var.numpy(),
                            self.rn.epsilon, self.rn.clip)
        return torch.from_numpy(np.asarray(y, np.float32))


def _keys():
    rows = {}
    with open(os.path.join(GOLD, "lstm_state_dict_keys.tsv")) as f:
        for line in f:
            name, key, shape, dtype = line.rstrip("\n").split("\t")
            rows.setdefault(name, []).append((key, shape, dtype))
    return rows


@pytest.mark.parametrize("name", ["critic", "actor"])
def test_lstm_state_dict_matches_reference(name):
    pol = CLASSES[name](_env(), hidden_size=512)
    want = _keys()[name]
    got = [(k, "x".join(map(str, v.shape)), str(v.dtype)) for k, v in pol.state_dict().items()]
    n_train = sum(p.numel() for p in pol.parameters() if p.requires_grad)
    got.append(("#trainable", str(n_train), "-"))
    assert got == want


def _check(pol, g, name, device):
    obs = torch.from_numpy(g["obs"]).to(device)
    hid = torch.from_numpy(g["hidden_in"]).to(device)
    with torch.no_grad():
        for training in (False, True):
            pol.train(training)
            tag = f"{name}_{'train' if training else 'eval'}"
            h, _ = pol.encode_observations(obs)
            probs, value = pol.decode_actions(hid)
            for k, v in (("encoded", h), ("mu", probs.mean), ("std", probs.stddev), ("value", value)):
                np.testing.assert_allclose(v.float().cpu().numpy(), g[f"{tag}_{k}"], atol=1e-5, rtol=1e-5,
                                           err_msg=f"{tag}_{k}")
            if training:
                np.testing.assert_allclose(float(pol.mean_bound_loss), float(g[f"{tag}_bound"]), atol=1e-6,
                                           rtol=1e-5)


@pytest.mark.parametrize("name", ["critic", "actor"])
def test_lstm_forward_matches_reference_cpu(name):
    g = dict(np.load(os.path.join(GOLD, "lstm_policy.npz")))
    pol = CLASSES[name](_env(), hidden_size=512)
    lstm_fill(pol)
    pol.obs_norm = _OracleNorm(pol.obs_norm)
    _check(pol, g, name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["critic", "actor"])
def test_lstm_forward_matches_reference_gpu(name):
    prec = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")  # the trainer sets "high" (core.py:38); fp32 here
    try:
        g = dict(np.load(os.path.join(GOLD, "lstm_policy.npz")))
        pol = CLASSES[name](_env(), hidden_size=512)
        lstm_fill(pol)
        _check(pol.to("cuda:0"), g, name, "cuda:0")
    finally:
        torch.set_float32_matmul_precision(prec)
