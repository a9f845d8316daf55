"""Policy surface and checkpoint layout vs the reference (CPU; no kernel calls)."""

import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from puffer_phc_amd.policies import PHCPolicy, Policy

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "state_dict_keys.tsv")


class Box:
    def __init__(self, n, high=1.0):
        self.shape = (n,)
        self.high = np.full(n, high, np.float32)


def _env(amp):
    return SimpleNamespace(single_observation_space=Box(934, np.inf), single_action_space=Box(69),
                           amp_observation_space=Box(1960, np.inf) if amp else None)


@pytest.mark.parametrize("amp", [False, True])
def test_state_dict_keys_shapes_match_reference(amp):
    rows = [line.rstrip("\n").split("\t") for line in open(GOLDEN)]
    ref = {k: s for a, k, s, _ in rows if a == str(int(amp)) and not k.startswith("#")}
    n_ref = [int(s) for a, k, s, _ in rows if a == str(int(amp)) and k == "#trainable"][0]
    pol = Policy(PHCPolicy(_env(amp), hidden_size=512, layer_sizes=(2048, 1536, 1024, 1024, 512)))
    ours = {k: "x".join(map(str, v.shape)) for k, v in pol.state_dict().items()}
    assert list(ours.keys()) == list(ref.keys())
    assert ours == ref
    assert sum(p.numel() for p in pol.policy.parameters() if p.requires_grad) == n_ref


def test_orthogonal_init_and_sigma():
    pol = PHCPolicy(_env(False))
    w = pol.actor_mlp[0].weight.detach()
    # orthogonal rows scaled by sqrt(2): W W^T = 2 I for a wide matrix (2048 x 934 -> columns orthogonal)
    g = w.T @ w
    assert torch.allclose(g, 2 * torch.eye(934), atol=1e-3)
    assert torch.all(pol.sigma == -2.9) and not pol.sigma.requires_grad
    wm = pol.mu[0].weight.detach()
    assert torch.allclose(wm @ wm.T, 1e-4 * torch.eye(69), atol=1e-6)


def test_bound_loss_matches_reference_formula():
    pol = PHCPolicy(_env(False))
    mu = torch.tensor([[-2.0, -0.9, 0.0, 0.95, 1.5]])
    sb = 0.9
    ref = torch.where(mu > sb, (mu - sb) ** 2, torch.where(mu < -sb, (mu + sb) ** 2, torch.zeros_like(mu))).mean()
    assert torch.allclose(pol.bound_loss(mu), ref)


def test_checkpoint_layout(tmp_path):
    from puffer_phc_amd.clean_pufferl.utils import save_checkpoint
    from puffer_phc_amd.config import TrainConfig

    pol = Policy(PHCPolicy(_env(False)))
    opt = torch.optim.Adam(pol.parameters(), lr=1e-4, eps=1e-5)
    cfg = TrainConfig(data_dir=str(tmp_path), device_type="cpu")
    path = save_checkpoint(pol, opt, cfg, "exp", 7, 1234)
    assert os.path.basename(path) == "model_000007.pt"
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"config", "state_dict"} and ck["config"]["batch_size"] == 131072
    st = torch.load(os.path.join(tmp_path, "exp", "trainer_state.pt"), weights_only=True)
    assert st["update"] == 7 and st["global_step"] == 1234 and st["model_name"] == "model_000007.pt"
    assert set(st) == {"optimizer_state_dict", "global_step", "agent_step", "update", "model_name", "exp_id"}


def test_cli_dotted_flags():
    from puffer_phc_amd import cli
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from dataclasses import dataclass, field

    @dataclass
    class App:
        mode: str = "train"
        env: EnvConfig = field(default_factory=EnvConfig)
        train: TrainConfig = field(default_factory=TrainConfig)

    a = cli.parse(App(), ["--env.num-envs", "64", "--train.batch-size", "1024", "--env.use-amp-obs",
                          "--train.no-norm-adv", "--mode", "play", "--train.target-kl", "0.05"])
    assert a.env.num_envs == 64 and a.train.batch_size == 1024 and a.env.use_amp_obs is True
    assert a.train.norm_adv is False and a.mode == "play" and a.train.target_kl == 0.05
