"""Checkpoint layout (clean_pufferl/utils.py:18-42 of the reference): save_checkpoint writes
model_{epoch:06d}.pt = {config, state_dict} and trainer_state.pt; try_load_checkpoint reads both
back with torch.load(weights_only=True) — the files hold tensors, plain containers and the
TrainConfig as a dict, nothing that needs unpickling of arbitrary objects."""

import torch

from puffer_phc_amd.clean_pufferl.utils import save_checkpoint, try_load_checkpoint
from puffer_phc_amd.config import TrainConfig


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.SiLU(), torch.nn.Linear(16, 3))


def test_checkpoint_round_trip_weights_only(tmp_path):
    cfg = TrainConfig(data_dir=str(tmp_path), device_type="cpu")
    m = _model(0)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, eps=1e-5)
    for _ in range(2):
        opt.zero_grad()
        m(torch.randn(4, 8)).square().sum().backward()
        opt.step()
    save_checkpoint(m, opt, cfg, "exp", 7, 1234)
    m2 = _model(1)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-3, eps=1e-5)
    state = try_load_checkpoint(m2, opt2, cfg, "exp")
    assert state["global_step"] == 1234 and state["update"] == 7 and state["model_name"] == "model_000007.pt"
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert s1.keys() == s2.keys()
    for k in s1:
        assert torch.equal(s1[k]["exp_avg_sq"], s2[k]["exp_avg_sq"])
    assert try_load_checkpoint(m2, opt2, cfg, "missing") is None
