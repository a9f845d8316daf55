"""Checkpoint layout and seeding (puffer_phc/clean_pufferl/utils.py:18-80)."""

import os
import random
from dataclasses import asdict, is_dataclass

import numpy as np
import torch


def save_checkpoint(uncompiled_policy, optimizer, train_cfg, exp_id, epoch, global_step):
    """experiments/<exp_id>/model_{epoch:06d}.pt = {config, state_dict} and an atomically
    renamed trainer_state.pt (utils.py:18-42)."""
    path = os.path.join(train_cfg.data_dir, exp_id)
    os.makedirs(path, exist_ok=True)
    model_name = f"model_{epoch:06d}.pt"
    model_path = os.path.join(path, model_name)
    if os.path.exists(model_path):
        return model_path
    cfg = asdict(train_cfg) if is_dataclass(train_cfg) else dict(vars(train_cfg))
    torch.save({"config": cfg, "state_dict": uncompiled_policy.state_dict()}, model_path)
    state = {"optimizer_state_dict": optimizer.state_dict(), "global_step": global_step, "agent_step": global_step,
             "update": epoch, "model_name": model_name, "exp_id": exp_id}
    state_path = os.path.join(path, "trainer_state.pt")
    torch.save(state, state_path + ".tmp")
    os.rename(state_path + ".tmp", state_path)
    return model_path


def try_load_checkpoint(policy, optimizer, train_cfg, exp_id):
    """Resume (the reference's helper at utils.py:45-56 is unused and passes a path to
    load_state_dict; this one loads the state dict it names)."""
    path = os.path.join(train_cfg.data_dir, exp_id)
    trainer_path = os.path.join(path, "trainer_state.pt")
    if not os.path.exists(trainer_path):
        return None
    state = torch.load(trainer_path, map_location=train_cfg.device, weights_only=True)
    ckpt = torch.load(os.path.join(path, state["model_name"]), map_location=train_cfg.device, weights_only=True)
    policy.load_state_dict(ckpt["state_dict"])
    optimizer.load_state_dict(state["optimizer_state_dict"])
    return state


def seed_everything(seed, torch_deterministic):
    random.seed(seed)
    np.random.seed(seed)
    if seed is not None:
        torch.manual_seed(seed)
    torch.backends.cudnn.deterministic = torch_deterministic


def count_params(policy):
    return sum(p.numel() for p in policy.parameters() if p.requires_grad)
