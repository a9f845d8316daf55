"""pufferlib.cleanrl.Policy / sample_logits for a continuous (Normal) head.

pufferlib 2.0.6 (kywch fork @ 47f8042) is un-vendored and not installable offline; this is the
published behaviour its call sites rely on (scripts/train.py:271, clean_pufferl/core.py:162,
:291-294): action = Normal.sample() unless given, logprob = log_prob(action).sum(1),
entropy = entropy().sum(1).  Parity unpinned (no reference fixture).
"""

import numpy as np
import torch
from torch import nn


class Linear(nn.Linear):
    """nn.Linear whose GEMM runs without the fused-bias epilogue: on gfx950 hipBLASLt serves the
    'high' float32 precision (xf32 emulation, 2x fp32 MFMA rate) only for plain GEMMs, so the
    bias is added by one elementwise pass.  Same parameters / state-dict keys as nn.Linear."""

    def forward(self, x):
        return torch.matmul(x, self.weight.t()) + self.bias


def layer_init(layer, std=np.sqrt(2), bias_const=0.0):
    """pufferlib.pytorch.layer_init: orthogonal weights, constant bias."""
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def sample_logits(probs, action=None):
    batch = probs.loc.shape[0]
    if action is None:
        # same law as probs.sample(); written as loc + scale * N(0,1) because torch.normal(mean,
        # std) host-checks std on ROCm and so cannot run inside a captured rollout graph
        with torch.no_grad():
            action = (probs.loc + probs.scale * torch.randn_like(probs.loc)).view(batch, -1)
    logprob = probs.log_prob(action.view(batch, -1)).sum(1)
    entropy = probs.entropy().view(batch, -1).sum(1)
    return action, logprob, entropy


class Policy(nn.Module):
    def __init__(self, policy):
        super().__init__()
        self.policy = policy
        self.is_continuous = True

    def get_value(self, x, state=None):
        _, value = self.policy(x)
        return value

    def get_action_and_value(self, x, action=None):
        hidden, lookup = self.policy.encode_observations(x)
        probs, value = self.policy.decode_actions(hidden, lookup)
        action, logprob, entropy = sample_logits(probs, action)
        return action, logprob, entropy, value

    def forward(self, x, action=None):
        return self.get_action_and_value(x, action)
