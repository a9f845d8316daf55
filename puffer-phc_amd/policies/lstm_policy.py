"""N4: the LSTM policies (puffer_phc/policies/lstm_policy.py:10-148) and the pufferlib wrappers they
run under (`pufferlib.models.LSTMWrapper`, `pufferlib.cleanrl.RecurrentPolicy`; scripts/train.py:
262-272 builds `RecurrentPolicy(Recurrent(env, policy))` for `--rnn-name Recurrent`).

pufferlib 2.0.6 (kywch fork @ 47f8042) is un-vendored and not importable here: the two wrappers are
restated from their published behaviour, which the reference's call sites rely on —
  * LSTMWrapper.forward(x, state): observations [B, *obs] (one step) or [B, T, *obs] (a bptt
    segment per row) -> policy.encode_observations on the B*T rows -> a single-layer nn.LSTM over
    time (T-major) from `state` = (h, c) [num_layers, B, hidden] -> policy.decode_actions on the
    B*T outputs; returns (probs, value, new_state).  LSTM weights orthogonal (gain 1), biases 0.
  * RecurrentPolicy.forward(x, state=None, action=None) -> (action, logprob, entropy, value,
    state) through sample_logits; `.lstm` is the wrapper's nn.LSTM (the trainer sizes the
    per-env (h, c) buffers from it: clean_pufferl/core.py:66, structs.py:68-73).
Parity unpinned (no reference fixture: pufferlib is absent).  These models are off the hot path —
the reference's README reports they did not help, and PHCPolicy is the benchmarked model — so they
run on PyTorch-ROCm modules (hipBLASLt GEMMs, MIOpen LSTM) in fp32, not on the fused MFMA kernels.
"""

import torch
from torch import nn

from .discriminator_policy import DiscriminatorPolicy
from .pufferl_policy import Linear, layer_init, sample_logits


class LSTMWrapper(nn.Module):
    """pufferlib.models.LSTMWrapper (see the module docstring)."""

    def __init__(self, env, policy, input_size=128, hidden_size=128, num_layers=1):
        super().__init__()
        self.obs_shape = tuple(env.single_observation_space.shape)
        self.policy = policy
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.is_continuous = getattr(policy, "is_continuous", True)
        self.recurrent = nn.LSTM(input_size, hidden_size, num_layers)
        for name, param in self.recurrent.named_parameters():
            if "bias" in name:
                nn.init.constant_(param, 0)
            elif "weight" in name:
                nn.init.orthogonal_(param, 1.0)

    def forward(self, x, state=None):
        space_n = len(self.obs_shape)
        if tuple(x.shape[-space_n:]) != self.obs_shape:
            raise ValueError(f"invalid input shape {tuple(x.shape)} for observations {self.obs_shape}")
        if x.dim() == space_n + 1:
            B, TT = x.shape[0], 1
        elif x.dim() == space_n + 2:
            B, TT = x.shape[:2]
        else:
            raise ValueError(f"invalid input shape {tuple(x.shape)}")
        if state is not None and not (state[0].shape[1] == state[1].shape[1] == B):
            raise ValueError("LSTM state batch does not match the observations")
        x = x.reshape(B * TT, *self.obs_shape)
        hidden, lookup = self.policy.encode_observations(x)
        hidden = hidden.reshape(B, TT, self.input_size).transpose(0, 1)
        hidden, state = self.recurrent(hidden, state)
        hidden = hidden.transpose(0, 1).reshape(B * TT, self.hidden_size)
        probs, value = self.policy.decode_actions(hidden, lookup)
        return probs, value, state


class Recurrent(LSTMWrapper):
    """lstm_policy.py:10-22: the wrapper exposing the inner policy's trainer hooks."""

    def __init__(self, env, policy, input_size=512, hidden_size=512, num_layers=1):
        super().__init__(env, policy, input_size, hidden_size, num_layers)
        self.set_deterministic_action = self.policy.set_deterministic_action
        self.discriminate = self.policy.discriminate
        self.discriminate_rows = self.policy.discriminate_rows
        self.adversarial_reward = self.policy.adversarial_reward
        self.update_obs_rms = self.policy.update_obs_rms
        self.update_amp_obs_rms = self.policy.update_amp_obs_rms

    @property
    def mean_bound_loss(self):
        return self.policy.mean_bound_loss

    @property
    def soft_bound(self):
        return self.policy.soft_bound

    @property
    def sigma(self):
        return self.policy.sigma

    def bound_loss(self, mu):
        return self.policy.bound_loss(mu)


class RecurrentPolicy(nn.Module):
    """pufferlib.cleanrl.RecurrentPolicy (see the module docstring).  The reference calls it as
    policy(obs, (h, c)) in evaluate (core.py:158) and policy(obs, info=state, action=atn) in train
    (core.py:288): both spellings are accepted."""

    def __init__(self, policy):
        super().__init__()
        self.policy = policy
        self.is_continuous = True

    @property
    def lstm(self):
        return self.policy.recurrent

    def get_action_and_value(self, x, state=None, action=None):
        probs, value, state = self.policy(x, state)
        action, logprob, entropy = sample_logits(probs, action)
        return action, logprob, entropy, value, state

    def forward(self, x, state=None, action=None, info=None):
        return self.get_action_and_value(x, state if info is None else info, action)


class LSTMCriticPolicy(DiscriminatorPolicy):
    """lstm_policy.py:25-87: the PHC actor MLP reads the normalised observations directly; the
    critic MLP feeds the LSTM, whose output the value head reads."""

    def __init__(self, env, hidden_size=512):
        super().__init__(env, hidden_size)
        self.actor_mlp = nn.Sequential(
            layer_init(Linear(self.input_size, 2048)), nn.SiLU(),
            layer_init(Linear(2048, 1536)), nn.SiLU(),
            layer_init(Linear(1536, 1024)), nn.SiLU(),
            layer_init(Linear(1024, 1024)), nn.SiLU(),
            layer_init(Linear(1024, 512)), nn.SiLU(),
            layer_init(Linear(512, hidden_size)), nn.SiLU(),
            layer_init(Linear(hidden_size, self.action_size), std=0.01),
        )
        self.mu = None
        self.critic_mlp = nn.Sequential(
            layer_init(Linear(self.input_size, 2048)), nn.ReLU(),
            layer_init(Linear(2048, 1024)), nn.ReLU(),
            layer_init(Linear(1024, 1024)), nn.ReLU(),
            layer_init(Linear(1024, hidden_size)), nn.ReLU(),
        )
        self.value = nn.Sequential(nn.ReLU(), layer_init(Linear(hidden_size, 1), std=0.01))

    def encode_observations(self, obs):
        self.obs_pointer = self.obs_norm(obs)
        return self.critic_mlp(self.obs_pointer), None

    def decode_actions(self, hidden, lookup=None):
        mu = self.actor_mlp(self.obs_pointer)
        std = torch.exp(self.sigma).expand_as(mu)
        if self._deterministic_action is True:
            std = torch.clamp(std, max=1e-6)
        probs = torch.distributions.Normal(mu, std)
        if self.training:
            self.mean_bound_loss = self.bound_loss(mu)
        return probs, self.value(hidden)


class LSTMActorPolicy(DiscriminatorPolicy):
    """lstm_policy.py:90-148: the actor MLP feeds the LSTM, whose output the mu head reads; a
    separate ReLU critic MLP reads the normalised observations."""

    def __init__(self, env, hidden_size=512):
        super().__init__(env, hidden_size)
        self.actor_mlp = nn.Sequential(
            layer_init(Linear(self.input_size, 2048)), nn.SiLU(),
            layer_init(Linear(2048, 2048)), nn.SiLU(),
            layer_init(Linear(2048, 1024)), nn.SiLU(),
            layer_init(Linear(1024, hidden_size)), nn.SiLU(),
        )
        self.mu = nn.Sequential(nn.SiLU(), layer_init(Linear(hidden_size, self.action_size), std=0.01))
        self.critic_mlp = nn.Sequential(
            layer_init(Linear(self.input_size, 1024)), nn.ReLU(),
            layer_init(Linear(1024, 1024)), nn.ReLU(),
            layer_init(Linear(1024, 512)), nn.ReLU(),
            layer_init(Linear(512, 256)), nn.ReLU(),
            layer_init(Linear(256, 1), std=0.01),
        )

    def encode_observations(self, obs):
        self.obs_pointer = self.obs_norm(obs)
        return self.actor_mlp(self.obs_pointer), None

    def decode_actions(self, hidden, lookup=None):
        mu = self.mu(hidden)
        std = torch.exp(self.sigma).expand_as(mu)
        if self._deterministic_action is True:
            std = torch.clamp(std, max=1e-6)
        probs = torch.distributions.Normal(mu, std)
        if self.training:
            self.mean_bound_loss = self.bound_loss(mu)
        return probs, self.critic_mlp(self.obs_pointer)
