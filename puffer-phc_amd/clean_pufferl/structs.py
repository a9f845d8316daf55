"""Trainer state (puffer_phc/clean_pufferl/structs.py) with the Experience buffer on device.

The reference keeps actions/logprobs/rewards/dones/values as CPU tensors, copies five of
them from the device every step and sorts a Python list of (env_id, step) tuples per epoch
(:113-145).  Here every buffer lives in HBM; the only per-step host read is the count of
mask-true rows (the reference's `mask.sum().item()`, core.py:136), and the (env, step) sort
is a stable device sort of the env ids (rows are stored in step order).
"""

import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np
import torch


# splitmix64 on int64 tensors (wrapping products, logical right shifts): the AMP replay buffer's
# counter-based draws
_GOLD = -7046029254386353131  # 0x9E3779B97F4A7C15
_M1 = -4658895280553007687    # 0xBF58476D1CE4E5B9
_M2 = -7723592293110705685    # 0x94D049BB133111EB
_PERM_SALT = 0x5DEECE66D


def _lsr(z, s):
    return (z >> s) & ((1 << (64 - s)) - 1)


def _mix64(z):
    z = (z ^ _lsr(z, 30)) * _M1
    z = (z ^ _lsr(z, 27)) * _M2
    return z ^ _lsr(z, 31)

class Experience:
    """Flat on-device storage, puffer_phc/clean_pufferl/structs.py:23-176."""

    def __init__(self, batch_size, bptt_horizon, minibatch_size, obs_shape, obs_dtype=np.float32, atn_shape=(69,),
                 atn_dtype=np.float32, cpu_offload=False, device="cuda", lstm=None, lstm_total_agents=0,
                 use_amp_obs=False, amp_obs_size=1960, amp_obs_update_prob=0.01):
        if minibatch_size is None:
            minibatch_size = batch_size
        self.obs = torch.zeros((batch_size, *obs_shape), dtype=torch.float32, device=device)
        self.actions = torch.zeros((batch_size, *atn_shape), dtype=torch.float32, device=device)
        self.logprobs = torch.zeros(batch_size, device=device)
        self.rewards = torch.zeros(batch_size, device=device)
        self.dones = torch.zeros(batch_size, device=device)
        self.truncateds = torch.zeros(batch_size, device=device)
        self.values = torch.zeros(batch_size, device=device)
        self.env_ids = torch.zeros(batch_size, dtype=torch.int64, device=device)
        self.lstm_h = self.lstm_c = None
        if lstm is not None:
            shape = (lstm.num_layers, lstm_total_agents, lstm.hidden_size)
            self.lstm_h = torch.zeros(shape, device=device)
            self.lstm_c = torch.zeros(shape, device=device)
        num_minibatches = batch_size / minibatch_size
        self.num_minibatches = int(num_minibatches)
        if self.num_minibatches != num_minibatches:
            raise ValueError("batch_size must be divisible by minibatch_size")
        minibatch_rows = minibatch_size / bptt_horizon
        self.minibatch_rows = int(minibatch_rows)
        if self.minibatch_rows != minibatch_rows:
            raise ValueError("minibatch_size must be divisible by bptt_horizon")
        self.batch_size = batch_size
        self.bptt_horizon = bptt_horizon
        self.minibatch_size = minibatch_size
        self.device = device
        self.ptr = 0
        self.step = 0
        self.use_amp_obs = use_amp_obs
        if use_amp_obs:
            self.amp_obs = torch.zeros((batch_size, amp_obs_size), device=device)
            self.amp_obs_replay = torch.zeros((batch_size, amp_obs_size), device=device)
            self.amp_obs_replay_filled = False
            self.amp_obs_update_prob = amp_obs_update_prob

    @property
    def full(self):
        return self.ptr >= self.batch_size

    def store(self, obs, amp_obs, value, action, logprob, reward, done, trunc, env_id, mask, n_valid=None):
        """Append the mask-true rows (structs.py:113-131).  Returns the number of rows taken."""
        ptr = self.ptr
        if n_valid is None:
            n_valid = int(mask.sum().item())
        take = min(n_valid, self.batch_size - ptr)
        if take <= 0:
            return 0
        end = ptr + take
        if n_valid == mask.shape[0]:
            sl = slice(0, take)
            self.obs[ptr:end] = obs[sl]
            self.values[ptr:end] = value[sl]
            self.actions[ptr:end] = action[sl]
            self.logprobs[ptr:end] = logprob[sl]
            self.rewards[ptr:end] = reward[sl]
            self.dones[ptr:end] = done[sl]
            self.truncateds[ptr:end] = trunc[sl]
            self.env_ids[ptr:end] = env_id[sl]
            if self.use_amp_obs:
                self.amp_obs[ptr:end] = amp_obs[sl]
        else:
            idx = torch.nonzero(mask).squeeze(-1)[:take]
            self.obs[ptr:end] = obs[idx]
            self.values[ptr:end] = value[idx]
            self.actions[ptr:end] = action[idx]
            self.logprobs[ptr:end] = logprob[idx]
            self.rewards[ptr:end] = reward[idx]
            self.dones[ptr:end] = done[idx].float()
            self.truncateds[ptr:end] = trunc[idx].float()
            self.env_ids[ptr:end] = env_id[idx]
            if self.use_amp_obs:
                self.amp_obs[ptr:end] = amp_obs[idx]
        self.ptr = end
        self.step += 1
        return take

    def sort_training_data(self):
        """(env_id, step) order == stable sort by env id (rows are in step order)."""
        idxs = torch.sort(self.env_ids, stable=True).indices
        self.b_idxs_obs = idxs.reshape(self.minibatch_rows, self.num_minibatches, self.bptt_horizon).transpose(0, 1)
        self.b_idxs = self.b_idxs_obs
        self.b_idxs_flat = self.b_idxs.reshape(self.num_minibatches, self.minibatch_size)
        return idxs

    def flatten_batch(self, skip_obs=False):
        """Gather the training tensors in minibatch order (structs.py:146-160); skip_obs when the
        trainer reads the observations through its own normalised copy instead."""
        b_idxs, b_flat = self.b_idxs, self.b_idxs_flat
        self.b_obs = None if skip_obs else self.obs[self.b_idxs_obs]
        self.b_actions = self.actions[b_idxs].contiguous()
        self.b_logprobs = self.logprobs[b_idxs]
        self.b_dones = self.dones[b_idxs]
        self.b_truncated = self.truncateds[b_idxs]
        self.b_values = self.values[b_flat]
        if self.use_amp_obs:
            # AMP rows stay where they are: the discriminator gathers them through these indices
            # (b_amp_obs / b_amp_obs_replay below materialise the reference's tensors on demand)
            self.b_amp_idx = b_flat
            # the replay refresh (structs.py:165-176: rand < p rows replaced, then a randperm of the
            # replay rows) from a counter-based draw keyed by a device iteration counter, and a
            # select instead of a boolean-mask write: no host value, no host sync, so the pass can
            # replay from a graph and draws the same numbers graphed or eager
            it = self._amp_draw_counter()
            idx = torch.arange(self.batch_size, device=self.device, dtype=torch.int64)
            if not self.amp_obs_replay_filled:
                self.amp_obs_replay[:] = self.amp_obs[:]
                self.amp_obs_replay_filled = True
            else:
                u = (_lsr(_mix64(idx + it * _GOLD), 40).float() * (1.0 / 16777216.0))
                upd = u < self.amp_obs_update_prob
                torch.where(upd.unsqueeze(1), self.amp_obs, self.amp_obs_replay, out=self.amp_obs_replay)
            keys = _mix64((idx + it * _GOLD) ^ _PERM_SALT)
            rep = torch.argsort(keys).reshape(self.num_minibatches, self.minibatch_size)
            self.b_amp_rep_idx = rep

    def _amp_draw_counter(self):
        """The AMP replay draws' device iteration counter, advanced once per flatten_batch (inside a
        captured pass too)."""
        c = getattr(self, "_amp_iter", None)
        if c is None:
            c = self._amp_iter = torch.zeros((), dtype=torch.int64, device=self.device)
        c += 1
        return c

    @property
    def b_amp_obs(self):
        """amp_obs in minibatch order, [num_minibatches, minibatch_size, amp_obs_size] (structs.py:157)."""
        return self.amp_obs[self.b_amp_idx]

    @property
    def b_amp_obs_replay(self):
        """The replay rows drawn for each minibatch (structs.py:158-160)."""
        return self.amp_obs_replay[self.b_amp_rep_idx]


@dataclass
class LossComponents:
    policy_loss: float = 0.0
    value_loss: float = 0.0
    disc_loss: float = 0.0
    disc_agent_acc: float = 0.0
    disc_demo_acc: float = 0.0
    entropy: float = 0.0
    old_approx_kl: float = 0.0
    approx_kl: float = 0.0
    clipfrac: float = 0.0
    explained_variance: float = 0.0
    mean_bound_loss: float = 0.0
    before_clip_grad_norm: float = 0.0
    l2_init_reg_loss: float = 0.0


class PendingLossComponents(LossComponents):
    """LossComponents whose values are still on their way from the device: a non-blocking copy
    into pinned host memory and the event after it.  The first attribute read waits for that
    event and fills the fields (fill(self, values)), so train() returns without draining the
    stream and the host goes on queueing the next rollout while the GPU finishes the update."""

    def __init__(self, host, event, fill):  # noqa: D107 (the dataclass fields are set by fill)
        object.__setattr__(self, "_pending", (host, event, fill))

    def __getattribute__(self, name):
        # every read but the marker itself resolves the copy first, dunders included: vars(),
        # __dict__, dataclasses.asdict / copy / pickle all see the filled fields
        d = object.__getattribute__(self, "__dict__")
        pend = d.get("_pending")
        if pend is not None and name != "_pending":
            d["_pending"] = None
            host, event, fill = pend
            event.synchronize()
            fill(self, host.numpy())
        return object.__getattribute__(self, name)


@dataclass
class StatsData:
    episode_length: List[float] = field(default_factory=list)
    episode_return: List[float] = field(default_factory=list)
    truncated_rate: List[float] = field(default_factory=list)
    rew_body_pos: List[float] = field(default_factory=list)
    rew_body_rot: List[float] = field(default_factory=list)
    rew_lin_vel: List[float] = field(default_factory=list)
    rew_ang_vel: List[float] = field(default_factory=list)
    rew_power: List[float] = field(default_factory=list)
    media_items: Dict[str, Any] = field(default_factory=dict)

    def add(self, key, value):
        if not hasattr(self, key):
            setattr(self, key, [])
        getattr(self, key).append(value)

    def extend(self, key, values):
        if not hasattr(self, key):
            setattr(self, key, [])
        getattr(self, key).extend(values)

    def clear(self):
        for k, v in list(vars(self).items()):
            if isinstance(v, list):
                setattr(self, k, [])
        self.media_items.clear()

    def items(self):
        return {k: float(np.mean(v)) for k, v in vars(self).items() if isinstance(v, list) and len(v) > 0}

    def mean_and_log(self, components, info, losses):
        if info.wandb is None:
            return
        from dataclasses import asdict

        info.last_log_time = time.time()
        info.wandb.log({"0verview/SPS": info.profile.SPS, "0verview/agent_steps": info.global_step,
                        "0verview/epoch": info.epoch,
                        "0verview/learning_rate": components.optimizer.param_groups[0]["lr"],
                        **{f"environment/{k}": v for k, v in self.items().items()},
                        **{f"losses/{k}": v for k, v in asdict(losses).items()}})


class Profiler:
    """pufferlib.utils.Profiler: accumulated wall time of a context."""

    def __init__(self):
        self.elapsed = 0.0
        self._t = None

    def __enter__(self):
        self._t = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.elapsed += time.perf_counter() - self._t


@dataclass
class Profile:
    SPS: float = 0
    uptime: float = 0
    remaining: float = 0
    eval_time: float = 0
    env_time: float = 0
    eval_forward_time: float = 0
    eval_misc_time: float = 0
    train_time: float = 0
    train_forward_time: float = 0
    learn_time: float = 0
    train_misc_time: float = 0

    def __post_init__(self):
        self.start = time.time()
        self.env = Profiler()
        self.eval_forward = Profiler()
        self.eval_misc = Profiler()
        self.train_forward = Profiler()
        self.learn = Profiler()
        self.train_misc = Profiler()
        self.evaluate = Profiler()
        self.train = Profiler()
        self.prev_steps = 0

    def update(self, components, info, interval_s=1):
        """SPS = agent steps / wall time (structs.py:340-368)."""
        if info.global_step == 0:
            return True
        uptime = time.time() - self.start
        if uptime - self.uptime < interval_s:
            return False
        self.SPS = (info.global_step - self.prev_steps) / (uptime - self.uptime)
        self.prev_steps = info.global_step
        self.uptime = uptime
        self.remaining = (info.config.total_timesteps - info.global_step) / max(self.SPS, 1e-9)
        self.eval_time = self.evaluate.elapsed
        self.eval_forward_time = self.eval_forward.elapsed
        self.env_time = self.env.elapsed
        self.eval_misc_time = self.eval_misc.elapsed
        self.train_time = self.train.elapsed
        self.train_forward_time = self.train_forward.elapsed
        self.learn_time = self.learn.elapsed
        self.train_misc_time = self.train_misc.elapsed
        return True


@dataclass
class TrainComponents:
    vecenv: Any
    policy: Any
    uncompiled_policy: Any
    experience: Experience
    optimizer: torch.optim.Optimizer
    scaler: Any = None
    # fp16: optimizer steps the loss scaler skipped (inf/nan gradients), a device counter
    skipped_steps: Any = None


@dataclass
class TrainInfo:
    config: Any
    exp_id: str
    env_name: str
    use_amp_obs: bool
    initial_params: Dict[str, torch.Tensor]
    msg: str
    last_log_time: float
    stats: StatsData
    profile: Profile
    wandb: Any
    global_step: int = 0
    epoch: int = 0
    dist: Optional[Any] = None


class Utilization:
    """structs.py:393-420 samples CPU/GPU utilisation on a thread; here a passive stand-in
    (psutil on demand) so the trainer API keeps its shape without a background thread."""

    def __init__(self, delay=1, maxlen=20):
        self.cpu_util, self.cpu_mem, self.gpu_util, self.gpu_mem = [], [], [], []

    def stop(self):
        pass
