"""PHCPufferEnv drop-in (puffer_phc/clean_pufferl/env.py:22-195): the pufferlib.PufferEnv
protocol over HumanoidPHC, with every per-step buffer on the device.

The reference moves actions D->H->D (np.clip + torch.from_numpy, :91-93) and finds resets
with torch.nonzero / .tolist() (:114-121).  Here `step` accepts device (or numpy) actions,
the fused step kernel writes terminals / truncations / masks / episode return and length,
and terminated envs are re-initialised by a kernel that reads reset_buf on the device.
Episode statistics accumulate in per-workgroup float64 rows and are reduced on the host only
every `log_interval` ticks (the reference's logging cadence, :145-162).
"""

import functools
from collections.abc import Mapping

import numpy as np
import torch

from .. import _native
from ..envs.humanoid_phc import HumanoidPHC


def env_creator(name="puffer_phc"):
    return functools.partial(make, name)


def make(cfg, motion_data=None):
    return PHCPufferEnv(cfg, motion_data=motion_data)


class PendingInfo(Mapping):
    """One mean_and_log() info dict whose statistics are still on their way from the device; any
    read waits for the copy and builds the dict (PHCPufferEnv._resolve_info)."""

    def __init__(self, env, host, event):
        self._src, self._d = (env, host, event), None

    def resolve(self):
        if self._d is None:
            env, host, event = self._src
            event.synchronize()
            self._d = env._resolve_info(host.numpy().copy())
            self._src = None
        return self._d

    def __getitem__(self, k):
        return self.resolve()[k]

    def __iter__(self):
        return iter(self.resolve())

    def __len__(self):
        return len(self.resolve())

    def __repr__(self):
        return repr(self.resolve())


class PHCPufferEnv:
    def __init__(self, cfg, motion_data=None, physics=None):
        self.render_mode = "native"
        self.cfg = cfg
        self.env = HumanoidPHC(cfg, motion_data=motion_data, physics=physics)
        self.driver_env = self
        self.single_observation_space = self.env.single_observation_space
        self.single_action_space = self.env.single_action_space
        self.amp_observation_space = self.env.amp_observation_space if cfg.use_amp_obs else None
        N, dev = self.num_agents, cfg.device
        self.observations = self.env.obs_buf
        self.rewards = self.env.rew_buf
        self.terminals = torch.zeros(N, dtype=torch.bool, device=dev)
        self.truncations = torch.zeros(N, dtype=torch.bool, device=dev)
        self.masks = torch.ones(N, dtype=torch.bool, device=dev)
        self.actions = torch.zeros((N, *self.single_action_space.shape), dtype=torch.float32, device=dev)
        self.episode_returns = torch.zeros(N, dtype=torch.float32, device=dev)
        self.episode_lengths = torch.zeros(N, dtype=torch.int32, device=dev)
        self.stats = torch.zeros((_native.lib().phc_stats_blocks(N), _native.STATS_SLOTS), dtype=torch.float64,
                                 device=dev)
        self.env.attach_puffer_buffers(self.terminals, self.truncations, self.masks, self.episode_returns,
                                       self.episode_lengths, self.stats)
        self.env_ids = torch.arange(N, device=dev)
        self.episode_count = 0
        self.tick = 0
        self._pending = None
        # pinned buffers for mean_and_log's non-blocking readback, reused round-robin
        self._info_ring = [[torch.empty(_native.STATS_SLOTS, dtype=torch.float64, pin_memory=True), None]
                           for _ in range(4)]
        self._info_i = 0

    @property
    def num_agents(self):
        return self.cfg.num_envs

    @property
    def agents_per_batch(self):
        return self.num_agents

    def reset(self, seed=None):
        self.tick = 0
        self.env.reset()
        self.amp_obs = self.env.amp_obs if self.cfg.use_amp_obs else None
        self.rewards.zero_()
        self.terminals.zero_()
        self.truncations.zero_()
        self.masks.fill_(True)
        self.actions.zero_()
        self.stats.zero_()
        return self.observations, []

    def step(self, actions):
        if isinstance(actions, np.ndarray):
            self.actions.copy_(torch.from_numpy(actions))
            actions = self.actions
        elif not (actions.device == self.actions.device and actions.dtype == torch.float32
                  and actions.is_contiguous() and tuple(actions.shape) == tuple(self.actions.shape)):
            self.actions.copy_(actions)
            actions = self.actions
        # a device float32 [N, 69] tensor is read in place by the step kernel (the reference's
        # `self.actions[:] = actions` copy, clean_pufferl/env.py, is a 1.1 MB device copy per step
        # with no other reader); clipping happens inside the action -> PD map (cfg.clip_actions
        # is always honoured); the fused kernel also performs the env.reset(reset_indices) of
        # :114-116, which leaves rew_buf untouched, so no defensive copy of the rewards is needed
        self.env.step(actions, auto_reset=True)
        rew = self.rewards
        self.amp_obs = self.env.amp_obs if self.cfg.use_amp_obs else None
        info = []
        self.tick += 1
        if self.tick % self.cfg.log_interval == 0:
            info = self.mean_and_log()
        return self.observations, rew, self.terminals, self.truncations, info

    # ----------------------------------------------- rollout blocks (captured graphs) --
    @property
    def block_steppable(self):
        """Whether steps can be captured into a rollout block graph: the fused replay launch (no
        per-step host value) with the env's in-launch auto-reset; with AMP its history launch too (it
        reads only device state)."""
        e = self.env
        return e.fused_env_step and hasattr(e.physics, "step_fused") and not e.flag_im_eval

    def block_stats(self, steps):
        """[steps, blocks, slots] float64 logging rows: step k of a block writes rows k."""
        buf = getattr(self, "_block_stats", None)
        if buf is None or buf.shape[0] < steps:
            buf = self._block_stats = torch.zeros((steps,) + tuple(self.stats.shape), dtype=torch.float64,
                                                  device=self.stats.device)
            self._block_env_c = None
        env_key = bytes(self.env._env_c)
        if self._block_env_c is None or self._block_env_key != env_key:  # copies of the current env struct
            self._block_env_c = [self.env.stats_env_struct(buf[k]) for k in range(buf.shape[0])]
            self._block_env_key = env_key
        return buf[:steps]

    def block_step(self, actions, k):
        """Step k of a captured block: step() without the host's tick / logging bookkeeping (done by
        finish_block for the whole block), the logging rows going to block_stats row k."""
        self.env.step(actions, auto_reset=True, env_c=self._block_env_c[k])

    def finish_block(self, steps):
        """After a replayed block of `steps` steps: advance the tick and emit the mean_and_log infos
        of every log point inside the block, each over exactly the log_interval steps before it (the
        rows of earlier eager steps in self.stats, then the block's rows up to the point); the rows
        after the last point carry into self.stats.  Returns the infos (PendingInfo)."""
        rows = self._block_stats[:steps]
        L = self.cfg.log_interval
        infos, a = [], 0
        first = (L - self.tick % L) % L  # steps until the next log point (0: the block's first step)
        for k in range(first if first > 0 else L, steps + 1, L):  # log after step index k - 1
            s = self.stats.sum(0) + rows[a:k].sum((0, 1))
            infos.append(self._pending_info(s))
            self.stats.zero_()
            a = k
        if a < steps:
            self.stats[0] += rows[a:steps].sum((0, 1))
        rows.zero_()  # the next replay adds into zeroed rows
        self.tick += steps
        return infos

    def _pending_info(self, s):
        slot = self._info_ring[self._info_i % len(self._info_ring)]
        self._info_i += 1
        if slot[1] is not None:
            slot[1].resolve()  # the copy that last used this buffer finished long ago
        host = slot[0]
        host.copy_(s, non_blocking=True)
        done = torch.cuda.Event()
        done.record()
        info = PendingInfo(self, host, done)
        slot[1] = info
        return info

    def mean_and_log(self):
        """Host reduction of the per-block statistics (clean_pufferl/env.py:145-188).  The sums come
        back by a non-blocking copy into pinned memory: the returned info resolves (waits for the
        copy) when first read, so the rollout does not drain the stream every log_interval steps;
        the trainer reads the step infos after its rollout loop."""
        info = self._pending_info(self.stats.sum(0))
        self.stats.zero_()
        return [info]

    def flush(self):
        """Resolve every outstanding mean_and_log info (waits for their copies): afterwards
        episode_count includes every log point emitted so far, as the reference's mean_and_log
        counts at call time (clean_pufferl/env.py:145-188).  The trainer calls it after each
        rollout loop, where it reads the infos anyway."""
        for slot in self._info_ring:
            if slot[1] is not None:
                slot[1].resolve()

    def _resolve_info(self, s):
        n_ep = s[7]
        self.episode_count += int(n_ep)
        denom = self.cfg.log_interval * self.num_agents
        info = {
            "rew_body_pos": s[0] / denom,
            "rew_body_rot": s[1] / denom,
            "rew_lin_vel": s[2] / denom,
            "rew_ang_vel": s[3] / denom,
            "rew_power": s[4] / denom,
        }
        if n_ep > 0:
            info.update(episode_return=s[5] / n_ep, episode_length=s[6] / n_ep, truncated_rate=s[8] / n_ep)
        return info

    # -------------------------------------------- pufferlib vecenv protocol --
    def async_reset(self, seed=None):
        obs, _ = self.reset(seed)
        self._pending = (obs, self.rewards, self.terminals, self.truncations, [], self.env_ids, self.masks)

    def send(self, actions):
        obs, rew, term, trunc, info = self.step(actions)
        self._pending = (obs, rew, term, trunc, info, self.env_ids, self.masks)

    def recv(self):
        return self._pending

    def render(self):
        return self.env.render()

    def close(self):
        self.env.close()

    def fetch_amp_obs_demo(self):
        return self.env.fetch_amp_obs_demo()
