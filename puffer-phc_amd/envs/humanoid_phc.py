"""HumanoidPHC drop-in (puffer_phc/envs/humanoid_phc.py:46-1454) on the HIP hot path.

Per step (HumanoidPHC.step, :105-172) the env launches, on the current HIP stream:
  with `ReplayPhysics` (BASELINE configs[1], "physics stubbed with replayed rigid-body states"; the
  default): ONE launch, phc_env_step_replay = the action -> PD map (R13) + the stand-in + the
  post-physics step below (cfg.fused_env_step = False: the three separate launches);
  with `physics.ArticulatedPhysics` (N3, cfg.physics = "articulated"):
  phc_physics_step_actions  the articulated-body PD step with R13 folded in, then
  phc_env_step       (R6,R7,R9-R12,R14) progress, reward(t), reset(t), obs(t+dt) and the
                     PufferEnv bookkeeping, fused in one kernel
and `reset_done()` / `reset(env_ids)` (R15) re-initialises terminated envs from the motion
library in one more kernel driven by the device reset flags — no host synchronisation.

Buffers keep the reference's names and layouts: `_rigid_body_state` [N,24,13] (Isaac Gym
rigid-body layout, :542-549), `_dof_state` [N,69,2], `dof_force_tensor` [N,69],
`progress_buf` int16, `reset_buf`/`_terminate_buf` bool, `obs_buf` [N,934], `rew_buf`,
`reward_raw` [N,5].
"""

import numpy as np
import torch

from .. import _native
from ..body_sets import BODY_NAMES, DOF_NAMES, EVAL_BODIES, KEY_BODIES, RESET_BODIES, TRACK_BODIES, dof_subset
from ..config import EnvConfig
from ..motion_lib import FixHeightMode, MotionLibSMPL
from ..skeleton import SkeletonTree
from .state_init import StateInit


class Box:
    """Minimal gym.spaces.Box (gym is not available offline)."""

    def __init__(self, low, high, dtype=np.float32):
        self.low = np.asarray(low, dtype=dtype)
        self.high = np.asarray(high, dtype=dtype)
        self.shape = self.low.shape
        self.dtype = np.dtype(dtype)

    def sample(self):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return np.random.uniform(lo, hi).astype(self.dtype)


class ReplayPhysics:
    """Physics stand-in: rigid bodies = reference state at the env's next control time plus
    gaussian noise (phc_physics_replay).  Not a reference interface.  The noise is keyed by the
    env's own device counters (episode rng counter, progress), so a step launch carries no per-step
    host value and a captured graph of steps replays fresh noise every time (the kernel's host
    counter argument stays 0)."""

    def __init__(self, pos_sigma=0.02, force_scale=50.0, seed=0):
        self.pos_sigma = pos_sigma
        self.force_scale = force_scale
        self.seed = seed
        self.counter = 0

    def step(self, env):
        _native.physics_replay(env._env_c, env._motion_lib.packed.c, env._step_params, self.pos_sigma,
                               self.force_scale, self.seed, self.counter)

    def step_fused(self, env, params, pd, timer=None, env_c=None):
        """The stand-in, the action -> PD map and the post-physics env step in one launch
        (phc_env_step_replay): the replayed state is the reference blend the env step reads
        anyway, so it never makes an HBM round trip.  env_c: the env struct to launch with (default
        the env's own)."""
        _native.env_step_replay(env._env_c if env_c is None else env_c, env._motion_lib.packed.c, params,
                                self.pos_sigma, self.force_scale, self.seed, self.counter, pd=pd, timer=timer)


class HumanoidPHC:
    def __init__(self, cfg: EnvConfig, motion_data=None, physics=None):
        self.cfg = cfg
        self.device = cfg.device
        if not self.device.startswith("cuda"):
            raise RuntimeError("HumanoidPHC runs on the HIP path only (device must be cuda:N)")
        self.dt = float(np.float32(2 * (1.0 / 60.0)))  # IsaacGymBase.dt, isaacgym_env.py:41
        self.num_envs = cfg.num_envs
        self.all_env_ids = torch.arange(cfg.num_envs, device=self.device)
        self.flag_test = False
        self.flag_im_eval = False
        self.flag_debug = False
        self._config_robot()
        self._config_env()
        self._define_gym_spaces()
        self._setup_env_buffers()
        if physics is None and cfg.physics == "articulated":
            from ..physics import ArticulatedPhysics, PhysicsConfig

            # RobotConfig.has_self_collision: the reference's --disable_self_collision flag clears it
            # and the asset's filter words then keep every shape pair apart (humanoid_phc.py:338, 370-381)
            physics = ArticulatedPhysics(PhysicsConfig(substeps=cfg.physics_substeps, kp_scale=cfg.kp_scale,
                                                       kd_scale=cfg.kd_scale,
                                                       self_collision=bool(cfg.robot.has_self_collision)),
                                         device=self.device)
        self.physics = physics or ReplayPhysics(cfg.replay_pos_sigma, cfg.replay_force_scale, cfg.seed)
        self._rng_seed = int(cfg.seed) * 7919 + 17
        self._rng_counter = 0
        self.kernel_timer = None  # bench: _native.KernelTimer timing every phc_env_step launch
        # the replay stand-in + R13 fused into the env step launch (False: the three launches)
        self.fused_env_step = bool(getattr(cfg, "fused_env_step", True))
        self._load_motion(cfg.motion_file if motion_data is None else motion_data)

    # ------------------------------------------------------------ setup --
    def _config_robot(self):
        self.skeleton_tree = SkeletonTree.smpl()
        self.skeleton_trees = [self.skeleton_tree] * self.cfg.num_envs
        self.num_bodies = len(BODY_NAMES)
        self.num_dof = len(DOF_NAMES) * 3
        self.dof_subset = torch.tensor(dof_subset(), device=self.device)
        self.gender_beta = np.zeros(17)
        self.humanoid_shapes = torch.zeros((self.cfg.num_envs, 17), device=self.device)
        self.humanoid_limb_and_weights = torch.zeros((self.cfg.num_envs, 10), device=self.device)
        # _build_pd_action_offset_scale (humanoid_phc.py:385-456): every SMPL 3-dof joint is limited
        # to +-180 or +-720 deg -> scale min(1.2*max, pi) = pi, offset 0; knees' y scale 5.
        off = torch.zeros(self.num_dof)
        scale = torch.full((self.num_dof,), float(np.float32(np.pi)))
        scale[DOF_NAMES.index("L_Knee") * 3 + 1] = 5
        scale[DOF_NAMES.index("R_Knee") * 3 + 1] = 5
        frozen = torch.zeros(self.num_dof, dtype=torch.uint8)
        names = []
        if self.cfg.robot.freeze_hand:
            names += ["L_Hand", "R_Hand"]
        if self.cfg.robot.freeze_toe:
            names += ["L_Toe", "R_Toe"]
        for n in names:
            frozen[DOF_NAMES.index(n) * 3: DOF_NAMES.index(n) * 3 + 3] = 1
        self._pd_action_offset = off.to(self.device)
        self._pd_action_scale = scale.to(self.device)
        self._pd_frozen = frozen.to(self.device)

    def _config_env(self):
        self._termination_distances = torch.full((self.num_bodies,), float(self.cfg.termination_distance),
                                                 device=self.device)
        self._termination_distances_backup = self._termination_distances.clone()
        self._key_body_ids = torch.tensor([BODY_NAMES.index(b) for b in KEY_BODIES], device=self.device)
        self._track_bodies_id = torch.tensor([BODY_NAMES.index(b) for b in TRACK_BODIES], device=self.device)
        self._reset_bodies_id = [BODY_NAMES.index(b) for b in RESET_BODIES]
        self._reset_bodies_id_backup = list(self._reset_bodies_id)
        self._eval_track_bodies_id = [BODY_NAMES.index(b) for b in EVAL_BODIES]

    def _define_gym_spaces(self):
        """humanoid_phc.py:458-495."""
        self._num_self_obs = 1 + self.num_bodies * (3 + 6 + 3 + 3) - 3
        self._task_obs_size = len(TRACK_BODIES) * self.num_bodies
        self.num_obs = self._num_self_obs + self._task_obs_size
        assert self.num_obs == 934
        self._dof_obs_size = len(DOF_NAMES) * 6
        self._num_amp_obs_per_step = 13 + self._dof_obs_size + self.num_dof + 3 * len(KEY_BODIES)
        if self.cfg.robot.has_dof_subset:
            self._num_amp_obs_per_step -= (6 + 3) * int((self.num_dof - len(self.dof_subset)) / 3)
        self.num_amp_obs = self.cfg.num_amp_obs_steps * self._num_amp_obs_per_step
        self.num_actions = self.num_dof
        self.single_observation_space = Box(np.full(self.num_obs, -np.inf), np.full(self.num_obs, np.inf))
        self.amp_observation_space = Box(np.full(self.num_amp_obs, -np.inf), np.full(self.num_amp_obs, np.inf))
        self.single_action_space = Box(-np.ones(self.num_actions), np.ones(self.num_actions))

    def _setup_env_buffers(self):
        N, dev = self.cfg.num_envs, self.device
        self._rigid_body_state = torch.zeros((N, self.num_bodies, 13), device=dev)
        self._rigid_body_state_reshaped = self._rigid_body_state
        self._rigid_body_pos = self._rigid_body_state[..., 0:3]
        self._rigid_body_rot = self._rigid_body_state[..., 3:7]
        self._rigid_body_vel = self._rigid_body_state[..., 7:10]
        self._rigid_body_ang_vel = self._rigid_body_state[..., 10:13]
        self._rigid_body_rot[..., 3] = 1.0
        self._humanoid_root_states = torch.zeros((N, 13), device=dev)
        self._dof_state = torch.zeros((N, self.num_dof, 2), device=dev)
        self._dof_pos = self._dof_state[..., 0]
        self._dof_vel = self._dof_state[..., 1]
        self.dof_force_tensor = torch.zeros((N, self.num_dof), device=dev)
        self.pd_target = torch.zeros((N, self.num_dof), device=dev)
        self.obs_buf = torch.zeros((N, self.num_obs), device=dev)
        self.rew_buf = torch.zeros(N, device=dev)
        self.reward_raw = torch.zeros((N, self.cfg.reward.imitation_reward_dim + 1), device=dev)
        self.progress_buf = torch.zeros(N, dtype=torch.int16, device=dev)
        self.reset_buf = torch.ones(N, dtype=torch.bool, device=dev)
        self._terminate_buf = torch.ones(N, dtype=torch.bool, device=dev)
        self.extras = {}
        self._global_offset = torch.zeros((N, 3), device=dev)
        self._motion_start_times = torch.zeros(N, device=dev)
        self._motion_start_times_offset = torch.zeros(N, device=dev)
        self._motion_sample_start_idx = 0
        self._sampled_motion_ids = torch.arange(N, device=dev)
        self._reset_mask = torch.zeros(N, dtype=torch.bool, device=dev)
        self._rng_counter_buf = torch.zeros(N, dtype=torch.int32, device=dev)
        # AMP history (humanoid_phc.py:600-611): frame 0 = current, 1.. = history
        self._amp_c = None
        if self.cfg.use_amp_obs:
            assert self._num_amp_obs_per_step == _native.AMP_OBS_STEP
            self._amp_obs_buf = torch.zeros((N, self.cfg.num_amp_obs_steps, self._num_amp_obs_per_step), device=dev)
            self._curr_amp_obs_buf = self._amp_obs_buf[:, 0]
            self._hist_amp_obs_buf = self._amp_obs_buf[:, 1:]
            self._amp_obs_demo_buf = torch.zeros_like(self._amp_obs_buf)
            self._amp_c = _native.amp_struct(self._amp_obs_buf, self._amp_obs_demo_buf)
        self._puffer = {}
        self._env_c = None
        # the policy's fused obs operand (set_obs_operand): (out, mean, var, eps, clip) or None, and
        # whether the last obs write (a fused step) also wrote it
        self._obs_operand = None
        self.obs_operand_fresh = False
        self._build_structs()

    def attach_puffer_buffers(self, terminals, truncations, masks, episode_return, episode_length, stats):
        """PHCPufferEnv's bookkeeping buffers, updated inside the fused step kernel."""
        self._puffer = dict(terminals=terminals, truncations=truncations, masks=masks,
                            episode_return=episode_return, episode_length=episode_length, stats=stats)
        self._build_structs()

    def _build_structs(self):
        self._env_c = _native.env_struct(
            self.cfg.num_envs, self._rigid_body_state, self._humanoid_root_states, self._dof_state,
            self.dof_force_tensor, self.progress_buf, self._sampled_motion_ids, self._motion_start_times,
            self._motion_start_times_offset, self._global_offset, self.obs_buf, self.rew_buf, self.reward_raw,
            self.reset_buf, self._terminate_buf, rng_counter=self._rng_counter_buf, **self._puffer)
        if self._obs_operand is not None:
            _native.set_obs_operand(self._env_c, *self._obs_operand)
        self._build_step_params()

    def set_obs_operand(self, out, mean, var, eps, clip):
        """R17 fused into the step: every phc_env_step / phc_env_step_replay launch also writes
        RunningNorm(obs) (running stats mean / var, eps, clip) as the policy's padded f16 / bf16
        first-GEMM operand into out [N, ld] (phc_obs_half's values).  The reset kernels do not:
        obs_operand_fresh says whether the operand matches obs_buf after the last launch.  out
        None detaches it."""
        self._obs_operand = None if out is None else (out, mean, var, float(eps), float(clip))
        _native.set_obs_operand(self._env_c, out, mean, var, eps, clip)
        self.obs_operand_fresh = False

    def _build_step_params(self):
        args = (self.dt, self.cfg.reward, self.cfg.rew_power_coef, self.cfg.reward.use_power_reward,
                self.cfg.enable_early_termination, self.flag_im_eval, self._reset_bodies_id,
                self._termination_distances.detach().cpu().tolist())
        seed = int(self.cfg.seed) * 7919 + 17
        # _sample_ref_state (humanoid_phc.py:843-855): StateInit.Start or eval (flag_test) -> time 0
        at_start = self.flag_test or self.cfg.state_init == StateInit.Start
        self._step_params = _native.step_params_struct(*args, auto_reset=False, seed=seed, reset_at_start=at_start)
        self._step_params_auto = _native.step_params_struct(*args, auto_reset=True, seed=seed,
                                                            reset_at_start=at_start)

    def _load_motion(self, motion_train_file):
        """humanoid_phc.py:620-657: train + eval libraries, even initial sampling."""
        from types import SimpleNamespace

        from ..motion_lib import PackedMotions

        if isinstance(motion_train_file, PackedMotions):
            self._motion_train_lib = MotionLibSMPL.from_packed(motion_train_file, self.device, self.dt)
            self._motion_eval_lib = self._motion_lib = self._motion_train_lib
            m = int(motion_train_file.num_frames.shape[0])
            if m < self.num_envs:
                # fewer clips than envs: env i plays clip i mod M (load_motions' remainder
                # sampling, motion_lib.py:304-312); the kernels index the library by these ids
                self._sampled_motion_ids.copy_(torch.arange(self.num_envs, device=self.device) % m)
            return
        mcfg = SimpleNamespace(motion_file=motion_train_file, device=self.device, fix_height=FixHeightMode.full_fix,
                               min_length=self.cfg.min_motion_len, max_length=self.cfg.max_episode_length,
                               im_eval=self.flag_im_eval, num_thread=1, smpl_type=self.cfg.robot.humanoid_type,
                               step_dt=self.dt, is_deterministic=self.flag_debug)
        self._motion_train_lib = MotionLibSMPL(mcfg)
        self._motion_lib = self._motion_train_lib
        ecfg = SimpleNamespace(**vars(mcfg))
        ecfg.im_eval = True
        self._motion_eval_lib = MotionLibSMPL(ecfg)
        interval = self.num_unique_motions / (self.cfg.num_envs + 50)
        idx = np.floor(np.arange(0, self.num_unique_motions, interval)).astype(int)[: self.cfg.num_envs]
        self._motion_lib.load_motions(skeleton_trees=self.skeleton_trees, gender_betas=self.humanoid_shapes.cpu(),
                                      limb_weights=self.humanoid_limb_and_weights.cpu(),
                                      sample_idxes=torch.from_numpy(idx).to(self.device))

    # ------------------------------------------------------------- API --
    def _next_counter(self):
        self._rng_counter += 1
        return self._rng_counter

    def reset(self, env_ids=None):
        """humanoid_phc.py:90-103.  A full reset re-initialises twice (the reference's
        squash-reset around one extra simulate; with replay physics the second draw wins)."""
        if env_ids is None:
            mask = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
            for _ in range(2):
                _native.reset_envs(self._env_c, self._motion_lib.packed.c, self._step_params, mask=mask,
                                   seed=self._rng_seed, counter=self._next_counter())
        else:
            env_ids = torch.as_tensor(env_ids, device=self.device).long()
            self._reset_mask.zero_()
            self._reset_mask[env_ids] = True
            _native.reset_envs(self._env_c, self._motion_lib.packed.c, self._step_params, mask=self._reset_mask,
                               seed=self._rng_seed, counter=self._next_counter())
        self.obs_operand_fresh = False  # the reset kernel writes obs rows but not the fused operand
        self._init_amp_obs()
        return self.obs_buf

    def _init_amp_obs(self):
        """_init_amp_obs (humanoid_phc.py:789-836) of every env that was just reset (progress 0)."""
        if self._amp_c is not None:
            _native.amp_obs(self._env_c, self._motion_lib.packed.c, self._amp_c, self.dt, _native.AMP_INIT)

    def reset_done(self):
        """Reset every env whose reset_buf is set (PHCPufferEnv's nonzero(reset_buf) + reset,
        clean_pufferl/env.py:114-116, without leaving the device)."""
        _native.reset_envs(self._env_c, self._motion_lib.packed.c, self._step_params, mask=None,
                           seed=self._rng_seed, counter=self._next_counter())
        self.obs_operand_fresh = False
        self._init_amp_obs()

    def launch_key(self):
        """Everything a captured step launch holds by value: the env struct, the packed library's
        descriptor (replaced by resample_motions / the eval toggles) and both step-parameter blocks.
        A graph captured under another key replays stale pointers.  The kernel timer (by its never-reused
        serial) is part of the key: a graph must not stamp into a timer that was replaced or freed."""
        parts = [bytes(self._env_c), bytes(self._motion_lib.packed.c), bytes(self._step_params)]
        auto = getattr(self, "_step_params_auto", None)
        if auto is not None:
            parts.append(bytes(auto))
        # a captured step launch stamps into its kernel timer's buffer (or into none): another timer, or
        # none, needs other launches
        timer = self.kernel_timer
        parts.append(str(timer.serial if timer is not None else 0).encode())
        return b"".join(parts)

    def stats_env_struct(self, stats):
        """A copy of the env struct whose per-workgroup logging rows go to `stats` (same shape as
        PHCPufferEnv.stats): the captured rollout block gives every step its own rows."""
        c = type(self._env_c).from_buffer_copy(self._env_c)
        c.stats = _native._ptr(stats, torch.float64, tuple(self._puffer["stats"].shape), "stats")
        return c

    def step(self, actions, auto_reset=False, env_c=None):
        """humanoid_phc.py:105-172 with the physics stand-in.  With auto_reset (used by
        PHCPufferEnv) the envs that come up for reset are re-initialised inside the same
        fused kernel, as PHCPufferEnv.step's env.reset(reset_indices) does next.  env_c: the env
        struct of the fused replay launch (stats_env_struct), default the env's own."""
        if actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.float().contiguous()
        # eval mode records MPJPE / positions of the step's own outcome before the envs reset
        # (the reference resets after HumanoidPHC.step returns): no in-launch reset there
        fused_reset = auto_reset and not self.flag_im_eval
        params = self._step_params_auto if fused_reset else self._step_params
        clip = bool(self.cfg.clip_actions)  # clean_pufferl/env.py:91: np.clip only when cfg.clip_actions
        pd = _native.pd_map(actions, self.pd_target, self._pd_action_offset, self._pd_action_scale, self._pd_frozen,
                            clip)
        if self.fused_env_step and hasattr(self.physics, "step_fused"):
            # R13 + the physics stand-in + the env step: one launch
            self.physics.step_fused(self, params, pd, timer=self.kernel_timer, env_c=env_c)
        else:
            if env_c is not None:
                raise ValueError("HumanoidPHC.step: env_c needs the fused replay step")
            if hasattr(self.physics, "step_actions"):  # R13 folded into the physics launch
                self.physics.step_actions(self, pd)
            else:
                _native.actions_to_pd(actions, self.pd_target, self._pd_action_offset, self._pd_action_scale,
                                      self._pd_frozen, clip)
                self.physics.step(self)
            _native.env_step(self._env_c, self._motion_lib.packed.c, params, timer=self.kernel_timer)
        if fused_reset and "terminals" in self._puffer:
            self.extras["terminate"] = self._puffer["terminals"]  # this step's outcome, written by the kernel
        else:
            self.extras["terminate"] = self._terminate_buf.clone()
        self.extras["reward_raw"] = self.reward_raw
        if self._amp_c is not None:
            # _update_hist_amp_obs + _compute_amp_observations (humanoid_phc.py:154-157); envs that
            # auto-reset in this step (progress 0) get _init_amp_obs instead, as reset() would
            _native.amp_obs(self._env_c, self._motion_lib.packed.c, self._amp_c, self.dt, _native.AMP_STEP)
            self.extras["amp_obs"] = self.amp_obs
        if self.flag_im_eval:
            t = self.progress_buf * self.dt + self._motion_start_times + self._motion_start_times_offset
            res = self._motion_lib.get_motion_state(self._sampled_motion_ids, t, self._global_offset)
            self.extras["mpjpe"] = (self._rigid_body_pos - res["rg_pos"]).norm(dim=-1).mean(dim=-1)
            self.extras["body_pos"] = self._rigid_body_pos.cpu().numpy()
            self.extras["body_pos_gt"] = res["rg_pos"].cpu().numpy()
        # every obs row of this step came from the step kernel, which also wrote the fused operand
        self.obs_operand_fresh = self._obs_operand is not None
        if auto_reset and not fused_reset:
            self.reset_done()  # PHCPufferEnv.step's env.reset(reset_indices), clean_pufferl/env.py:114-116
        return self.obs_buf, self.rew_buf, self.reset_buf, self.extras

    def render(self):
        pass

    def close(self):
        pass

    # ---------------------------------------------------- eval / motions --
    def set_termination_distances(self, termination_distances):
        self._termination_distances[:] = termination_distances
        self._build_step_params()

    def resample_motions(self):
        """humanoid_phc.py:1361-1377."""
        if self.flag_test:
            self.forward_motion_samples()
            return
        self._motion_lib.load_motions(skeleton_trees=self.skeleton_trees,
                                      limb_weights=self.humanoid_limb_and_weights.cpu(),
                                      gender_betas=self.humanoid_shapes.cpu(),
                                      random_sample=(not self.flag_test) and (not self.cfg.seq_motions))
        t = self.progress_buf * self.dt + self._motion_start_times + self._motion_start_times_offset
        root = self._motion_lib.get_root_pos_smpl(self._sampled_motion_ids, t)["root_pos"]
        self._global_offset[:, :2] = self._humanoid_root_states[:, :2] - root[:, :2]
        self.reset()

    def begin_seq_motion_samples(self, start_idx=0):
        self._motion_sample_start_idx = start_idx
        self._motion_lib.load_motions(skeleton_trees=self.skeleton_trees, gender_betas=self.humanoid_shapes.cpu(),
                                      limb_weights=self.humanoid_limb_and_weights.cpu(), random_sample=False,
                                      start_idx=self._motion_sample_start_idx)
        self.reset()

    def forward_motion_samples(self):
        # eval sharded over data-parallel ranks: this rank's next batch is `world` batches on
        self._motion_sample_start_idx += self.cfg.num_envs * getattr(self, "_eval_world", 1)
        self._motion_lib.load_motions(skeleton_trees=self.skeleton_trees, gender_betas=self.humanoid_shapes.cpu(),
                                      limb_weights=self.humanoid_limb_and_weights.cpu(), random_sample=False,
                                      start_idx=self._motion_sample_start_idx)
        self.reset()

    @property
    def num_unique_motions(self):
        return self._motion_lib._num_unique_motions

    @property
    def current_motion_ids(self):
        return self._motion_lib._curr_motion_ids

    @property
    def motion_sample_start_idx(self):
        return self._motion_sample_start_idx

    @property
    def motion_data_keys(self):
        return self._motion_lib._motion_data_keys

    def get_motion_steps(self):
        return self._motion_lib.get_motion_num_steps()

    def toggle_eval_mode(self, shard=(0, 1)):
        """humanoid_phc.py:1424-1436.  shard = (rank, world): the sequential motion batches are
        dealt round-robin over the data-parallel ranks (batch b on rank b % world; eval_stats.py
        merges the ranks' results)."""
        rank, world = shard
        self._eval_world = int(world)
        self.flag_test = True
        self.flag_im_eval = True
        self._termination_distances[:] = 0.5
        self._motion_lib = self._motion_eval_lib
        if len(self._reset_bodies_id) > 15:
            self._reset_bodies_id = list(self._eval_track_bodies_id)
        self._build_step_params()
        self.begin_seq_motion_samples(int(rank) * self.cfg.num_envs)
        return self._motion_lib._num_unique_motions

    def untoggle_eval_mode(self, failed_keys):
        """humanoid_phc.py:1438-1454."""
        self.flag_test = False
        self.flag_im_eval = False
        self._eval_world = 1
        self._termination_distances[:] = self._termination_distances_backup
        self._motion_lib = self._motion_train_lib
        self._reset_bodies_id = list(self._reset_bodies_id_backup)
        self._build_step_params()
        if self.cfg.auto_pmcp:
            self._motion_lib.update_hard_sampling_weight(failed_keys)
        elif self.cfg.auto_pmcp_soft:
            self._motion_lib.update_soft_sampling_weight(failed_keys)
        return self._motion_lib._termination_history.clone()

    @property
    def amp_obs(self):
        return self._amp_obs_buf.view(-1, self.num_amp_obs) if self._amp_c is not None else None

    def fetch_amp_obs_demo(self):
        return self._amp_obs_demo_buf.view(-1, self.num_amp_obs) if self._amp_c is not None else None
