"""Configuration dataclasses (puffer_phc/config.py:9-196), same fields and defaults.

tyro is not available offline; `scripts/train.py` parses the same dotted flags
(`--env.num-envs`, `--train.batch-size`, ...) with argparse.  `robot` and `reward` stay
non-CLI (the reference marks them `Suppress`).
"""

import os
from dataclasses import dataclass, field
from typing import Literal, Optional, Tuple

from .envs.state_init import StateInit


def env_flag(name, default):
    """A boolean switch from the environment, read when a config is constructed (not at import):
    1 / true / yes / on enable it, 0 / false / no / off disable it, anything else is an error."""
    v = os.environ.get(name)
    if v is None or v.strip() == "":
        return default
    v = v.strip().lower()
    if v in ("1", "true", "yes", "on"):
        return True
    if v in ("0", "false", "no", "off"):
        return False
    raise ValueError(f"{name}={v!r}: expected 1/true/yes/on or 0/false/no/off")


@dataclass
class DeviceConfig:
    device_type: Literal["cpu", "cuda"] = "cuda"
    device_id: int = 0

    @property
    def device(self) -> str:
        return "cpu" if self.device_type == "cpu" else f"cuda:{self.device_id}"


@dataclass
class RewardConfig:
    k_pos: float = 100.0
    k_rot: float = 10.0
    k_vel: float = 0.1
    k_ang_vel: float = 0.1
    w_pos: float = 0.5
    w_rot: float = 0.3
    w_vel: float = 0.1
    w_ang_vel: float = 0.1
    imitation_reward_dim: int = 4
    full_body_reward: bool = True
    use_power_reward: bool = True


@dataclass
class RobotConfig:
    humanoid_type: Literal["smpl"] = "smpl"
    has_self_collision: bool = True
    has_smpl_pd_offset: bool = False
    has_upright_start: bool = True
    has_dof_subset: bool = True
    has_mesh: bool = False
    has_shape_obs: bool = False
    has_shape_obs_disc: bool = False
    has_limb_weight_obs: bool = False
    has_limb_weight_obs_disc: bool = False
    reduce_action: bool = False
    freeze_hand: bool = True
    freeze_toe: bool = True
    reduced_action_idx = (0, 1, 2, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 16, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28,
                          29, 30, 31, 32, 33, 34, 36, 37, 42, 43, 44, 47, 48, 49, 50, 57, 58, 59, 62, 63, 64, 65)
    bias_offset: bool = False


@dataclass
class EnvConfig(DeviceConfig):
    """Environment configuration"""

    name: str = "humanoid_phc"
    motion_file: str = "data/motion/amass_train_take6_upright.pkl"
    num_envs: int = 4096
    headless: bool = True
    exp_name: str = "puffer_phc"

    clip_actions: bool = True
    use_amp_obs: bool = False
    enable_early_termination: bool = True
    termination_distance: float = 0.25
    max_episode_length: int = 300

    auto_pmcp: bool = False
    auto_pmcp_soft: bool = True

    kp_scale: float = 1.0
    kd_scale: float = 1.0
    log_interval: int = 32

    res_action: bool = False

    rew_power_coef: float = 0.0005
    env_spacing: int = 5
    state_init: StateInit = StateInit.Random

    divide_group: bool = False
    collect_dataset: bool = False

    local_root_obs: bool = True
    root_height_obs: bool = True

    add_obs_noise: bool = False
    obs_noise_std: float = 0.1
    add_action_noise: bool = False
    action_noise_std: float = 0.05

    num_states: int = 0
    control_mode: Literal["isaac_pd"] = "isaac_pd"

    seq_motions: bool = False
    min_motion_len: int = 5
    max_motion_len: int = 600
    hybrid_init_prob: float = 0.5

    num_amp_obs_steps: int = 10
    amp_root_height_obs: bool = True

    # physics: "replay" = the stand-in of BASELINE configs[1] (replayed reference states + gaussian
    # noise); "articulated" = the N3 articulated-body step (physics.ArticulatedPhysics)
    physics: Literal["replay", "articulated"] = "replay"
    physics_substeps: int = 8
    replay_pos_sigma: float = 0.02
    replay_force_scale: float = 50.0
    # replay physics: the action -> PD map, the stand-in and the env step in one launch
    # (phc_env_step_replay); False = three launches (same values)
    fused_env_step: bool = True
    seed: int = 0

    robot: RobotConfig = field(default_factory=RobotConfig)
    reward: RewardConfig = field(default_factory=RewardConfig)

    @property
    def num_agents(self) -> int:
        return self.num_envs


@dataclass
class PolicyConfig:
    hidden_size: int = 512
    layer_sizes: Tuple[int, ...] = (2048, 1536, 1024, 1024, 512)


@dataclass
class RNNConfig:
    input_size: int = 512
    hidden_size: int = 512


@dataclass
class TrainConfig(DeviceConfig):
    """Training configuration"""

    seed: int = 1
    torch_deterministic: bool = True
    cpu_offload: bool = False
    compile: bool = False
    norm_adv: bool = True
    target_kl: Optional[float] = None

    total_timesteps: int = 500_000_000
    eval_timesteps: int = 1_310_000

    data_dir: str = "experiments"
    checkpoint_interval: int = 1500
    motion_resample_interval: int = 500

    num_workers: int = 1
    num_envs: int = 1
    batch_size: int = 131072
    minibatch_size: int = 32768

    learning_rate: float = 0.0001
    anneal_lr: bool = False
    lr_decay_rate: float = 1.5e-4
    lr_decay_floor: float = 0.2

    update_epochs: int = 4
    bptt_horizon: int = 8
    gae_lambda: float = 0.2
    gamma: float = 0.98
    clip_coef: float = 0.01
    vf_coef: float = 1.2
    clip_vloss: bool = True
    vf_clip_coef: float = 0.2
    max_grad_norm: float = 10.0
    ent_coef: float = 0.0
    disc_coef: float = 5.0
    bound_coef: float = 10.0
    # the reference reads policy.mean_bound_loss ONCE at the start of train() (core.py:225): the
    # value of the last rollout forward, computed under no_grad, so `loss += mean_bound_loss *
    # bound_coef` (core.py:349-350) adds a constant -- no gradient -- and the logged value is
    # that constant.  False (default) = exactly that; True = a per-minibatch bound loss that
    # does backpropagate into mu (a deliberate deviation, off by default)
    bound_loss_grad: bool = False
    l2_reg_coef: float = 0.0
    # policy GEMM arithmetic.  "fp16" (default) = fp16 GEMM operands on the hand-written MFMA
    # GEMM (phc_gemm.hip), fp32 accumulation and outputs, epilogues in fp32: TF32's arithmetic
    # (the reference sets torch.set_float32_matmul_precision("high"), clean_pufferl/core.py:38)
    # with dynamic loss scaling for fp16's narrower exponent range (tests/test_gpu_twin_mlp.py
    # test_fp16_operands_match_tf32_error); "xf32" = float32 storage with hipBLASLt's xf32
    # emulation (torch "high" on gfx950, bf16x3: more accurate than TF32, 2.3x slower);
    # "bf16" = bf16 operands (BASELINE config C5).
    precision: str = "fp16"
    # replay policy inference + experience store of each rollout step from a captured hipGraph
    # (the env step itself stays eager); False = the reference's eager loop
    rollout_graph: bool = field(default_factory=lambda: env_flag("PHC_ROLLOUT_GRAPH", True))
    # PPO objective (ratio / clipping / value / bound losses and their gradients) in two HIP
    # kernels (clean_pufferl/ppo_loss.py); False = the reference's eager expression
    fused_loss: bool = True
    # rollout inference tail (LayerNorm+SiLU, mu / value heads, Normal sample, log_prob) in one
    # HIP kernel (phc_policy_act) on the half-precision MFMA path; False = the policy module
    fused_act: bool = True
    # train(): normalise + round the whole batch's observations into the first GEMM's half
    # operand once per call, in minibatch order (phc_obs_half); False = per minibatch, fp32
    fused_obs: bool = True
    # rollout: the env step kernel also writes RunningNorm(obs) as the first GEMM's half operand
    # (HumanoidPHC.set_obs_operand); False = a phc_obs_half launch per rollout step
    fused_obs_operand: bool = field(default_factory=lambda: env_flag("PHC_FUSED_OBS_OPERAND", True))
