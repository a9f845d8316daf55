"""ctypes binding of libphc_hip.so (include/phc.h) on PyTorch-ROCm tensors.

PyTorch is plumbing here: it owns device memory and streams.  Every op validates shape,
dtype, device and contiguity (raising ValueError like the reference's
gymtorch.unwrap_tensor, gymtorch/gymtorch/wrapper.py:47-56) and then calls the C ABI on the
current HIP stream.  There is no CPU fallback: if the library cannot be loaded, importing
any op raises.
"""

import ctypes
import itertools
import os

import numpy as np
import torch

_LIB_PATH = os.environ.get(
    "PHC_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libphc_hip.so")
)

NUM_BODIES = 24
NUM_DOF = 69
BODY_STRIDE = 13
OBS_DIM = 934
AMP_OBS_STEP = 196
AMP_STEP, AMP_INIT = 0, 1
STATS_SLOTS = 16

c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p


class MotionLibC(ctypes.Structure):
    _fields_ = [("frames", c_vp), ("local_rot", c_vp), ("dof_vel", c_vp), ("motion_len", c_vp),
                ("motion_dt", c_vp), ("num_frames", c_vp), ("length_starts", c_vp),
                ("num_motions", c_i64), ("num_frames_total", c_i64)]


class RefStateC(ctypes.Structure):
    _fields_ = [("body", c_vp), ("dof_pos", c_vp), ("dof_vel", c_vp)]


class EnvBuffersC(ctypes.Structure):
    _fields_ = [("num_envs", c_i64), ("rigid_body_state", c_vp), ("root_state", c_vp), ("dof_state", c_vp),
                ("dof_force", c_vp), ("progress", c_vp), ("motion_ids", c_vp), ("motion_start_times", c_vp),
                ("motion_start_offset", c_vp), ("global_offset", c_vp), ("obs", c_vp), ("rew", c_vp),
                ("reward_raw", c_vp), ("reset", c_vp), ("terminate", c_vp), ("terminals", c_vp),
                ("truncations", c_vp), ("masks", c_vp), ("episode_return", c_vp), ("episode_length", c_vp),
                ("stats", c_vp), ("rng_counter", c_vp), ("obs_operand", c_vp), ("obs_norm_mean", c_vp),
                ("obs_norm_var", c_vp), ("obs_norm_eps", ctypes.c_float), ("obs_norm_clip", ctypes.c_float),
                ("obs_operand_ld", ctypes.c_int32), ("obs_operand_dtype", ctypes.c_int32)]


def set_obs_operand(env_c, out, mean, var, eps, clip):
    """Have phc_env_step / phc_env_step_replay also write RunningNorm(obs) as the policy's padded
    f16 / bf16 first-GEMM operand into out [N, ld] (phc_obs_half's values); out None clears it."""
    if out is None:
        env_c.obs_operand = None
        env_c.obs_norm_mean = env_c.obs_norm_var = None
        env_c.obs_operand_ld = env_c.obs_operand_dtype = 0
        return
    N = int(env_c.num_envs)
    if out.dim() != 2 or out.shape[0] != N or out.shape[1] < OBS_DIM or out.shape[1] % 8 or not out.is_contiguous() \
            or out.data_ptr() % 16 or out.dtype not in (torch.float16, torch.bfloat16) or not out.is_cuda:
        raise ValueError("obs operand must be a contiguous 16-B aligned f16 / bf16 device [num_envs, ld] tensor, "
                         "ld >= 934, ld % 8 == 0")
    env_c.obs_operand = out.data_ptr()
    env_c.obs_norm_mean = _ptr(mean.reshape(-1), torch.float32, (OBS_DIM,), "running_mean")
    env_c.obs_norm_var = _ptr(var.reshape(-1), torch.float32, (OBS_DIM,), "running_var")
    env_c.obs_norm_eps, env_c.obs_norm_clip = float(eps), float(clip)
    env_c.obs_operand_ld = out.shape[1]
    env_c.obs_operand_dtype = DTYPE_CODE[out.dtype]


class StepParamsC(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_float), ("k_pos", ctypes.c_float), ("k_rot", ctypes.c_float),
                ("k_vel", ctypes.c_float), ("k_ang_vel", ctypes.c_float), ("w_pos", ctypes.c_float),
                ("w_rot", ctypes.c_float), ("w_vel", ctypes.c_float), ("w_ang_vel", ctypes.c_float),
                ("power_coef", ctypes.c_float), ("use_power_reward", ctypes.c_int32),
                ("enable_early_termination", ctypes.c_int32), ("use_mean_termination", ctypes.c_int32),
                ("reset_body_mask", ctypes.c_uint32), ("termination_distance", ctypes.c_float * NUM_BODIES),
                ("auto_reset", ctypes.c_int32), ("reset_at_start", ctypes.c_int32), ("seed", ctypes.c_uint64)]


class PhysicsParamsC(ctypes.Structure):
    _fields_ = [("sim_dt", ctypes.c_float), ("control_freq_inv", ctypes.c_int32), ("substeps", ctypes.c_int32),
                ("tree_depth", ctypes.c_int32), ("kp_scale", ctypes.c_float), ("kd_scale", ctypes.c_float),
                ("contact_stiffness", ctypes.c_float), ("contact_damping", ctypes.c_float),
                ("friction", ctypes.c_float), ("friction_damping", ctypes.c_float), ("gravity", ctypes.c_float),
                ("angular_damping", ctypes.c_float), ("max_angular_velocity", ctypes.c_float),
                ("self_collision", ctypes.c_int32)]


class PdMapC(ctypes.Structure):
    _fields_ = [("actions", c_vp), ("pd_target", c_vp), ("offset", c_vp), ("scale", c_vp), ("frozen", c_vp),
                ("clip", ctypes.c_int32)]


class ReplayParamsC(ctypes.Structure):
    _fields_ = [("pos_sigma", ctypes.c_float), ("force_scale", ctypes.c_float), ("seed", ctypes.c_uint64),
                ("counter", ctypes.c_uint64)]


class RowFieldC(ctypes.Structure):
    _fields_ = [("src", c_vp), ("dst", c_vp), ("row_elems", c_i64), ("kind", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


MAX_ROW_FIELDS = 12
ROW_COPY32, ROW_COPY64, ROW_U8_TO_F32 = 0, 1, 2
ROW_SRC_WORDS = 1  # phc_row_field.flags: the source's covering aligned words are inside its allocation


def _words_inside_storage(t):
    """Whether every aligned 4-byte word overlapping t's bytes lies inside t's storage (what
    PHC_ROW_SRC_WORDS vouches for: a flag field may then be read through its aligned words)."""
    st = t.untyped_storage()
    base, end = st.data_ptr(), st.data_ptr() + st.nbytes()
    lo = t.data_ptr()
    hi = lo + t.numel() * t.element_size()
    return t.numel() > 0 and (lo & ~3) >= base and ((hi - 1) & ~3) + 4 <= end


class PpoCoefsC(ctypes.Structure):
    _fields_ = [("clip_coef", ctypes.c_float), ("vf_clip_coef", ctypes.c_float), ("vf_coef", ctypes.c_float),
                ("ent_coef", ctypes.c_float), ("bound_coef", ctypes.c_float), ("soft_bound", ctypes.c_float),
                ("clip_vloss", ctypes.c_int32), ("reserved", ctypes.c_int32)]


PPO_STATS = 7


class TailLnArgsC(ctypes.Structure):
    _fields_ = [("trunk_out", c_vp), ("ln_gamma", c_vp * 2), ("ln_beta", c_vp * 2), ("w_value", c_vp),
                ("b_value", c_vp), ("h_actor", c_vp), ("value", c_vp), ("rows", c_i64), ("hidden", ctypes.c_int32),
                ("ln_eps", ctypes.c_float)]


class AmpBuffersC(ctypes.Structure):
    _fields_ = [("amp_obs", c_vp), ("amp_obs_demo", c_vp), ("num_steps", ctypes.c_int32)]


class GemmDescC(ctypes.Structure):
    _fields_ = [("a", c_vp), ("b", c_vp), ("a_batch_stride", c_i64), ("b_batch_stride", c_i64), ("lda", c_i64),
                ("ldb", c_i64), ("m", c_i64), ("n", ctypes.c_int32), ("k", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("dtype", ctypes.c_int32), ("epilogue", ctypes.c_int32),
                ("out_dtype", ctypes.c_int32), ("bias", c_vp), ("aux", c_vp), ("out", c_vp),
                ("aux_layout", ctypes.c_int32), ("out_layout", ctypes.c_int32), ("twin_groups", ctypes.c_int32),
                ("twin_cols", ctypes.c_int32), ("aux_dtype", ctypes.c_int32), ("max_workgroups", ctypes.c_int32),
                ("k_valid", ctypes.c_int32)]


EPI_STORE, EPI_BIAS, EPI_BIAS_SILU, EPI_SILU_GRAD, EPI_BIAS_RELU, EPI_RELU_GRAD = 0, 1, 2, 3, 4, 5
# the silu'-aux pair (phc.h): the forward stores silu'(pre) instead of pre, the input gradient multiplies by it
EPI_BIAS_SILU_D, EPI_DSILU_GRAD = 6, 7


class WgradDescC(ctypes.Structure):
    _fields_ = [("g", c_vp), ("z", c_vp), ("g_batch_stride", c_i64), ("z_batch_stride", c_i64), ("ldg", c_i64),
                ("ldz", c_i64), ("rows", c_i64), ("m", ctypes.c_int32), ("n", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("dtype", ctypes.c_int32), ("splits", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("out", c_vp)]


class WgradProblemC(ctypes.Structure):
    _fields_ = [("g", c_vp), ("z", c_vp), ("g_batch_stride", c_i64), ("z_batch_stride", c_i64), ("ldg", c_i64),
                ("ldz", c_i64), ("dst", c_vp * 2), ("ldd", c_i64), ("m", ctypes.c_int32), ("n", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("split_row", ctypes.c_int32), ("n_valid", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


WGRAD_GROUP_MAX = 8


class ReduceJobC(ctypes.Structure):
    _fields_ = [("src", c_vp), ("dst", c_vp), ("rows", c_i64), ("cols", c_i64), ("src_ld", c_i64),
                ("part_stride", c_i64), ("parts", ctypes.c_int32), ("accumulate", ctypes.c_int32)]


MAX_REDUCE_JOBS = 32


class PackJobC(ctypes.Structure):
    _fields_ = [("src", c_vp), ("dst", c_vp), ("dst_t", c_vp), ("rows", c_i64), ("cols", c_i64), ("src_ld", c_i64),
                ("dst_ld", c_i64), ("dst_t_ld", c_i64), ("dtype", ctypes.c_int32), ("reserved", ctypes.c_int32)]


MAX_PACK_JOBS = 32


class AdamJobC(ctypes.Structure):
    _fields_ = [("off", c_i64), ("rows", c_i64), ("cols", c_i64), ("dst", c_vp), ("dst_t", c_vp), ("dst_ld", c_i64),
                ("dst_t_ld", c_i64), ("first_block", c_i64), ("tiles_c", c_i64), ("dtype", ctypes.c_int32),
                ("kind", ctypes.c_int32)]


MAX_ADAM_JOBS = 256
ADAM_FLAT, ADAM_TILE = 0, 1


class PolicyActArgsC(ctypes.Structure):
    _fields_ = [("trunk_out", c_vp), ("ln_gamma", c_vp * 2), ("ln_beta", c_vp * 2), ("w_mu", c_vp), ("b_mu", c_vp),
                ("w_value", c_vp), ("b_value", c_vp), ("log_sigma", c_vp), ("noise", c_vp), ("actions", c_vp),
                ("logprob", c_vp), ("value", c_vp), ("mu", c_vp), ("rows", c_i64), ("hidden", ctypes.c_int32),
                ("num_actions", ctypes.c_int32), ("ln_eps", ctypes.c_float), ("std_max", ctypes.c_float),
                ("w_mu_t", c_vp), ("ld_w_mu_t", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class AdamParamsC(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("max_norm", ctypes.c_float), ("use_loss_scale", ctypes.c_int32), ("growth_factor", ctypes.c_float),
                ("backoff_factor", ctypes.c_float), ("growth_interval", ctypes.c_int32),
                ("lr_from_state", ctypes.c_int32)]


class OptStateC(ctypes.Structure):
    _fields_ = [("loss_scale", ctypes.c_float), ("growth_tracker", ctypes.c_int32), ("step", ctypes.c_int32),
                ("skipped", ctypes.c_int32), ("grad_mul", ctypes.c_float), ("step_size", ctypes.c_float),
                ("bc2_sqrt", ctypes.c_float), ("skip", ctypes.c_int32), ("lr", ctypes.c_float),
                ("reserved", ctypes.c_int32)]


_EXPORTS = {
    "phc_version": (ctypes.c_int, []),
    "phc_last_error": (ctypes.c_char_p, []),
    "phc_stats_blocks": (c_i64, [c_i64]),
    "phc_motion_state": (ctypes.c_int, [ctypes.POINTER(MotionLibC), c_vp, c_vp, c_vp, c_i64,
                                         ctypes.POINTER(RefStateC), c_vp]),
    "phc_env_step": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                     ctypes.POINTER(StepParamsC), c_vp]),
    "phc_timer_create": (c_vp, [ctypes.c_int32]),
    "phc_timer_destroy": (None, [c_vp]),
    "phc_timer_reset": (None, [c_vp]),
    "phc_timer_count": (ctypes.c_int32, [c_vp]),
    "phc_timer_set_period": (None, [c_vp, ctypes.c_int32]),
    "phc_timer_offered": (ctypes.c_int64, [c_vp]),
    "phc_timer_total_ms": (ctypes.c_double, [c_vp]),
    "phc_timer_work": (ctypes.c_double, [c_vp]),
    "phc_timer_durations": (ctypes.c_int32, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int32]),
    "phc_gemm_set_timer": (None, [c_vp]),
    "phc_env_step_timed": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                           ctypes.POINTER(StepParamsC), c_vp, c_vp]),
    "phc_reset_envs": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                       ctypes.POINTER(StepParamsC), c_vp, c_vp, ctypes.c_uint64, ctypes.c_uint64,
                                       c_vp]),
    "phc_amp_obs": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                    ctypes.POINTER(AmpBuffersC), ctypes.c_float, ctypes.c_int32, c_vp]),
    "phc_actions_to_pd": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, ctypes.c_int32, c_vp]),
    "phc_compact_workspace_bytes": (ctypes.c_size_t, [c_i64]),
    "phc_compact_rows": (ctypes.c_int, [ctypes.POINTER(RowFieldC), ctypes.c_int32, c_vp, c_i64, c_vp, c_i64, c_vp,
                                         c_vp, c_vp]),
    "phc_ln_silu_fwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_float, ctypes.c_int32, c_vp]),
    "phc_ln_silu_workspace_bytes": (ctypes.c_size_t, [c_i64, ctypes.c_int32, ctypes.c_int32]),
    "phc_ln_silu_bwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_int32, c_vp, c_vp]),
    "phc_twin_gemm_workspace_bytes": (ctypes.c_size_t, [c_i64, ctypes.c_int32, ctypes.c_int32]),
    "phc_twin_gemm": (ctypes.c_int, [ctypes.POINTER(GemmDescC), c_vp, c_vp, c_vp]),
    "phc_twin_gemm_m_tiles": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "phc_weight_grad": (ctypes.c_int, [ctypes.POINTER(WgradDescC), c_vp]),
    "phc_weight_grad_group": (ctypes.c_int, [ctypes.POINTER(WgradProblemC), ctypes.c_int32, c_i64, ctypes.c_int32,
                                              ctypes.c_int32, c_vp]),
    "phc_reduce_into": (ctypes.c_int, [ctypes.POINTER(ReduceJobC), ctypes.c_int32, c_vp]),
    "phc_pack_weights": (ctypes.c_int, [ctypes.POINTER(PackJobC), ctypes.c_int32, c_vp]),
    "phc_obs_half": (ctypes.c_int, [c_vp, c_vp, c_i64, ctypes.c_int32, c_vp, c_vp, ctypes.c_float, ctypes.c_float,
                                     c_vp, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "phc_policy_act": (ctypes.c_int, [ctypes.POINTER(PolicyActArgsC), c_vp]),
    "phc_opt_block_elems": (c_i64, []),
    "phc_opt_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "phc_opt_step": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, ctypes.c_int32, c_vp, ctypes.c_int32,
                                     ctypes.POINTER(AdamParamsC), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "phc_opt_step_operands": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, ctypes.c_int32, c_vp,
                                              ctypes.c_int32, ctypes.POINTER(AdamParamsC), c_vp, c_vp, c_vp, c_vp,
                                              c_vp, c_vp, ctypes.c_int32, c_i64, c_vp]),
    "phc_adam_job_blocks": (c_i64, [ctypes.c_int32, c_i64, c_i64]),
    "phc_ppo_workspace_bytes": (ctypes.c_size_t, [c_i64]),
    "phc_tail_layout": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    "phc_tail_blocks": (ctypes.c_int32, [c_i64]),
    "phc_tail_ln_fwd": (ctypes.c_int, [ctypes.POINTER(TailLnArgsC), c_vp]),
    "phc_mu_head_fwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "phc_mu_head_dgrad": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "phc_mu_head_wgrad": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          c_vp]),
    "phc_tail_ln_bwd": (ctypes.c_int, [ctypes.POINTER(TailLnArgsC), c_vp, c_vp, c_vp, ctypes.c_int32, c_vp,
                                        ctypes.c_int32, c_vp, c_vp]),
    "phc_ppo_loss_fwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int32,
                                         ctypes.POINTER(PpoCoefsC), c_vp, c_vp, c_vp, c_vp, c_vp]),
    "phc_ppo_loss_bwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int32,
                                         ctypes.POINTER(PpoCoefsC), c_vp, c_vp, c_vp]),
    "phc_bias_act_fwd": (ctypes.c_int, [c_vp, ctypes.c_int32, c_vp, c_vp, c_vp, ctypes.c_int32, c_i64, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "phc_act_bwd_workspace_bytes": (ctypes.c_size_t, [c_i64, ctypes.c_int32, ctypes.c_int32]),
    "phc_act_bwd": (ctypes.c_int, [c_vp, ctypes.c_int32, c_vp, ctypes.c_int32, c_vp, c_vp, ctypes.c_int32, c_vp,
                                    c_i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, c_vp, c_vp]),
    "phc_physics_replay": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                           ctypes.POINTER(StepParamsC), ctypes.c_float, ctypes.c_float,
                                           ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    "phc_physics_step": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), c_vp, c_vp, ctypes.POINTER(PhysicsParamsC),
                                         c_vp]),
    "phc_physics_step_timed": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), c_vp, c_vp,
                                               ctypes.POINTER(PhysicsParamsC), c_vp, c_vp]),
    "phc_physics_step_actions": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(PdMapC), c_vp,
                                                 ctypes.POINTER(PhysicsParamsC), c_vp, c_vp]),
    "phc_env_step_replay": (ctypes.c_int, [ctypes.POINTER(EnvBuffersC), ctypes.POINTER(MotionLibC),
                                            ctypes.POINTER(StepParamsC), ctypes.POINTER(ReplayParamsC),
                                            ctypes.POINTER(PdMapC), c_vp, c_vp]),
    "phc_fk_workspace_bytes": (ctypes.c_size_t, [c_i64]),
    "phc_fk_motions": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp,
                                       ctypes.c_int32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "phc_gae_workspace_bytes": (ctypes.c_size_t, [c_i64]),
    "phc_gae": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, ctypes.c_float, ctypes.c_float, c_vp, c_vp, c_vp]),
    "phc_rms_workspace_bytes": (ctypes.c_size_t, [c_i64, c_i64]),
    "phc_rms_update": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "phc_rms_moments": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "phc_rms_apply": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "phc_rms_normalize": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, ctypes.c_float, ctypes.c_float,
                                          c_vp]),
    "phc_disc_head_bwd_blocks": (c_i64, [c_i64]),
    "phc_disc_head_fwd": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_int32, ctypes.c_int32, c_vp, c_vp, c_vp, c_vp,
                                          c_vp]),
    "phc_disc_head_bwd": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_int32, ctypes.c_int32, c_vp, c_vp, c_vp, c_i64,
                                          c_vp, c_vp]),
}


def load_library(path=_LIB_PATH):
    """Load libphc_hip.so and declare every exported symbol; raises if absent."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"libphc_hip.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback for the PHC hot path)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = load_library()
    return _lib


def _check(rc, what):
    if rc != 0:
        msg = lib().phc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def _ptr(t, dtype, shape=None, name="tensor", nullable=False):
    if t is None:
        if nullable:
            return None
        raise ValueError(f"{name} must not be None")
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device (cuda/HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    return t.data_ptr()


def _stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


# ------------------------------------------------------------------ structs --
def motion_lib_struct(frames, local_rot, dof_vel, motion_len, motion_dt, num_frames, length_starts):
    F = frames.shape[0]
    M = motion_len.shape[0]
    return MotionLibC(
        _ptr(frames, torch.float32, (F, NUM_BODIES, BODY_STRIDE), "frames"),
        _ptr(local_rot, torch.float32, (F, NUM_BODIES, 4), "local_rot"),
        _ptr(dof_vel, torch.float32, (F, NUM_BODIES - 1, 3), "dof_vel"),
        _ptr(motion_len, torch.float32, (M,), "motion_len"),
        _ptr(motion_dt, torch.float32, (M,), "motion_dt"),
        _ptr(num_frames, torch.int64, (M,), "num_frames"),
        _ptr(length_starts, torch.int64, (M,), "length_starts"),
        M, F)


def step_params_struct(dt, reward, power_coef, use_power_reward, enable_early_termination, use_mean,
                       reset_body_ids, termination_distances, auto_reset=False, seed=0, reset_at_start=False):
    p = StepParamsC()
    p.auto_reset = int(bool(auto_reset))
    p.reset_at_start = int(bool(reset_at_start))
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.dt = float(dt)
    p.k_pos, p.k_rot, p.k_vel, p.k_ang_vel = reward.k_pos, reward.k_rot, reward.k_vel, reward.k_ang_vel
    p.w_pos, p.w_rot, p.w_vel, p.w_ang_vel = reward.w_pos, reward.w_rot, reward.w_vel, reward.w_ang_vel
    p.power_coef = float(power_coef)
    p.use_power_reward = int(bool(use_power_reward))
    p.enable_early_termination = int(bool(enable_early_termination))
    p.use_mean_termination = int(bool(use_mean))
    mask = 0
    for b in reset_body_ids:
        mask |= 1 << int(b)
    p.reset_body_mask = mask
    td = [float(x) for x in termination_distances]
    if len(td) != NUM_BODIES:
        raise ValueError("termination_distances must have 24 entries")
    for i, x in enumerate(td):
        p.termination_distance[i] = x
    return p


def env_struct(num_envs, rigid_body_state, root_state, dof_state, dof_force, progress, motion_ids, start_times,
               start_offset, global_offset, obs, rew, reward_raw, reset, terminate, terminals=None, truncations=None,
               masks=None, episode_return=None, episode_length=None, stats=None, rng_counter=None):
    N = num_envs
    u8 = torch.uint8
    return EnvBuffersC(
        N,
        _ptr(rigid_body_state, torch.float32, (N, NUM_BODIES, BODY_STRIDE), "rigid_body_state"),
        _ptr(root_state, torch.float32, (N, BODY_STRIDE), "root_state", nullable=True),
        _ptr(dof_state, torch.float32, (N, NUM_DOF, 2), "dof_state"),
        _ptr(dof_force, torch.float32, (N, NUM_DOF), "dof_force"),
        _ptr(progress, torch.int16, (N,), "progress"),
        _ptr(motion_ids, torch.int64, (N,), "motion_ids"),
        _ptr(start_times, torch.float32, (N,), "motion_start_times"),
        _ptr(start_offset, torch.float32, (N,), "motion_start_offset"),
        _ptr(global_offset, torch.float32, (N, 3), "global_offset"),
        _ptr(obs, torch.float32, (N, OBS_DIM), "obs"),
        _ptr(rew, torch.float32, (N,), "rew"),
        _ptr(reward_raw, torch.float32, (N, 5), "reward_raw"),
        _ptr(_as_u8(reset), u8, (N,), "reset"),
        _ptr(_as_u8(terminate), u8, (N,), "terminate"),
        _ptr(_as_u8(terminals), u8, (N,), "terminals", nullable=True),
        _ptr(_as_u8(truncations), u8, (N,), "truncations", nullable=True),
        _ptr(_as_u8(masks), u8, (N,), "masks", nullable=True),
        _ptr(episode_return, torch.float32, (N,), "episode_return", nullable=True),
        _ptr(episode_length, torch.int32, (N,), "episode_length", nullable=True),
        _ptr(stats, torch.float64, (lib().phc_stats_blocks(N), STATS_SLOTS), "stats", nullable=True),
        _ptr(rng_counter, torch.int32, (N,), "rng_counter", nullable=True),
    )


def _as_u8(t):
    """bool tensors are passed as their uint8 storage (same bytes, 0/1)."""
    if t is None:
        return None
    if t.dtype == torch.bool:
        return t.view(torch.uint8)
    return t


# ---------------------------------------------------------------------- ops --
def motion_state(mlib, motion_ids, motion_times, offset=None, want_dof=True):
    """R6+R7 (motion_lib.py:549-626).  Returns body [n,24,13], dof_pos/dof_vel [n,69]."""
    n = motion_ids.shape[0]
    dev = motion_ids.device
    body = torch.empty((n, NUM_BODIES, BODY_STRIDE), dtype=torch.float32, device=dev)
    dof_pos = torch.empty((n, NUM_DOF), dtype=torch.float32, device=dev) if want_dof else None
    dof_vel = torch.empty((n, NUM_DOF), dtype=torch.float32, device=dev) if want_dof else None
    out = RefStateC(body.data_ptr(), dof_pos.data_ptr() if want_dof else None,
                    dof_vel.data_ptr() if want_dof else None)
    rc = lib().phc_motion_state(ctypes.byref(mlib), _ptr(motion_ids, torch.int64, (n,), "motion_ids"),
                                _ptr(motion_times, torch.float32, (n,), "motion_times"),
                                _ptr(offset, torch.float32, (n, 3), "offset", nullable=True), n,
                                ctypes.byref(out), _stream())
    _check(rc, "phc_motion_state")
    return body, dof_pos, dof_vel


def env_step(env_c, mlib, params, timer=None):
    if timer is not None:
        _check(lib().phc_env_step_timed(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(params), timer.handle,
                                        _stream()), "phc_env_step_timed")
        return
    _check(lib().phc_env_step(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(params), _stream()),
           "phc_env_step")


class KernelTimer:
    """Per-launch kernel time stamped by the timed kernels themselves (phc_timer_*: workgroup starts
    and wave ends from the device's constant-rate clock): no event is recorded around the dispatch,
    and launches inside a captured hipGraph are timed too (a graph's slots hold its last replay)."""

    _serials = itertools.count(1)

    def __init__(self, capacity=4096, period=1):
        # never reused (unlike id() or the handle's address): the key of graphs whose launches stamp into it
        self.serial = next(KernelTimer._serials)
        self.handle = lib().phc_timer_create(int(capacity))
        if not self.handle:
            _check(-1, "phc_timer_create")
        if period > 1:  # time every period-th launch only (phc_timer_set_period)
            lib().phc_timer_set_period(self.handle, int(period))

    def reset(self):
        lib().phc_timer_reset(self.handle)

    @property
    def count(self):
        """Launches timed."""
        return lib().phc_timer_count(self.handle)

    @property
    def offered(self):
        """Launches offered to the timer (timed or skipped by the sampling period)."""
        return lib().phc_timer_offered(self.handle)

    def total_ms(self):
        ms = lib().phc_timer_total_ms(self.handle)
        if ms < 0:
            raise RuntimeError("phc_timer_total_ms failed")
        return ms

    @property
    def work(self):
        """Algorithmic work of the timed launches (phc_twin_gemm: FLOPs)."""
        return lib().phc_timer_work(self.handle)

    def durations_ms(self, cap=65536):
        """Per-launch ms of the counted launches, in the order they were taken (diagnostics)."""
        buf = (ctypes.c_double * cap)()
        n = lib().phc_timer_durations(self.handle, buf, cap)
        if n < 0:
            raise RuntimeError("phc_timer_durations failed")
        return list(buf[:min(n, cap)])

    def __del__(self):
        if getattr(self, "handle", None) and _lib is not None:
            _lib.phc_timer_destroy(self.handle)
            self.handle = None


_GEMM_TIMER = [None]


def gemm_set_timer(timer):
    """Offer the PPO update's trunk GEMM launches to `timer` (None: off); a launch captured into a
    graph keeps the timer it was captured with (its slot)."""
    lib().phc_gemm_set_timer(timer.handle if timer is not None else None)
    _GEMM_TIMER[0] = timer


def gemm_timer_id():
    """Identity of the timer set by gemm_set_timer (a captured graph's key: its launches carry
    that timer's slots, or none)."""
    return _GEMM_TIMER[0].serial if _GEMM_TIMER[0] is not None else None


def reset_envs(env_c, mlib, params, mask=None, phase=None, seed=0, counter=0, num_envs=None):
    n = env_c.num_envs
    _check(lib().phc_reset_envs(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(params),
                                _ptr(_as_u8(mask), torch.uint8, (n,), "mask", nullable=True),
                                _ptr(phase, torch.float32, (n,), "phase", nullable=True),
                                ctypes.c_uint64(seed), ctypes.c_uint64(counter), _stream()),
           "phc_reset_envs")


def amp_struct(amp_obs, amp_obs_demo):
    """phc_amp_buffers over [N, S, 196] float32 tensors (demo nullable)."""
    if amp_obs is None or amp_obs.dim() != 3 or amp_obs.shape[2] != AMP_OBS_STEP:
        raise ValueError("amp_obs: expected a [N, num_steps, 196] tensor")
    shape = tuple(amp_obs.shape)
    return AmpBuffersC(_ptr(amp_obs, torch.float32, shape, "amp_obs"),
                       _ptr(amp_obs_demo, torch.float32, shape, "amp_obs_demo", nullable=True), shape[1])


def amp_obs(env_c, mlib, amp_c, dt, mode=AMP_STEP):
    """R16: AMP history step (mode AMP_STEP) or re-initialisation of just-reset envs (AMP_INIT)."""
    _check(lib().phc_amp_obs(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(amp_c), float(dt), int(mode),
                             _stream()),
           "phc_amp_obs")


# ------------------------------------------------------- twin MLP epilogues --
DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
SPLIT, GROUPED = 0, 1
ACT_NONE, ACT_SILU = 0, 1


def _twin(t, dtype, layout, rows, groups, cols, name, nullable=False):
    shape = (rows, groups * cols) if layout == SPLIT else (groups, rows, cols)
    return _ptr(t, dtype, shape, name, nullable=nullable)


def bias_act_fwd(y, y_layout, bias, pre, out, out_layout, rows, groups, cols, act):
    """pre = y + bias, out = act(pre) over a twin tensor (phc_bias_act_fwd); out may be f16 / bf16
    from an f32 y."""
    dt = y.dtype
    ot = out.dtype if out is not None else dt
    if dt not in DTYPE_CODE or ot not in DTYPE_CODE:
        raise ValueError(f"bias_act_fwd: unsupported dtypes {dt} -> {ot}")
    _check(lib().phc_bias_act_fwd(_twin(y, dt, y_layout, rows, groups, cols, "y"), y_layout,
                                  _ptr(bias, torch.float32, (groups * cols,), "bias", nullable=True),
                                  _twin(pre, dt, y_layout, rows, groups, cols, "pre", nullable=True),
                                  _twin(out, ot, out_layout, rows, groups, cols, "out", nullable=True), out_layout,
                                  rows, groups, cols, act, DTYPE_CODE[dt], DTYPE_CODE[ot], _stream()),
           "phc_bias_act_fwd")


def ln_silu_fwd(y, gamma, beta, eps):
    """z = silu(LayerNorm(y)) per group of a GROUPED [G, M, N] tensor (phc_ln_silu_fwd)."""
    G, M, N_ = y.shape
    dt = y.dtype
    z = torch.empty((G, M, N_), dtype=torch.float32, device=y.device)
    mr = torch.empty((G * M, 2), dtype=torch.float32, device=y.device)
    _check(lib().phc_ln_silu_fwd(_ptr(y, dt, (G, M, N_), "y"), _ptr(gamma, torch.float32, (G * N_,), "gamma"),
                                 _ptr(beta, torch.float32, (G * N_,), "beta"), z.data_ptr(), mr.data_ptr(), M, G, N_,
                                 float(eps), DTYPE_CODE[dt], _stream()),
           "phc_ln_silu_fwd")
    return z, mr


def ln_silu_bwd(y, gamma, beta, mean_rstd, dz):
    G, M, N_ = y.shape
    dt = y.dtype
    dy = torch.empty_like(y)
    dg = torch.empty(G * N_, dtype=torch.float32, device=y.device)
    db = torch.empty(G * N_, dtype=torch.float32, device=y.device)
    ws = _workspace(lib().phc_ln_silu_workspace_bytes(M, G, N_), y.device)
    _check(lib().phc_ln_silu_bwd(_ptr(y, dt, (G, M, N_), "y"), _ptr(gamma, torch.float32, (G * N_,), "gamma"),
                                 _ptr(beta, torch.float32, (G * N_,), "beta"),
                                 _ptr(mean_rstd, torch.float32, (G * M, 2), "mean_rstd"),
                                 _ptr(dz, torch.float32, (G, M, N_), "dz"), dy.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                 M, G, N_, DTYPE_CODE[dt], ws.data_ptr(), _stream()),
           "phc_ln_silu_bwd")
    return dy, dg, db


def _operand(t, name):
    """(pointer, batch stride, leading dimension, batch, rows, cols) of a [rows, k] or
    [batch, rows, k] half-precision GEMM operand with unit column stride."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype not in (torch.float16, torch.bfloat16):
        raise ValueError(f"twin_gemm {name}: expected a f16 / bf16 device tensor")
    if t.dim() == 2:
        t3, bs = t[None], 0
    elif t.dim() == 3:
        t3, bs = t, t.stride(0)
    else:
        raise ValueError(f"twin_gemm {name}: expected 2-D or 3-D, got {tuple(t.shape)}")
    if t3.stride(2) != 1:
        raise ValueError(f"twin_gemm {name}: columns must be contiguous")
    return t3.data_ptr(), bs, t3.stride(1), t3.shape[0], t3.shape[1], t3.shape[2]


def twin_gemm_m_tiles(m, n, batch):
    """Rows of the bias-gradient partials a grad-epilogue launch of this shape leaves."""
    return int(lib().phc_twin_gemm_m_tiles(int(m), int(n), int(batch)))


# trunk-GEMM launches issued (phc_twin_gemm of more than 4,096 rows, phc_weight_grad, phc_weight_grad_group:
# the family phc_gemm_set_timer offers): a captured graph adds what it holds on every replay
# (clean_pufferl.core), so bench.py counts the launches of its timed region whatever replays them
GEMM_LAUNCHES = [0]


def twin_gemm(a, b, epilogue, out, twin, bias=None, aux=None, aux_layout=GROUPED, out_layout=GROUPED,
              bias_grad=None, max_workgroups=0, bias_partial=None, k_valid=0):
    """out = epilogue(a[b] @ b[b]^T) for a [batch?, m, k], b [batch?, n, k] (phc_twin_gemm).
    twin = (groups, cols) of the output / aux tensors' logical columns.  max_workgroups > 0:
    a persistent grid of that many workgroups looping over the tiles.  Grad epilogues: bias_grad
    [batch * n] receives the column sums; or bias_partial, fp32 [twin_gemm_m_tiles(m, n, batch),
    batch * n], the per-m-tile column sums for the caller to reduce (no second launch).  k_valid: the
    algorithmic depth when a's / b's last columns are zero padding (the kernel timer's FLOP count only)."""
    pa, abs_, lda, ba, m, k = _operand(a, "a")
    pb, bbs, ldb, bb, n, kb = _operand(b, "b")
    if kb != k or (ba != bb and ba != 1 and bb != 1):
        raise ValueError(f"twin_gemm: operand shapes {tuple(a.shape)} x {tuple(b.shape)}^T do not match")
    if m > 4096:
        GEMM_LAUNCHES[0] += 1
    if a.dtype != b.dtype:
        raise ValueError("twin_gemm: operands must share a dtype")
    batch = max(ba, bb)
    G, C = twin
    if out.dtype not in (torch.float32, a.dtype) or not out.is_contiguous() or out.numel() != m * batch * n:
        raise ValueError("twin_gemm: out must be contiguous f32 / operand-dtype with m * batch * n elements")
    if aux is not None and (aux.dtype not in (torch.float32, a.dtype) or not aux.is_contiguous()
                            or aux.numel() != out.numel()):
        raise ValueError("twin_gemm: aux must be a contiguous f32 / operand-dtype tensor shaped like out")
    d = GemmDescC(pa, pb, abs_, bbs, lda, ldb, m, n, k, batch, DTYPE_CODE[a.dtype], epilogue, DTYPE_CODE[out.dtype],
                  _ptr(bias, torch.float32, (batch * n,), "bias", nullable=True),
                  aux.data_ptr() if aux is not None else None, out.data_ptr(), aux_layout, out_layout, G, C,
                  DTYPE_CODE[aux.dtype] if aux is not None else 0, int(max_workgroups), int(k_valid))
    ws = None
    if bias_grad is not None:
        _ptr(bias_grad, torch.float32, (batch * n,), "bias_grad")
        ws = _workspace(lib().phc_twin_gemm_workspace_bytes(m, batch, n), a.device).data_ptr()
    elif bias_partial is not None:
        ws = _ptr(bias_partial, torch.float32, (twin_gemm_m_tiles(m, n, batch), batch * n), "bias_partial")
    _check(lib().phc_twin_gemm(ctypes.byref(d), bias_grad.data_ptr() if bias_grad is not None else None, ws,
                               _stream()),
           "phc_twin_gemm")
    return out


def weight_grad(g, z, splits, out=None):
    """Split-K partials of dW[b] = g[b]^T z[b] (phc_weight_grad): g [batch?, rows, m], z
    [batch?, rows, n] f16 / bf16 with contiguous columns (a 2-D operand is shared by the batch);
    returns fp32 [splits, batch, m, n] (sum over dim 0 = the gradient)."""
    GEMM_LAUNCHES[0] += 1
    pg, gbs, ldg, bg, rows, m = _operand(g, "g")
    pz, zbs, ldz, bz, rz, n = _operand(z, "z")
    if rz != rows or (bg != bz and bg != 1 and bz != 1) or g.dtype != z.dtype:
        raise ValueError(f"weight_grad: operands {tuple(g.shape)} / {tuple(z.shape)} do not match")
    batch = max(bg, bz)
    shape = (splits, batch, m, n)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=g.device)
    elif out.dtype != torch.float32 or not out.is_contiguous() or tuple(out.shape) != shape:
        raise ValueError(f"weight_grad: out must be a contiguous fp32 {shape} tensor")
    d = WgradDescC(pg, pz, gbs, zbs, ldg, ldz, rows, m, n, batch, DTYPE_CODE[g.dtype], splits, 0, out.data_ptr())
    _check(lib().phc_weight_grad(ctypes.byref(d), _stream()), "phc_weight_grad")
    return out


def weight_grad_group(problems, accumulate=True):
    """Weight gradients of up to 8 layers in one launch (phc_weight_grad_group): each problem is
    (g [batch?, rows, m], z [batch?, rows, n], dsts, split_row, n_valid) with dsts one or two dense
    fp32 [*, n_valid] destinations; output row r of batch b goes to dsts[b + (r >= split_row)]
    (split_row = m: no split).  dst (+)= g[b]^T z[b] over all rows."""
    GEMM_LAUNCHES[0] += 1
    if not 1 <= len(problems) <= WGRAD_GROUP_MAX:
        raise ValueError(f"weight_grad_group: 1..{WGRAD_GROUP_MAX} problems")
    arr = (WgradProblemC * len(problems))()
    rows = dtype = None
    for i, (g, z, dsts, split_row, n_valid) in enumerate(problems):
        pg, gbs, ldg, bg, r, m = _operand(g, "g")
        pz, zbs, ldz, bz, rz, n = _operand(z, "z")
        if rz != r or (bg != bz and bg != 1 and bz != 1) or g.dtype != z.dtype:
            raise ValueError(f"weight_grad_group: problem {i}: operands {tuple(g.shape)} / {tuple(z.shape)}")
        if rows is None:
            rows, dtype = r, g.dtype
        elif r != rows or g.dtype != dtype:
            raise ValueError("weight_grad_group: every problem must share rows and dtype")
        dsts = list(dsts)
        for d in dsts:
            if d.dtype != torch.float32 or not d.is_cuda or not d.is_contiguous() or d.shape[-1] != n_valid:
                raise ValueError(f"weight_grad_group: problem {i}: destinations must be dense fp32 [*, {n_valid}]")
        batch = max(bg, bz)
        need = batch + (1 if split_row < m else 0)
        if len(dsts) != need:
            raise ValueError(f"weight_grad_group: problem {i}: {need} destinations expected")
        rows_per = [split_row, m - split_row] if split_row < m else [m] * batch
        for d, rr in zip(dsts, rows_per):
            if d.numel() != rr * n_valid:
                raise ValueError(f"weight_grad_group: problem {i}: destination of {rr} x {n_valid} expected")
        ptrs = [d.data_ptr() for d in dsts] + [None] * (2 - len(dsts))
        arr[i] = WgradProblemC(pg, pz, gbs, zbs, ldg, ldz, (c_vp * 2)(*ptrs), n_valid, m, n, batch, split_row,
                               n_valid, 0)
    _check(lib().phc_weight_grad_group(arr, len(problems), rows, DTYPE_CODE[dtype], int(accumulate), _stream()),
           "phc_weight_grad_group")


def reduce_into(jobs, accumulate=True):
    """jobs: (src, dst) pairs; src [parts, rows, cols] (any row stride, unit column stride) or
    [rows, cols]; dst a dense fp32 tensor of rows * cols elements: dst (+)= src.sum(0) in one
    launch (phc_reduce_into).  The sources must stay alive until the launch has run (stream
    order: the caching allocator guarantees it for tensors freed after this call)."""
    for i in range(0, len(jobs), MAX_REDUCE_JOBS):
        chunk = jobs[i:i + MAX_REDUCE_JOBS]
        arr = (ReduceJobC * len(chunk))()
        for q, (src, dst) in enumerate(chunk):
            if src.dim() == 2:
                src = src[None]
            P, R, C = src.shape
            if src.dtype != torch.float32 or dst.dtype != torch.float32 or not src.is_cuda or not dst.is_cuda:
                raise ValueError("reduce_into: fp32 device tensors only")
            if src.stride(2) != 1 or not dst.is_contiguous() or dst.numel() != R * C:
                raise ValueError(f"reduce_into: job {q}: src {tuple(src.shape)} / dst {tuple(dst.shape)} mismatch")
            arr[q] = ReduceJobC(src.data_ptr(), dst.data_ptr(), R, C, src.stride(1) if R > 1 else C,
                                src.stride(0) if P > 1 else 0, P, int(accumulate))
        _check(lib().phc_reduce_into(arr, len(chunk), _stream()), "phc_reduce_into")


def _rows2d(t, name):
    if t.dim() == 1:
        t = t[None]
    if t.dim() != 2 or not t.is_cuda or (t.shape[1] > 1 and t.stride(1) != 1):
        raise ValueError(f"pack_weights: {name} must be a 1-D or 2-D device tensor with contiguous columns")
    return t, (t.stride(0) if t.shape[0] > 1 else t.shape[1])


class PackPlan:
    """A fixed list of operand-refresh jobs (phc_pack_weights): (src fp32 [rows, cols], dst
    [rows, cols] or None, dst_t [cols, rows] or None), f16 / bf16 / fp32 destinations.  The C
    argument arrays are built once; run() is one launch per 32 jobs."""

    def __init__(self, jobs):
        self._keep, self._arrs = [], []
        for i in range(0, len(jobs), MAX_PACK_JOBS):
            chunk = jobs[i:i + MAX_PACK_JOBS]
            arr = (PackJobC * len(chunk))()
            for q, (src, dst, dst_t) in enumerate(chunk):
                if src.dtype != torch.float32:
                    raise ValueError("pack_weights: fp32 sources only")
                s2, sld = _rows2d(src, "src")
                rows, cols = s2.shape
                dt = (dst if dst is not None else dst_t).dtype
                if dt not in DTYPE_CODE:
                    raise ValueError(f"pack_weights: unsupported destination dtype {dt}")
                d_ptr = dt_ptr = None
                dld = dtld = 0
                if dst is not None:
                    d2, dld = _rows2d(dst, "dst")
                    if tuple(d2.shape) != (rows, cols) or dst.dtype != dt:
                        raise ValueError(f"pack_weights: job {q}: dst {tuple(dst.shape)} vs src {tuple(src.shape)}")
                    d_ptr = d2.data_ptr()
                if dst_t is not None:
                    t2, dtld = _rows2d(dst_t, "dst_t")
                    if tuple(t2.shape) != (cols, rows) or dst_t.dtype != dt:
                        raise ValueError(f"pack_weights: job {q}: dst_t {tuple(dst_t.shape)} vs src {tuple(src.shape)}")
                    dt_ptr = t2.data_ptr()
                arr[q] = PackJobC(s2.data_ptr(), d_ptr, dt_ptr, rows, cols, sld, dld, dtld, DTYPE_CODE[dt], 0)
                self._keep += [src, dst, dst_t]
            self._arrs.append(arr)

    def run(self):
        for arr in self._arrs:
            _check(lib().phc_pack_weights(arr, len(arr), _stream()), "phc_pack_weights")


def obs_half(obs, mean, var, eps, clip, out, rows=None):
    """out [m, ld] (f16 / bf16) = RunningNorm(obs[rows]) rounded once, zero-padded (phc_obs_half)."""
    d = obs.shape[1]
    m, ld = out.shape
    _ptr(obs, torch.float32, None, "obs")
    if obs.dim() != 2:
        raise ValueError("obs_half: obs must be [rows, features]")
    if out.dtype not in (torch.float16, torch.bfloat16) or not out.is_cuda or not out.is_contiguous():
        raise ValueError("obs_half: out must be a contiguous f16 / bf16 device tensor")
    if rows is None and obs.shape[0] != m:
        raise ValueError(f"obs_half: {obs.shape[0]} obs rows for {m} output rows")
    _check(lib().phc_obs_half(obs.data_ptr(), _ptr(rows, torch.int64, (m,), "rows", nullable=True), m, d,
                              _ptr(mean.reshape(-1), torch.float32, (d,), "mean"),
                              _ptr(var.reshape(-1), torch.float32, (d,), "var"), float(eps), float(clip),
                              out.data_ptr(), ld, DTYPE_CODE[out.dtype], _stream()),
           "phc_obs_half")
    return out


def policy_act(trunk_out, ln_actor, ln_critic, eps, w_mu, b_mu, w_value, b_value, log_sigma, noise, actions, logprob, value,
               mu=None, std_max=float("inf"), w_mu_t=None):
    """Rollout tail after the trunks: LayerNorm+SiLU of both trunks (ln_* = (weight, bias)),
    mu / value heads, Normal sample and log-prob (phc_policy_act).  w_mu_t: optional [hidden, ld]
    transposed copy of w_mu (ld % 4 == 0, 16-B aligned): the mu head's weight reads coalesce."""
    G, M, H = trunk_out.shape
    A = w_mu.shape[0]
    wt_ptr, wt_ld = None, 0
    if w_mu_t is not None:
        if w_mu_t.dtype != torch.float32 or w_mu_t.dim() != 2 or w_mu_t.shape[0] != H or w_mu_t.stride(1) != 1 \
                or w_mu_t.stride(0) < A or w_mu_t.stride(0) % 4 or w_mu_t.data_ptr() % 16 or not w_mu_t.is_cuda:
            raise ValueError("policy_act: w_mu_t must be a 16-B aligned fp32 [hidden, ld >= actions, ld % 4 == 0] "
                             "device tensor")
        wt_ptr, wt_ld = w_mu_t.data_ptr(), w_mu_t.stride(0)
    if G != 2:
        raise ValueError("policy_act: trunk_out must be [2, rows, hidden]")
    args = PolicyActArgsC(_ptr(trunk_out, torch.float32, (2, M, H), "trunk_out"),
                          (c_vp * 2)(_ptr(ln_actor[0], torch.float32, (H,), "actor ln weight"),
                                     _ptr(ln_critic[0], torch.float32, (H,), "critic ln weight")),
                          (c_vp * 2)(_ptr(ln_actor[1], torch.float32, (H,), "actor ln bias"),
                                     _ptr(ln_critic[1], torch.float32, (H,), "critic ln bias")),
                          _ptr(w_mu, torch.float32, (A, H), "w_mu"), _ptr(b_mu, torch.float32, (A,), "b_mu"),
                          _ptr(w_value.reshape(-1), torch.float32, (H,), "w_value"),
                          _ptr(b_value.reshape(-1), torch.float32, (1,), "b_value"),
                          _ptr(log_sigma.reshape(-1), torch.float32, (A,), "log_sigma"),
                          _ptr(noise, torch.float32, (M, A), "noise"), _ptr(actions, torch.float32, (M, A), "actions"),
                          _ptr(logprob, torch.float32, (M,), "logprob"), _ptr(value, torch.float32, (M,), "value"),
                          _ptr(mu, torch.float32, (M, A), "mu", nullable=True), M, H, A, float(eps),
                          min(float(std_max), 3.0e38), wt_ptr, wt_ld, 0)
    _check(lib().phc_policy_act(ctypes.byref(args), _stream()), "phc_policy_act")


_WS = {}


def _workspace(nbytes, device):
    key = (device.index if device.index is not None else torch.cuda.current_device(), torch.cuda.current_stream())
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def act_bwd(grad_out, go_layout, pre, pre_layout, grad_pre, gp_layout, bias_grad, rows, groups, cols, act,
            pre_bias=None):
    """grad_pre = grad_out * act'(pre + pre_bias), bias_grad = column sums (phc_act_bwd); grad_pre
    may be f16 / bf16 from an f32 grad_out / pre."""
    dt = grad_out.dtype
    ot = grad_pre.dtype if grad_pre is not None else dt
    if dt not in DTYPE_CODE or ot not in DTYPE_CODE:
        raise ValueError(f"act_bwd: unsupported dtypes {dt} -> {ot}")
    ws = None
    if bias_grad is not None:
        ws = _workspace(lib().phc_act_bwd_workspace_bytes(rows, groups, cols), grad_out.device).data_ptr()
    _check(lib().phc_act_bwd(_twin(grad_out, dt, go_layout, rows, groups, cols, "grad_out"), go_layout,
                             _twin(pre, dt, pre_layout, rows, groups, cols, "pre", nullable=act == ACT_NONE),
                             pre_layout, _ptr(pre_bias, torch.float32, (groups * cols,), "pre_bias", nullable=True),
                             _twin(grad_pre, ot, gp_layout, rows, groups, cols, "grad_pre", nullable=True),
                             gp_layout, _ptr(bias_grad, torch.float32, (groups * cols,), "bias_grad", nullable=True),
                             rows, groups, cols, act, DTYPE_CODE[dt], DTYPE_CODE[ot], ws, _stream()),
           "phc_act_bwd")


# ------------------------------------------------------- AMP discriminator --
def _half2d(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype not in (torch.float16, torch.bfloat16) \
            or t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D f16 / bf16 device tensor with contiguous columns")
    return t


def disc_head_fwd(h, w, b, logits=None, reward=None):
    """logits = h . w + b and / or the adversarial reward -log(max(1 - sigmoid(logits), 1e-4)) for
    h [rows, width] f16 / bf16 (phc_disc_head_fwd)."""
    _half2d(h, "disc_head_fwd h")
    rows, width = h.shape
    _check(lib().phc_disc_head_fwd(h.data_ptr(), h.stride(0), rows, width, DTYPE_CODE[h.dtype],
                                   _ptr(w.reshape(-1), torch.float32, (width,), "w"),
                                   _ptr(b.reshape(-1), torch.float32, (1,), "b"),
                                   _ptr(logits, torch.float32, (rows,), "logits", nullable=True),
                                   _ptr(reward, torch.float32, (rows,), "reward", nullable=True), _stream()),
           "phc_disc_head_fwd")


def disc_head_bwd(h, w, grad_logits, grad_h):
    """grad_h = grad_logits * w * [h > 0] (operand dtype) and the per-block partial rows
    [blocks, 2 * width + 4] = (head weight grad | second layer bias grad | head bias grad | 0 0 0)
    (phc_disc_head_bwd); returns the partials."""
    _half2d(h, "disc_head_bwd h")
    _half2d(grad_h, "disc_head_bwd grad_h")
    rows, width = h.shape
    if tuple(grad_h.shape) != (rows, width) or grad_h.dtype != h.dtype:
        raise ValueError("disc_head_bwd: grad_h must match h")
    parts = torch.empty((lib().phc_disc_head_bwd_blocks(rows), 2 * width + 4), dtype=torch.float32, device=h.device)
    _check(lib().phc_disc_head_bwd(h.data_ptr(), h.stride(0), rows, width, DTYPE_CODE[h.dtype],
                                   _ptr(w.reshape(-1), torch.float32, (width,), "w"),
                                   _ptr(grad_logits, torch.float32, (rows,), "grad_logits"), grad_h.data_ptr(),
                                   grad_h.stride(0), parts.data_ptr(), _stream()),
           "phc_disc_head_bwd")
    return parts


# ------------------------------------------------------------ PPO objective --
def ppo_coefs(clip_coef, vf_clip_coef, vf_coef, ent_coef, bound_coef, soft_bound, clip_vloss):
    return PpoCoefsC(float(clip_coef), float(vf_clip_coef), float(vf_coef), float(ent_coef), float(bound_coef),
                     float(soft_bound), int(bool(clip_vloss)), 0)


def ppo_loss_fwd(mu, log_sigma, actions, old_logprob, adv, adv_mean_std, value, old_value, returns, coefs,
                 stats_acc=None):
    """(stats [1 + PPO_STATS], row_coef [m, 2]) of phc_ppo_loss_fwd; stats_acc (float64 [PPO_STATS],
    optional) += stats[1:] in the same launch."""
    m, a = mu.shape
    dev = mu.device
    stats = torch.empty(1 + PPO_STATS, dtype=torch.float32, device=dev)
    row_coef = torch.empty((m, 2), dtype=torch.float32, device=dev)
    ws = _workspace(lib().phc_ppo_workspace_bytes(m), dev)
    f32 = torch.float32
    _check(lib().phc_ppo_loss_fwd(_ptr(mu, f32, (m, a), "mu"), _ptr(log_sigma, f32, (a,), "log_sigma"),
                                  _ptr(actions, f32, (m, a), "actions"), _ptr(old_logprob, f32, (m,), "old_logprob"),
                                  _ptr(adv, f32, (m,), "adv"), _ptr(adv_mean_std, f32, (2,), "adv_mean_std"),
                                  _ptr(value, f32, (m,), "value"), _ptr(old_value, f32, (m,), "old_value"),
                                  _ptr(returns, f32, (m,), "returns"), m, a, ctypes.byref(coefs),
                                  row_coef.data_ptr(), stats.data_ptr(),
                                  _ptr(stats_acc, torch.float64, (PPO_STATS,), "stats_acc", nullable=True),
                                  ws.data_ptr(), _stream()),
           "phc_ppo_loss_fwd")
    return stats, row_coef


def ppo_loss_bwd(mu, log_sigma, actions, row_coef, grad_loss, coefs):
    m, a = mu.shape
    f32 = torch.float32
    gmu = torch.empty_like(mu)
    gv = torch.empty(m, dtype=f32, device=mu.device)
    _check(lib().phc_ppo_loss_bwd(_ptr(mu, f32, (m, a), "mu"), _ptr(log_sigma, f32, (a,), "log_sigma"),
                                  _ptr(actions, f32, (m, a), "actions"), _ptr(row_coef, f32, (m, 2), "row_coef"),
                                  _ptr(grad_loss, f32, (), "grad_loss"), m, a, ctypes.byref(coefs),
                                  gmu.data_ptr(), gv.data_ptr(), _stream()),
           "phc_ppo_loss_bwd")
    return gmu, gv


# ------------------------------------------------------ fused PPO tail --
TAIL_HIDDEN = 512
TAIL_MAX_ACTIONS = 72
TAIL_FIELDS = ("b_mu", "w_value", "b_value", "gamma", "beta", "b6", "stride")


def tail_layout(num_actions, hidden=TAIL_HIDDEN):
    """Column offsets of one block's partial row of phc_tail_ln_bwd (dict over TAIL_FIELDS)."""
    off = (ctypes.c_int32 * 7)()
    _check(lib().phc_tail_layout(num_actions, hidden, off), "phc_tail_layout")
    return dict(zip(TAIL_FIELDS, list(off)))


class TailLN:
    """phc_tail_ln_fwd / _bwd for one minibatch: LayerNorm + SiLU of both trunks of y [2, M, 512]
    fp32 with the critic's value head; h_actor and value are allocated here."""

    def __init__(self, y, ln_a, ln_c, eps, w_v, b_v):
        G, M, H = y.shape
        if G != 2 or H != TAIL_HIDDEN:
            raise ValueError(f"tail_ln: y must be [2, rows, {TAIL_HIDDEN}]")
        f32, dev = torch.float32, y.device
        self.M, self.H = M, H
        self.h_actor = torch.empty((M, H), dtype=f32, device=dev)
        self.value = torch.empty(M, dtype=f32, device=dev)
        self.keep = (y, ln_a, ln_c, w_v, b_v)  # the pointers below stay valid while this object lives
        self.args = TailLnArgsC(
            _ptr(y, f32, (2, M, H), "trunk_out"),
            (c_vp * 2)(_ptr(ln_a[0], f32, (H,), "actor ln weight"), _ptr(ln_c[0], f32, (H,), "critic ln weight")),
            (c_vp * 2)(_ptr(ln_a[1], f32, (H,), "actor ln bias"), _ptr(ln_c[1], f32, (H,), "critic ln bias")),
            _ptr(w_v.reshape(-1), f32, (H,), "w_value"), _ptr(b_v.reshape(-1), f32, (1,), "b_value"),
            self.h_actor.data_ptr(), self.value.data_ptr(), M, H, float(eps))

    def forward(self):
        _check(lib().phc_tail_ln_fwd(ctypes.byref(self.args), _stream()), "phc_tail_ln_fwd")
        return self.h_actor, self.value

    def backward(self, dh_actor, dmu, dvalue, dtype):
        """(dy [2, M, H] in dtype, partial [blocks, stride] fp32, layout)."""
        M, H = self.M, self.H
        A = dmu.shape[1]
        f32, dev = torch.float32, self.value.device
        lay = tail_layout(A, H)
        part = torch.empty((int(lib().phc_tail_blocks(M)), lay["stride"]), dtype=f32, device=dev)
        dy = torch.empty((2, M, H), dtype=dtype, device=dev)
        _check(lib().phc_tail_ln_bwd(ctypes.byref(self.args), _ptr(dh_actor, f32, (M, H), "dh_actor"),
                                     _ptr(dmu, f32, (M, A), "dmu"), _ptr(dvalue.reshape(-1), f32, (M,), "dvalue"),
                                     A, dy.data_ptr(), DTYPE_CODE[dtype], part.data_ptr(), _stream()),
               "phc_tail_ln_bwd")
        return dy, part, lay


# ------------------------------------------------------------- mu head --
MU_HEAD_MAX_ACTIONS = 80


def mu_head_fwd(h, w, b, out=None):
    """mu [M, A] = h [M, H] @ w [A, H]^T + b in fp32 (phc_mu_head_fwd, fp32-input MFMA)."""
    M, H = h.shape
    A = w.shape[0]
    f32 = torch.float32
    if out is None:
        out = torch.empty((M, A), dtype=f32, device=h.device)
    _check(lib().phc_mu_head_fwd(_ptr(h, f32, (M, H), "h"), _ptr(w, f32, (A, H), "w"),
                                 _ptr(b.reshape(-1), f32, (A,), "b"), _ptr(out, f32, (M, A), "mu"), M, H, A,
                                 _stream()), "phc_mu_head_fwd")
    return out


def mu_head_dgrad(dmu, w, out=None):
    """dh [M, H] = dmu [M, A] @ w [A, H] in fp32 (phc_mu_head_dgrad)."""
    M, A = dmu.shape
    H = w.shape[1]
    f32 = torch.float32
    if out is None:
        out = torch.empty((M, H), dtype=f32, device=dmu.device)
    _check(lib().phc_mu_head_dgrad(_ptr(dmu, f32, (M, A), "dmu"), _ptr(w, f32, (A, H), "w"),
                                   _ptr(out, f32, (M, H), "dh"), M, H, A, _stream()), "phc_mu_head_dgrad")
    return out


def mu_head_wgrad_parts(dmu, h, splits=128):
    """[splits, A, H] fp32 partials of dmu^T @ h over row chunks (phc_mu_head_wgrad); their sum
    over dim 0 is the weight gradient (phc_reduce_into sums them straight into .grad)."""
    M, A = dmu.shape
    H = h.shape[1]
    f32 = torch.float32
    splits = max(1, min(int(splits), M))
    part = torch.empty((splits, A, H), dtype=f32, device=dmu.device)
    _check(lib().phc_mu_head_wgrad(_ptr(dmu, f32, (M, A), "dmu"), _ptr(h, f32, (M, H), "h"), part.data_ptr(), M, H,
                                   A, splits, _stream()), "phc_mu_head_wgrad")
    return part


# ------------------------------------------------------- experience store --
class RowCompactor:
    """Experience.store on the device (phc_compact_rows): a fixed list of (src [n, ...],
    dst [capacity, ...]) tensor pairs, a device cursor and {n_valid, taken} counts.  The C
    argument array is built once, so repeated calls (or a captured graph) reuse it."""

    def __init__(self, pairs, n, capacity, device):
        if not 1 <= len(pairs) <= MAX_ROW_FIELDS:
            raise ValueError(f"RowCompactor: 1..{MAX_ROW_FIELDS} fields")
        self.n, self.capacity = n, capacity
        # [cursor, n_valid, taken, sum n_valid, sum taken] in ONE buffer: the rollout reads the cursor
        # and the running sums back in one copy (state())
        self._buf = torch.zeros(5, dtype=torch.int64, device=device)
        self.cursor = self._buf[0:1]
        # {n_valid, taken} of the last call, then their running sums since reset()
        self.counts = self._buf[1:5]
        self.workspace = torch.empty(lib().phc_compact_workspace_bytes(n), dtype=torch.uint8, device=device)
        self._keep = []
        arr = (RowFieldC * len(pairs))()
        for k, (src, dst) in enumerate(pairs):
            if src.shape[0] != n or dst.shape[0] != capacity or src.shape[1:] != dst.shape[1:]:
                raise ValueError(f"RowCompactor field {k}: src {tuple(src.shape)} vs dst {tuple(dst.shape)}")
            elems = int(np.prod(src.shape[1:])) if src.dim() > 1 else 1
            if src.dtype in (torch.bool, torch.uint8) and dst.dtype == torch.float32:
                kind = ROW_U8_TO_F32
                src = _as_u8(src)
            elif src.dtype == dst.dtype and src.element_size() == 4:
                kind = ROW_COPY32
            elif src.dtype == dst.dtype and src.element_size() == 8:
                kind = ROW_COPY64
            else:
                raise ValueError(f"RowCompactor field {k}: unsupported {src.dtype} -> {dst.dtype}")
            _ptr(src, src.dtype, None, f"src{k}")
            _ptr(dst, dst.dtype, None, f"dst{k}")
            flags = ROW_SRC_WORDS if kind == ROW_U8_TO_F32 and _words_inside_storage(src) else 0
            arr[k] = RowFieldC(src.data_ptr(), dst.data_ptr(), elems, kind, flags)
            self._keep += [src, dst]
        self._arr, self._nf = arr, len(pairs)

    def __call__(self, mask=None):
        _check(lib().phc_compact_rows(self._arr, self._nf,
                                      _ptr(_as_u8(mask), torch.uint8, (self.n,), "mask", nullable=True), self.n,
                                      self.cursor.data_ptr(), self.capacity, self.counts.data_ptr(),
                                      self.workspace.data_ptr(), _stream()),
               "phc_compact_rows")

    def reset(self, ptr=0):
        self._buf.zero_()
        if ptr:
            self.cursor.fill_(ptr)

    def state(self):
        """(cursor, sum of n_valid, sum of taken) since reset(), in one device -> host read."""
        c, _, _, nv, tk = self._buf.tolist()
        return c, nv, tk

    def snapshot(self):
        """Queue state()'s copy into pinned host memory on the current stream, without waiting: work
        queued after it may keep running while snapshot_read() waits for this copy only."""
        if getattr(self, "_pinned", None) is None:
            self._pinned = torch.empty(5, dtype=torch.int64, pin_memory=True)
            self._pinned_done = torch.cuda.Event()
        self._pinned.copy_(self._buf, non_blocking=True)
        self._pinned_done.record()

    def snapshot_read(self):
        """The (cursor, sum of n_valid, sum of taken) of the last snapshot()."""
        self._pinned_done.synchronize()
        c, _, _, nv, tk = self._pinned.tolist()
        return c, nv, tk


def physics_replay(env_c, mlib, params, pos_sigma, force_scale, seed, counter):
    _check(lib().phc_physics_replay(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(params),
                                    float(pos_sigma), float(force_scale), ctypes.c_uint64(seed),
                                    ctypes.c_uint64(counter), _stream()),
           "phc_physics_replay")


BODY_MODEL_STRIDE = 80


def physics_env_struct(rigid_body_state, dof_state, dof_force, root_state=None):
    """An env struct carrying only the buffers phc_physics_step touches (standalone use / tests)."""
    n = rigid_body_state.shape[0]
    e = EnvBuffersC()
    e.num_envs = n
    e.rigid_body_state = _ptr(rigid_body_state, torch.float32, (n, NUM_BODIES, BODY_STRIDE), "rigid_body_state")
    e.root_state = _ptr(root_state, torch.float32, (n, BODY_STRIDE), "root_state", nullable=True)
    e.dof_state = _ptr(dof_state, torch.float32, (n, NUM_DOF, 2), "dof_state")
    e.dof_force = _ptr(dof_force, torch.float32, (n, NUM_DOF), "dof_force")
    return e


def physics_step(env_c, pd_target, body_model, params, timer=None):
    """N3 articulated-body step (phc_physics_step) over the env buffers of env_c; with `timer`
    (a KernelTimer) the launch's own start/stop events are recorded."""
    n = int(env_c.num_envs)
    args = (ctypes.byref(env_c), _ptr(pd_target, torch.float32, (n, NUM_DOF), "pd_target"),
            _ptr(body_model, torch.float32, (NUM_BODIES, BODY_MODEL_STRIDE), "body_model"), ctypes.byref(params))
    if timer is not None:
        _check(lib().phc_physics_step_timed(*args, timer.handle, _stream()), "phc_physics_step")
    else:
        _check(lib().phc_physics_step(*args, _stream()), "phc_physics_step")


def pd_map(actions, pd_out, offset, scale, frozen, clip=True):
    """phc_pd_map of R13 (the action -> PD-target map folded into its consumer kernel); clip =
    EnvConfig.clip_actions (clean_pufferl/env.py:91)."""
    n = actions.shape[0]
    return PdMapC(_ptr(actions, torch.float32, (n, NUM_DOF), "actions"),
                  _ptr(pd_out, torch.float32, (n, NUM_DOF), "pd_target"),
                  _ptr(offset, torch.float32, (NUM_DOF,), "offset"), _ptr(scale, torch.float32, (NUM_DOF,), "scale"),
                  _ptr(_as_u8(frozen), torch.uint8, (NUM_DOF,), "frozen", nullable=True), int(bool(clip)))


def env_step_replay(env_c, mlib, params, pos_sigma, force_scale, seed, counter, pd=None, timer=None):
    """phc_env_step_replay: R13 + the physics stand-in + the fused env step in one launch."""
    rp = ReplayParamsC(float(pos_sigma), float(force_scale), int(seed) & 0xFFFFFFFFFFFFFFFF,
                       int(counter) & 0xFFFFFFFFFFFFFFFF)
    if pd is not None and pd.actions and int(env_c.num_envs) <= 0:
        raise ValueError("env_step_replay: empty env")
    _check(lib().phc_env_step_replay(ctypes.byref(env_c), ctypes.byref(mlib), ctypes.byref(params), ctypes.byref(rp),
                                     ctypes.byref(pd) if pd is not None else None,
                                     timer.handle if timer is not None else None, _stream()),
           "phc_env_step_replay")


def physics_step_actions(env_c, pd, body_model, params, timer=None):
    """N3 step with the PD targets computed in-kernel from the actions (phc_physics_step_actions)."""
    _ptr(body_model, torch.float32, (NUM_BODIES, BODY_MODEL_STRIDE), "body_model")
    _check(lib().phc_physics_step_actions(ctypes.byref(env_c), ctypes.byref(pd), body_model.data_ptr(),
                                          ctypes.byref(params), timer.handle if timer is not None else None, _stream()),
           "phc_physics_step_actions")


def actions_to_pd(actions, pd_out, offset, scale, frozen, clip=True):
    n = actions.shape[0]
    _check(lib().phc_actions_to_pd(_ptr(actions, torch.float32, (n, NUM_DOF), "actions"),
                                   _ptr(pd_out, torch.float32, (n, NUM_DOF), "pd_target"), n,
                                   _ptr(offset, torch.float32, (NUM_DOF,), "offset"),
                                   _ptr(scale, torch.float32, (NUM_DOF,), "scale"),
                                   _ptr(_as_u8(frozen), torch.uint8, (NUM_DOF,), "frozen", nullable=True),
                                   int(bool(clip)), _stream()),
           "phc_actions_to_pd")


def fk_motions(quat_global, root_trans, starts, counts, fps, parents, local_translation, gauss_weights):
    """R3-R5: returns (frames [F,24,13], local_rot [F,24,4], dof_vel [F,23,3])."""
    F = quat_global.shape[0]
    M = starts.shape[0]
    dev = quat_global.device
    frames = torch.empty((F, NUM_BODIES, BODY_STRIDE), dtype=torch.float32, device=dev)
    lrs = torch.empty((F, NUM_BODIES, 4), dtype=torch.float32, device=dev)
    dvs = torch.empty((F, NUM_BODIES - 1, 3), dtype=torch.float32, device=dev)
    ws = torch.empty(int(lib().phc_fk_workspace_bytes(F)), dtype=torch.uint8, device=dev)
    radius = (gauss_weights.shape[0] - 1) // 2
    rc = lib().phc_fk_motions(
        _ptr(quat_global, torch.float64, (F, NUM_BODIES, 4), "quat_global"),
        _ptr(root_trans, torch.float64, (F, 3), "root_trans"),
        _ptr(starts, torch.int64, (M,), "starts"), _ptr(counts, torch.int64, (M,), "counts"),
        _ptr(fps, torch.float32, (M,), "fps"), M, F,
        _ptr(parents, torch.int64, (NUM_BODIES,), "parents"),
        _ptr(local_translation, torch.float32, (NUM_BODIES, 3), "local_translation"),
        _ptr(gauss_weights, torch.float64, None, "gauss_weights"), radius,
        frames.data_ptr(), lrs.data_ptr(), dvs.data_ptr(), ws.data_ptr(), _stream())
    _check(rc, "phc_fk_motions")
    return frames, lrs, dvs


class GAE:
    """compute_gae (c_gae.pyx:11-32) on device with a cached workspace."""

    def __init__(self):
        self._ws = None

    def __call__(self, dones, values, rewards, gamma, lam, out=None):
        n = rewards.shape[0]
        need = int(lib().phc_gae_workspace_bytes(n))
        if self._ws is None or self._ws.numel() < need or self._ws.device != rewards.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=rewards.device)
        if out is None:
            out = torch.empty_like(rewards)
        rc = lib().phc_gae(_ptr(dones, torch.float32, (n,), "dones"), _ptr(values, torch.float32, (n,), "values"),
                           _ptr(rewards, torch.float32, (n,), "rewards"), n, float(gamma), float(lam),
                           _ptr(out, torch.float32, (n,), "advantages"), self._ws.data_ptr(), _stream())
        _check(rc, "phc_gae")
        return out


_gae = GAE()


def compute_gae(dones, values, rewards, gamma, lam, out=None):
    return _gae(dones, values, rewards, gamma, lam, out)


def rms_update(x, mean, var, count, workspace=None):
    rows, cols = x.shape
    need = int(lib().phc_rms_workspace_bytes(rows, cols))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    rc = lib().phc_rms_update(_ptr(x, torch.float32, (rows, cols), "x"), rows, cols,
                              _ptr(mean, torch.float32, None, "running_mean"),
                              _ptr(var, torch.float32, None, "running_var"),
                              _ptr(count, torch.float32, (1,), "count"), workspace.data_ptr(), _stream())
    _check(rc, "phc_rms_update")
    return workspace


def rms_moments(x, workspace=None):
    """This rank's batch moments [cols, 2] float64 = (mean, M2) of x [rows, cols] (phc_rms_moments)."""
    rows, cols = x.shape
    need = int(lib().phc_rms_workspace_bytes(rows, cols))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    mom = torch.empty((cols, 2), dtype=torch.float64, device=x.device)
    _check(lib().phc_rms_moments(_ptr(x, torch.float32, (rows, cols), "x"), rows, cols, mom.data_ptr(),
                                 workspace.data_ptr(), _stream()), "phc_rms_moments")
    return mom, workspace


def rms_apply(moments, part_rows, mean, var, count):
    """Merge every rank's moments [parts, cols, 2] (rows per part: part_rows [parts] float64) in
    part order and apply the running update (phc_rms_apply)."""
    parts, cols, _ = moments.shape
    _check(lib().phc_rms_apply(_ptr(moments, torch.float64, (parts, cols, 2), "moments"),
                               _ptr(part_rows, torch.float64, (parts,), "part_rows"), parts, cols,
                               _ptr(mean, torch.float32, None, "running_mean"),
                               _ptr(var, torch.float32, None, "running_var"),
                               _ptr(count, torch.float32, (1,), "count"), _stream()), "phc_rms_apply")


def rms_normalize(x, mean, var, eps=1e-5, clip=10.0, out=None):
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    rc = lib().phc_rms_normalize(_ptr(x, torch.float32, (rows, cols), "x"),
                                 _ptr(out, torch.float32, (rows, cols), "out"), rows, cols,
                                 _ptr(mean, torch.float32, None, "running_mean"),
                                 _ptr(var, torch.float32, None, "running_var"), float(eps), float(clip), _stream())
    _check(rc, "phc_rms_normalize")
    return out
