/*
 * phc.h — C ABI of libphc_hip.so, the MI355X-native hot path of the PHC imitation
 * rollout + PPO step (howird/puffer-phc).
 *
 * Conventions:
 *   - every pointer is a device pointer owned by the caller (PyTorch caching allocator);
 *     the library never allocates on the hot path and never frees;
 *   - every call is stream-ordered on `stream` (a hipStream_t passed as void*), returns 0
 *     or a negative PHC_E* code and never throws; phc_last_error() gives a thread-local
 *     message for the last failing call;
 *   - tensors are dense, C-contiguous float32 unless stated; quaternions are xyzw;
 *   - rigid-body records are 13 floats: pos(3) rot(4) vel(3) ang_vel(3) (the Isaac Gym
 *     rigid-body state layout, puffer_phc/envs/humanoid_phc.py:542-549).
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef PHC_H_
#define PHC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PHC_NUM_BODIES 24
#define PHC_NUM_DOF 69
#define PHC_BODY_STRIDE 13
#define PHC_SELF_OBS 358
#define PHC_TASK_OBS 576
#define PHC_OBS_DIM 934
#define PHC_AMP_OBS_STEP 196
#define PHC_STATS_SLOTS 16

enum {
  PHC_OK = 0,
  PHC_EINVAL = -1,  /* bad argument (null pointer, size, alignment) */
  PHC_ELAUNCH = -2, /* kernel launch failed */
};

/* Packed motion library (MotionLibBase.load_motions packing, puffer_phc/motion_lib.py:396-419).
 * frames[f, b, :] = gts(3) grs(4) gvs(3) gavs(3); one 1248-byte record per frame. */
typedef struct phc_motion_lib {
  const float *frames;          /* [F, 24, 13] */
  const float *local_rot;       /* [F, 24, 4]  lrs */
  const float *dof_vel;         /* [F, 23, 3]  dvs */
  const float *motion_len;      /* [M] seconds, (nf-1)/fps */
  const float *motion_dt;       /* [M] 1/fps */
  const int64_t *num_frames;    /* [M] */
  const int64_t *length_starts; /* [M] exclusive cumsum of num_frames */
  int64_t num_motions;
  int64_t num_frames_total;
} phc_motion_lib;

/* Reference-state output of phc_motion_state (get_motion_state's dict, motion_lib.py:612-626). */
typedef struct phc_ref_state {
  float *body;    /* [n, 24, 13] rg_pos, rb_rot, body_vel, body_ang_vel */
  float *dof_pos; /* [n, 69] (nullable) */
  float *dof_vel; /* [n, 69] (nullable) */
} phc_ref_state;

/* Per-env device buffers of HumanoidPHC + PHCPufferEnv (humanoid_phc.py:498-618,
 * clean_pufferl/env.py:41-60). */
typedef struct phc_env_buffers {
  int64_t num_envs;
  float *rigid_body_state;    /* [N, 24, 13] sim rigid bodies (read by step, written by reset) */
  float *root_state;          /* [N, 13] actor root state (written by reset; nullable) */
  float *dof_state;           /* [N, 69, 2] (pos, vel) */
  const float *dof_force;     /* [N, 69] */
  int16_t *progress;          /* [N] progress_buf */
  int64_t *motion_ids;        /* [N] _sampled_motion_ids */
  float *motion_start_times;  /* [N] */
  float *motion_start_offset; /* [N] _motion_start_times_offset */
  float *global_offset;       /* [N, 3] */
  float *obs;                 /* [N, 934] obs_buf */
  float *rew;                 /* [N] rew_buf */
  float *reward_raw;          /* [N, 5] pos, rot, vel, ang_vel, power */
  uint8_t *reset;             /* [N] reset_buf (bool) */
  uint8_t *terminate;         /* [N] _terminate_buf (bool) */
  uint8_t *terminals;         /* [N] PHCPufferEnv.terminals */
  uint8_t *truncations;       /* [N] PHCPufferEnv.truncations */
  uint8_t *masks;             /* [N] PHCPufferEnv.masks */
  float *episode_return;      /* [N] */
  int32_t *episode_length;    /* [N] */
  double *stats;              /* [phc_stats_blocks(N), PHC_STATS_SLOTS] per-block log sums */
  uint32_t *rng_counter;      /* [N] per-env counter of the counter-based RNG (nullable) */
  /* optional (R17 fused into the step): the policy's first trunk-GEMM operand of every obs row the
   * step writes — RunningNorm(obs) (policies/running_norm.py:15-20) rounded once to f16 / bf16,
   * [N, obs_operand_ld] zero-padded past 934 — the values phc_obs_half writes, bit for bit.
   * Written by phc_env_step / phc_env_step_replay when obs_operand is set (reset kernels do not). */
  void *obs_operand;
  const float *obs_norm_mean; /* [934] running_mean */
  const float *obs_norm_var;  /* [934] running_var */
  float obs_norm_eps, obs_norm_clip;
  int32_t obs_operand_ld;     /* % 8 == 0, >= 934; obs_operand 16-byte aligned */
  int32_t obs_operand_dtype;  /* PHC_DT_F16 or PHC_DT_BF16 */
} phc_env_buffers;

/* Step constants: RewardConfig (config.py:23-36), EnvConfig power coef / early termination
 * (config.py:79-101), termination distances and reset bodies (humanoid_phc.py:235-253). */
typedef struct phc_step_params {
  float dt; /* control dt as float32 (2/60) */
  float k_pos, k_rot, k_vel, k_ang_vel;
  float w_pos, w_rot, w_vel, w_ang_vel;
  float power_coef;     /* 0.0005 */
  int32_t use_power_reward;
  int32_t enable_early_termination;
  int32_t use_mean_termination;  /* eval mode: mean body distance vs termination_distance[first] */
  uint32_t reset_body_mask;      /* bit b set = body b counts for termination */
  float termination_distance[PHC_NUM_BODIES];
  int32_t auto_reset;            /* phc_env_step also re-initialises envs that reset (R15 fused) */
  int32_t reset_at_start;        /* reset to motion time 0 (StateInit.Start / eval flag_test,
                                    humanoid_phc.py:843-855) instead of a sampled time */
  uint64_t seed;                 /* RNG seed of the reset time draw (with env->rng_counter) */
} phc_step_params;

/* Number of per-block statistics rows phc_env_step writes for `num_envs` envs. */
int64_t phc_stats_blocks(int64_t num_envs);

/* R6+R7: MotionLibBase.get_motion_state (puffer_phc/motion_lib.py:549-626).  offset nullable. */
int phc_motion_state(const phc_motion_lib *lib, const int64_t *motion_ids, const float *motion_times,
                     const float *offset, int64_t n, phc_ref_state *out, void *stream);

/* R6,R7,R9-R12,R14 fused: HumanoidPHC.step post-physics (humanoid_phc.py:136-146 ->
 * _compute_reward :1228-1303, _compute_reset :1311-1333, _compute_observations :935-959)
 * plus PHCPufferEnv.step bookkeeping (clean_pufferl/env.py:103-140).  Increments progress.
 * With p->auto_reset, envs whose reset flag comes up are re-initialised in the same launch
 * exactly as phc_reset_envs would (PHCPufferEnv.step's env.reset(reset_indices), :114-116):
 * their obs row is the post-reset observation and reset/terminate read back as 0, while
 * terminals/truncations/masks/episode stats keep this step's outcome. */
int phc_env_step(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                 void *stream);

/* Kernel timer for measurement (bench.py): a timed launch stamps its own start (per workgroup) and
 * end (per wave, after its memory operations complete) from the device's constant-rate clock into a
 * slot of the timer's device buffer, so the span is the kernel's own execution as rocprofv3 reports
 * it, no event is recorded around the dispatch (the stream sees no idle time), and launches captured
 * into a hipGraph are timed too (their slots hold the LAST replay).  Up to `capacity` timed launches.
 * phc_timer_reset starts a new measurement: launches stamped before it no longer count, except slots
 * inside a captured graph that a later replay re-stamps.  count / work / total_ms wait for the device
 * and report the counted launches (total_ms negative on error). */
typedef struct phc_kernel_timer phc_kernel_timer;
phc_kernel_timer *phc_timer_create(int32_t capacity);
void phc_timer_destroy(phc_kernel_timer *timer);
void phc_timer_reset(phc_kernel_timer *timer);
int32_t phc_timer_count(phc_kernel_timer *timer);
/* Sample: time only every period-th launch offered to the timer (1 = every launch, the default).
 * A timed launch costs its workgroups one store and its waves one wait + atomic at the end;
 * phc_timer_offered counts every launch offered. */
void phc_timer_set_period(phc_kernel_timer *timer, int32_t period);
int64_t phc_timer_offered(const phc_kernel_timer *timer);
double phc_timer_total_ms(phc_kernel_timer *timer);
double phc_timer_work(phc_kernel_timer *timer); /* algorithmic work of the counted launches (GEMM: FLOPs) */
/* per-launch ms of the counted launches in the order they were taken (up to cap; diagnostics);
 * returns the number counted, negative on error */
int32_t phc_timer_durations(phc_kernel_timer *timer, double *out, int32_t cap);
/* the PPO update's trunk GEMMs (phc_twin_gemm launches of more than 4,096 rows, phc_weight_grad,
 * phc_weight_grad_group) are offered to `timer` (NULL: off) with their 2 m n k batch FLOPs; a
 * measurement aid for bench.py's GEMM roofline. */
void phc_gemm_set_timer(phc_kernel_timer *timer);
int phc_env_step_timed(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                       phc_kernel_timer *timer, void *stream);

/* R15: HumanoidPHC.reset(env_ids) with StateInit.Random (humanoid_phc.py:90-103, 663-778,
 * 843-929 + motion_lib.py:526-535) for every env whose flag in `env_mask` is set (env_mask
 * nullable = use env->reset).  `phase` [N] holds the uniform draws (nullable = counter-based
 * in-kernel RNG keyed by seed/counter).  Rewrites sim state, progress, start times, offsets,
 * reset/terminate flags and the env's obs row. */
int phc_reset_envs(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                   const uint8_t *env_mask, const float *phase, uint64_t seed, uint64_t counter,
                   void *stream);

/* AMP observation history of HumanoidPHC (humanoid_phc.py:600-611): amp_obs[N, S, 196] with
 * frame 0 = current (_curr_amp_obs_buf) and frames 1..S-1 = history; amp_obs_demo same shape. */
typedef struct phc_amp_buffers {
  float *amp_obs;      /* [N, num_steps, PHC_AMP_OBS_STEP] */
  float *amp_obs_demo; /* [N, num_steps, PHC_AMP_OBS_STEP] */
  int32_t num_steps;   /* cfg.num_amp_obs_steps (10) */
} phc_amp_buffers;

enum {
  PHC_AMP_STEP = 0, /* every env: progress == 0 -> init, else shift history + current frame */
  PHC_AMP_INIT = 1, /* envs with progress == 0 only: init; other envs untouched */
};

/* R16: AMP observations (envs/common.py:180-267 build_amp_observations_smpl with local root obs,
 * root height, dof subset, upright).  PHC_AMP_STEP = _update_hist_amp_obs +
 * _compute_amp_observations of HumanoidPHC.step (humanoid_phc.py:154-157, 1123-1160, 1339-1348);
 * init (envs that were just reset, progress == 0) = _init_amp_obs (:789-836): frame 0 from the
 * sim state, frame k from the motion library at motion_start_time - k*dt (no offset), and
 * amp_obs_demo[env] = amp_obs[env].  Run after phc_env_step (STEP) and after phc_reset_envs
 * (INIT).  Reads rigid_body_state, dof_state, progress, motion_ids, motion_start_times. */
int phc_amp_obs(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_amp_buffers *amp, float dt,
                int32_t mode, void *stream);

/* R13: clip(a,-1,1) when `clip` (EnvConfig.clip_actions), pd = offset + scale*a, frozen dofs = 0
 * (clean_pufferl/env.py:91-93, humanoid_phc.py:106-128, 1216-1226). */
int phc_actions_to_pd(const float *actions, float *pd_target, int64_t n, const float *offset,
                      const float *scale, const uint8_t *frozen, int32_t clip, void *stream);

/* Physics stand-in (NOT a reference interface; BASELINE configs[1] "physics stubbed"):
 * writes rigid bodies = reference state at the env's next control time + N(0, sigma) noise,
 * dof_vel = reference dof vel + noise, dof_force = noise * force_scale. */
int phc_physics_replay(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                       float pos_sigma, float force_scale, uint64_t seed, uint64_t counter, void *stream);

/* R13 folded into the kernel that consumes the PD targets: the action -> PD-target map of
 * phc_actions_to_pd as an argument block (pd_target is still written, as the env buffer). */
typedef struct phc_pd_map {
  const float *actions; /* [N, 69] policy actions */
  float *pd_target;     /* [N, 69] written */
  const float *offset;  /* [69] */
  const float *scale;   /* [69] */
  const uint8_t *frozen; /* [69] nullable */
  int32_t clip;          /* 1: clip(a, -1, 1) first (EnvConfig.clip_actions, clean_pufferl/env.py:91) */
} phc_pd_map;

typedef struct phc_replay_params {
  float pos_sigma, force_scale;
  uint64_t seed, counter;
} phc_replay_params;

/* HumanoidPHC.step with the physics stand-in in ONE launch (R13 + stand-in + R6,R7,R9-R12,R14):
 * the same buffers and values as phc_actions_to_pd (pd nullable: skipped) -> phc_physics_replay ->
 * phc_env_step, bit for bit; the replayed state IS the blended reference at the step's time, so its
 * frame rows are gathered once and the sim record / dof velocities / forces never make an HBM round
 * trip.  timer nullable (the launch stamps itself into it, as phc_env_step_timed). */
int phc_env_step_replay(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                        const phc_replay_params *replay, const phc_pd_map *pd, phc_kernel_timer *timer,
                        void *stream);

/* N3: articulated-body physics step, replacing `gym.simulate(sim)` x control_freq_inv
 * (puffer_phc/envs/humanoid_phc.py:129-134; sim params envs/isaacgym_env.py:6-42; PD drives
 * humanoid_phc.py:274-281; ground plane :255-262).  Featherstone ABA over the 24-body tree (6-DoF
 * root, 23 ball joints), implicit joint-space PD to pd_target [N,69] (exp-map targets, stiffness /
 * damping x kp_scale / kd_scale), penalty ground contact with capped viscous friction,
 * control_freq_inv x substeps semi-implicit Euler substeps of sim_dt / substeps, optional penalty
 * self-collision, per-link angular damping, angular-velocity clamp.  Reads the root record of
 * rigid_body_state and dof_state, writes rigid_body_state [N,24,13], root_state (if set),
 * dof_state [N,69,2] and dof_force [N,69] (the applied PD torques of the last substep).  Rigid-body
 * linear velocities are those of each body's centre of mass (PhysX's convention; the root record's
 * is read back as such).
 * body_model: device float [PHC_NUM_BODIES][PHC_BODY_MODEL_STRIDE] (layout in phc_physics.hip,
 * packed by puffer-phc_amd/physics.py from assets/smpl_body_model.json). */
#define PHC_BODY_MODEL_STRIDE 80
typedef struct phc_physics_params {
  float sim_dt;             /* 1/60 (isaacgym_env.py:38) */
  int32_t control_freq_inv; /* 2 */
  int32_t substeps;         /* semi-implicit Euler substeps per sim step */
  int32_t tree_depth;       /* deepest body level of the model (root = 0), 1..15; range-checked only:
                               the kernel takes the depth from the body table itself */
  float kp_scale, kd_scale; /* EnvConfig kp_scale / kd_scale */
  float contact_stiffness;  /* N/m per contact point */
  float contact_damping;    /* N s/m per contact point */
  float friction;           /* Coulomb coefficient (ground plane friction 1.0) */
  float friction_damping;   /* N s/m: tangential force = -min(friction_damping, mu fn / |vt|) vt */
  float gravity;            /* m/s^2 along z (-9.81) */
  float angular_damping;    /* per-link angular damping (AssetOptions.angular_damping 0.01,
                               humanoid_phc.py:212): torque -d I_com omega on every body */
  float max_angular_velocity; /* AssetOptions.max_angular_velocity 100 (humanoid_phc.py:213): the
                                 root's and every joint's angular velocity clamped to this magnitude */
  int32_t self_collision;   /* RobotConfig.has_self_collision: penalty contact between the body pairs
                               of the model's collision masks (the reference's shape filter bits,
                               humanoid_phc.py:370-381, minus jointed parent / child pairs) */
} phc_physics_params;
int phc_physics_step(const phc_env_buffers *env, const float *pd_target, const float *body_model,
                     const phc_physics_params *p, void *stream);
/* the same launch stamped into `timer` (bench.py; work = num_envs env-steps) */
int phc_physics_step_timed(const phc_env_buffers *env, const float *pd_target, const float *body_model,
                           const phc_physics_params *p, phc_kernel_timer *timer, void *stream);
/* the same step with R13 folded in: PD targets computed in-kernel from pd->actions (and written to
 * pd->pd_target), replacing phc_actions_to_pd + phc_physics_step (timer nullable) */
int phc_physics_step_actions(const phc_env_buffers *env, const phc_pd_map *pd, const float *body_model,
                             const phc_physics_params *p, phc_kernel_timer *timer, void *stream);

/* R3-R5: load-time FK + velocities (poselib_skeleton.py:518-619, 1230-1251; motion_lib.py:119-140)
 * for `num_motions` clips packed back to back.  quat_global f64 [F,24,4], root_trans f64 [F,3],
 * starts/counts int64 [num_motions], fps float [num_motions].  Writes lib frames/local_rot/
 * dof_vel.  workspace: phc_fk_workspace_bytes(F) bytes. */
size_t phc_fk_workspace_bytes(int64_t num_frames_total);
int phc_fk_motions(const double *quat_global, const double *root_trans, const int64_t *starts,
                   const int64_t *counts, const float *fps, int64_t num_motions, int64_t num_frames_total,
                   const int64_t *parents, const float *local_translation, const double *gauss_weights,
                   int32_t gauss_radius, float *frames, float *local_rot, float *dof_vel, void *workspace,
                   void *stream);

/* R20: compute_gae (puffer_phc/c_gae.pyx:11-32) as a parallel affine scan.
 * workspace: phc_gae_workspace_bytes(n) bytes. */
size_t phc_gae_workspace_bytes(int64_t n);
int phc_gae(const float *dones, const float *values, const float *rewards, int64_t n, float gamma,
            float lam, float *advantages, void *workspace, void *stream);

/* R17: RunningNorm.update / forward (puffer_phc/policies/running_norm.py:15-34).
 * mean/var [cols], count [1] are updated in place; workspace: phc_rms_workspace_bytes(rows, cols). */
size_t phc_rms_workspace_bytes(int64_t rows, int64_t cols);
int phc_rms_update(const float *x, int64_t rows, int64_t cols, float *mean, float *var, float *count,
                   void *workspace, void *stream);
int phc_rms_normalize(const float *x, float *y, int64_t rows, int64_t cols, const float *mean,
                      const float *var, float eps, float clip, void *stream);
/* R17 under data parallelism: phc_rms_moments writes this rank's batch moments
 * moments[cols][2] = (mean, M2) in float64 (same chunked Chan merge as phc_rms_update);
 * the caller gathers every rank's moments [parts][cols][2] and row counts part_rows [parts] and
 * phc_rms_apply merges them in part order (identical on every rank) and applies the running
 * update + count increment.  With one part the result equals phc_rms_update's bit for bit. */
int phc_rms_moments(const float *x, int64_t rows, int64_t cols, double *moments, void *workspace, void *stream);
int phc_rms_apply(const double *moments, const double *part_rows, int32_t parts, int64_t cols, float *mean,
                  float *var, float *count, void *stream);

/* R19/R21: fused epilogues of the twin actor/critic SiLU trunks (policies/phc_policy.py:10-61:
 * nn.Linear bias + nn.SiLU forward, their backward and the bias gradient).  A twin tensor holds
 * `groups` trunks of `cols` columns for `rows` rows, laid out SPLIT [rows, groups*cols] or
 * GROUPED [groups, rows, cols]; elements are dtype (f32 | f16 | bf16), arithmetic fp32, bias
 * and bias_grad fp32 [groups*cols].  cols % 4 == 0. */
enum { PHC_DT_F32 = 0, PHC_DT_F16 = 1, PHC_DT_BF16 = 2 };
enum { PHC_LAYOUT_SPLIT = 0, PHC_LAYOUT_GROUPED = 1 };
enum { PHC_ACT_NONE = 0, PHC_ACT_SILU = 1 };

/* pre = y + bias (same layout and type as y; may be y itself, nullable), out = act(pre) in
 * out_layout (nullable) as out_dtype: equal to dtype, or f16 / bf16 from an f32 y (fp32 GEMM
 * outputs feeding half-precision operands of the next GEMM). */
int phc_bias_act_fwd(const void *y, int32_t y_layout, const float *bias, void *pre, void *out, int32_t out_layout,
                     int64_t rows, int32_t groups, int32_t cols, int32_t act, int32_t dtype, int32_t out_dtype,
                     void *stream);

/* grad_pre = grad_out * act'(pre + pre_bias) (nullable; may be grad_out or pre itself when the
 * layouts and types agree; pre_bias fp32 [groups*cols] nullable, so the forward may keep the raw
 * GEMM output instead of writing pre) and bias_grad = column sums of grad_pre in fp32 (nullable;
 * needs phc_act_bwd_workspace_bytes of workspace).  grad_out and pre are dtype, grad_pre is
 * out_dtype (as phc_bias_act_fwd). */
size_t phc_act_bwd_workspace_bytes(int64_t rows, int32_t groups, int32_t cols);
int phc_act_bwd(const void *grad_out, int32_t grad_out_layout, const void *pre, int32_t pre_layout,
                const float *pre_bias, void *grad_pre, int32_t grad_pre_layout, float *bias_grad, int64_t rows,
                int32_t groups, int32_t cols, int32_t act, int32_t dtype, int32_t out_dtype, void *workspace,
                void *stream);

/* R19/R21: the twin trunks' GEMMs with their epilogues fused (phc_gemm.hip).  For b < batch:
 * C[b] = A[b] · B[b]^T with A[b] [m, k] (lda) and B[b] [n, k] (ldb) row-major f16 / bf16 (dtype),
 * fp32 accumulation; k % 64 == 0 (zero-pad), lda / ldb multiples of 8, 16-byte aligned operands.
 * Output column j of batch b is logical column c = b * n + j of a twin tensor of twin_groups x
 * twin_cols columns (out_layout / aux_layout SPLIT or GROUPED, as phc_bias_act_fwd).  Epilogues
 * (what nn.Linear + nn.SiLU and their autograd backward compute, policies/phc_policy.py:10-61):
 *   STORE     out = C
 *   BIAS      out = C + bias[c]
 *   BIAS_SILU aux = C + bias[c] (fp32 or dtype, nullable), out = silu(C + bias[c])
 *   SILU_GRAD out = C * silu'(aux + bias[c]) (aux fp32 or dtype; bias nullable, e.g. when aux is the
 *             pre-activation BIAS_SILU wrote, bias included), and
 *             bias_grad[c] = column sums of that product in fp32 (nullable; needs
 *             phc_twin_gemm_workspace_bytes of workspace)
 *   BIAS_RELU out = relu(C + bias[c])   (AMP discriminator Linear + ReLU,
 *             puffer_phc/policies/discriminator_policy.py:43-53)
 *   RELU_GRAD out = C * [aux + bias[c] > 0] (aux = the BIAS_RELU output, bias null: torch's
 *             threshold_backward reads the ReLU result), bias_grad as SILU_GRAD
 *   BIAS_SILU_D  as BIAS_SILU, but aux = silu'(C + bias[c]) = s (1 + z (1 - s)), s = sigmoid(z): the
 *             one thing the backward needs of the pre-activation z, in the same bytes (round 5)
 *   DSILU_GRAD   out = C * aux (aux = BIAS_SILU_D's silu'; bias must be null), bias_grad as SILU_GRAD
 * out is fp32 or dtype (out_dtype). */
enum { PHC_EPI_STORE = 0, PHC_EPI_BIAS = 1, PHC_EPI_BIAS_SILU = 2, PHC_EPI_SILU_GRAD = 3, PHC_EPI_BIAS_RELU = 4,
       PHC_EPI_RELU_GRAD = 5, PHC_EPI_BIAS_SILU_D = 6, PHC_EPI_DSILU_GRAD = 7 };
typedef struct phc_gemm_desc {
  const void *a;
  const void *b;
  int64_t a_batch_stride, b_batch_stride; /* elements */
  int64_t lda, ldb;                       /* elements */
  int64_t m;
  int32_t n, k, batch, dtype;
  int32_t epilogue, out_dtype;
  const float *bias; /* [batch * n] */
  void *aux;         /* pre-activation (BIAS_SILU: written, SILU_GRAD: read), aux_dtype */
  void *out;
  int32_t aux_layout, out_layout;
  int32_t twin_groups, twin_cols;
  int32_t aux_dtype; /* PHC_DT_F32, or dtype: the pre-activation kept in the operand type, as
                        torch.autocast's Linear output and SiLU's saved input are */
  int32_t max_workgroups; /* 0: one workgroup per output tile; else at most this many
                             workgroups, each looping over tiles (persistent) */
  int32_t k_valid;        /* 0, or the algorithmic depth when the operands' last k - k_valid columns are
                             zero padding (the first layer's 934 observations padded to 960): only the
                             kernel timer's FLOP count (phc_gemm_set_timer) uses it */
} phc_gemm_desc;
size_t phc_twin_gemm_workspace_bytes(int64_t m, int32_t batch, int32_t n);
/* SILU_GRAD / RELU_GRAD: with a workspace and bias_grad NULL, the launch leaves the bias gradient
 * as per-m-tile column sums, fp32 [phc_twin_gemm_m_tiles(m, n, batch)][batch * n] at the start
 * of the workspace, for the caller to sum (e.g. inside its own phc_reduce_into launch); with
 * bias_grad set they are summed into it by a second launch. */
int64_t phc_twin_gemm_m_tiles(int64_t m, int32_t n, int32_t batch);
int phc_twin_gemm(const phc_gemm_desc *desc, float *bias_grad, void *workspace, void *stream);

/* R21: the twin trunks' weight gradients (the reference's autograd of nn.Linear,
 * policies/phc_policy.py:10-38 under clean_pufferl/core.py:354 loss.backward()).  For b < batch
 * and split s < splits: out[s][b] = G[b][rows_s]^T · Z[b][rows_s] with G[b] [rows, m] (ldg) the
 * layer's output gradient and Z[b] [rows, n] (ldz) its input, row-major f16 / bf16 (dtype), the
 * feature dimension contiguous (as phc_twin_gemm writes them), rows_s the s-th of `splits` equal
 * row chunks; fp32 accumulation, out fp32 [splits, batch, m, n] (summed by the caller, e.g.
 * phc_reduce_into straight into the gradient buffers).  m, n, ldg, ldz, batch strides % 8 == 0,
 * rows % (64 * splits) == 0, 16-byte aligned operands; a batch stride of 0 shares the operand. */
typedef struct phc_wgrad_desc {
  const void *g;
  const void *z;
  int64_t g_batch_stride, z_batch_stride; /* elements */
  int64_t ldg, ldz;                       /* elements */
  int64_t rows;
  int32_t m, n, batch, dtype;
  int32_t splits, reserved;
  float *out;
} phc_wgrad_desc;
int phc_weight_grad(const phc_wgrad_desc *desc, void *stream);

/* The same weight gradients for up to 8 layers in one launch, without a split: problem i adds
 * (accumulate) or stores G[b]^T · Z[b] over all `rows` into fp32 destinations — output row r of
 * batch b goes to dst[b + (r >= split_row)] row r (- split_row when r >= split_row), columns
 * < n_valid, row stride ldd (the first layer's SPLIT [rows, 2 * out] input gradient against the
 * shared padded input: batch 1, split_row = out, n_valid = the unpadded width).  Every output
 * element has one writer: deterministic.  rows % 64 == 0. */
typedef struct phc_wgrad_problem {
  const void *g;
  const void *z;
  int64_t g_batch_stride, z_batch_stride, ldg, ldz; /* elements */
  float *dst[2];
  int64_t ldd;
  int32_t m, n, batch, split_row, n_valid, reserved;
} phc_wgrad_problem;
int phc_weight_grad_group(const phc_wgrad_problem *problems, int32_t count, int64_t rows, int32_t dtype,
                          int32_t accumulate, void *stream);

/* R17 + R19: RunningNorm forward (policies/running_norm.py:15-20) of float32 observations
 * obs [*, d], rows gathered through `rows` (int64 [m], nullable = identity), rounded into the
 * first trunk GEMM's f16 / bf16 operand out [m, ld_out] (columns d..ld_out-1 zero; ld_out % 8
 * == 0, out 16-byte aligned).  Same arithmetic as phc_rms_normalize before the rounding. */
int phc_obs_half(const float *obs, const int64_t *rows, int64_t m, int32_t d, const float *mean,
                 const float *var, float eps, float clip, void *out, int32_t ld_out, int32_t dtype,
                 void *stream);

/* R19 rollout tail (policies/phc_policy.py:40-61, discriminator_policy.py:55-67, pufferlib
 * sample_logits): per row of the twin-trunk output trunk_out [2, rows, hidden] fp32 (actor rows,
 * then critic rows, last Linear bias included): h_g = silu(LayerNorm_g(trunk_out[g])),
 * mu = w_mu h_0 + b_mu, value = w_value . h_1 + b_value, std_j = min(exp(log_sigma_j), std_max),
 * actions = mu + std * noise, logprob = sum_j Normal(mu, std).log_prob(actions).
 * hidden in {256, 512, 768, 1024}; num_actions <= PHC_NUM_DOF + 3; mu nullable; trunk_out
 * 16-byte aligned (the parameters may be 4-byte aligned views into a flat buffer). */
typedef struct phc_policy_act_args {
  const float *trunk_out;             /* [2, rows, hidden] */
  const float *ln_gamma[2];           /* [hidden] each: actor, critic LayerNorm weight */
  const float *ln_beta[2];            /* [hidden] each: actor, critic LayerNorm bias */
  const float *w_mu, *b_mu;           /* [num_actions, hidden], [num_actions] */
  const float *w_value, *b_value;     /* [hidden], [1] */
  const float *log_sigma;             /* [num_actions] */
  const float *noise;                 /* [rows, num_actions] standard normal draws */
  float *actions, *logprob, *value;   /* [rows, num_actions], [rows], [rows] */
  float *mu;                          /* [rows, num_actions], nullable */
  int64_t rows;
  int32_t hidden, num_actions;
  float ln_eps, std_max;
  /* optional: W_mu transposed, [hidden, ld_w_mu_t] fp32, 16-byte aligned, ld_w_mu_t % 4 == 0, >= num_actions:
   * the mu head then reads W rows coalesced across the actions (nullable: w_mu is read) */
  const float *w_mu_t;
  int32_t ld_w_mu_t, reserved;
} phc_policy_act_args;
int phc_policy_act(const phc_policy_act_args *args, void *stream);

/* R19/R21: the twin trunks' LayerNorm(cols) + SiLU (policies/phc_policy.py:16-30) over a GROUPED
 * [groups, rows, cols] tensor y (dtype) with per-group gamma/beta [groups*cols] fp32:
 * z = silu((y - mean) * rstd * gamma + beta) in fp32, mean_rstd [groups*rows, 2] saved.
 * Backward: dy (dtype) and dgamma / dbeta [groups*cols] fp32 from dz [groups, rows, cols] fp32
 * (workspace: phc_ln_silu_workspace_bytes).  cols % 256 == 0, cols <= 1024. */
int phc_ln_silu_fwd(const void *y, const float *gamma, const float *beta, float *z, float *mean_rstd, int64_t rows,
                    int32_t groups, int32_t cols, float eps, int32_t dtype, void *stream);
size_t phc_ln_silu_workspace_bytes(int64_t rows, int32_t groups, int32_t cols);
int phc_ln_silu_bwd(const void *y, const float *gamma, const float *beta, const float *mean_rstd, const float *dz,
                    void *dy, float *dgamma, float *dbeta, int64_t rows, int32_t groups, int32_t cols, int32_t dtype,
                    void *workspace, void *stream);

/* R18: Experience.store (clean_pufferl/structs.py:113-131) on the device.  Each field copies
 * row r of src [n, row_elems] to row (*cursor + rank(r)) of dst [capacity, row_elems] for the
 * rows whose mask byte is set (mask NULL = all rows), in row order, while rows remain;
 * counts[0] = mask-true rows (n_valid), counts[1] = rows taken, counts[2] += n_valid,
 * counts[3] += taken (running sums, zeroed by the caller), *cursor += taken.  cursor and
 * counts are device int64 so a captured hipGraph can replay the call. */
#define PHC_MAX_ROW_FIELDS 12
enum { PHC_ROW_COPY32 = 0, PHC_ROW_COPY64 = 1, PHC_ROW_U8_TO_F32 = 2 };
/* flags: PHC_ROW_SRC_WORDS = the caller guarantees that every aligned 4-byte word overlapping the
 * source's bytes lies inside the source allocation.  A PHC_ROW_U8_TO_F32 field may then be read
 * through its aligned words (the one-round flat copy); without it a flag field takes the per-field
 * byte-load path, so a source that ends (or starts) exactly at an allocation edge is never
 * over-read. */
enum { PHC_ROW_SRC_WORDS = 1 };
typedef struct phc_row_field {
  const void *src;
  void *dst;
  int64_t row_elems; /* elements per row (4-byte, 8-byte or 1-byte source elements by kind) */
  int32_t kind;
  int32_t flags; /* PHC_ROW_SRC_WORDS */
} phc_row_field;
size_t phc_compact_workspace_bytes(int64_t n);
int phc_compact_rows(const phc_row_field *fields, int32_t num_fields, const uint8_t *mask, int64_t n,
                     int64_t *cursor, int64_t capacity, int64_t *counts, void *workspace, void *stream);

/* R21: the update tail of a PPO minibatch (clean_pufferl/core.py:360-372: clip_grad_norm_ +
 * torch.optim.Adam(eps=1e-5), under torch.amp.GradScaler when use_loss_scale) on FLAT fp32
 * buffers param / grad / exp_avg / exp_avg_sq of n elements (16-byte aligned).  The gradient
 * is cut into nblk blocks of at most phc_opt_block_elems() elements that never straddle a
 * parameter: blk_range [nblk, 2] = (start, end), seg_blk [nseg + 1] = first block of each
 * parameter (device int64 / int32 tables).  One call: per-parameter norms of the unscaled
 * gradients, clip coefficient max_norm / (total + 1e-6) (<= 1), loss-scale update and skip
 * on inf / nan (GradScaler: backoff, growth after growth_interval clean steps), Adam step with
 * bias corrections.  state lives in device memory (a captured graph can replay the call);
 * norm_out (device, nullable) = [sum of per-parameter norms, total norm, l2]; with param_init
 * (the flat initial parameters, nullable) l2 = sum over parameters of mean((p - p0)^2) before
 * this step's update (the L2-init regulariser the reference logs, core.py:352-359); norm_acc (device
 * float64 [3], nullable, needs norm_out) += norm_out (a trainer's running sums, no extra launch). */
typedef struct phc_adam_params {
  float lr, beta1, beta2, eps;
  float max_norm;
  int32_t use_loss_scale;
  float growth_factor, backoff_factor;
  int32_t growth_interval;
  int32_t lr_from_state; /* 1: the learning rate is state->lr (device memory), so a captured hipGraph of
                          * the update follows a schedule written between replays; 0: lr above */
} phc_adam_params;
typedef struct phc_opt_state {
  float loss_scale;
  int32_t growth_tracker;
  int32_t step;    /* Adam steps taken */
  int32_t skipped; /* steps skipped for inf / nan gradients */
  float grad_mul, step_size, bc2_sqrt; /* this step's coefficients (written by the call) */
  int32_t skip;
  float lr; /* the learning rate read when phc_adam_params.lr_from_state */
  int32_t reserved;
} phc_opt_state;
int64_t phc_opt_block_elems(void);
size_t phc_opt_workspace_bytes(int32_t nblk);
int phc_opt_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, const int64_t *blk_range,
                 int32_t nblk, const int32_t *seg_blk, int32_t nseg, const phc_adam_params *hp, phc_opt_state *state,
                 float *norm_out, const float *param_init, void *workspace, double *norm_acc, void *stream);
/* The same step with the GEMM-operand copies of the parameters written by the Adam pass itself
 * (what phc_pack_weights would write right after it, from the same fp32 values: f16 / bf16 / fp32
 * copies, row-wise into dst and transposed into dst_t), so no separate operand refresh re-reads the
 * parameters.  `jobs` is a DEVICE table of njobs entries covering [0, n) in order: kind
 * PHC_ADAM_FLAT = elements [off, off + rows) with no copy; kind PHC_ADAM_TILE = a parameter [rows,
 * cols] (row-major, cols contiguous) at flat offset off, processed in 64 x 64 tiles, with
 * dst (nullable, ld dst_ld) and dst_t (nullable, ld dst_t_ld) in `dtype`.  first_block = the job's
 * first workgroup (ascending, first_block[0] = 0), tiles_c = its column tiles (tile jobs);
 * nblocks = the total.  phc_adam_job_blocks() gives a job's workgroup count. */
enum { PHC_ADAM_FLAT = 0, PHC_ADAM_TILE = 1 };
#define PHC_MAX_ADAM_JOBS 256
typedef struct phc_adam_job {
  int64_t off, rows, cols;
  void *dst, *dst_t;
  int64_t dst_ld, dst_t_ld;
  int64_t first_block, tiles_c;
  int32_t dtype, kind;
} phc_adam_job;
int64_t phc_adam_job_blocks(int32_t kind, int64_t rows, int64_t cols);
int phc_opt_step_operands(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                          const int64_t *blk_range, int32_t nblk, const int32_t *seg_blk, int32_t nseg,
                          const phc_adam_params *hp, phc_opt_state *state, float *norm_out, const float *param_init,
                          void *workspace, double *norm_acc, const phc_adam_job *jobs, int32_t njobs, int64_t nblocks,
                          void *stream);

/* R21 gradient plumbing: for each job, dst[r, c] (+= when accumulate) = sum over s < parts of
 * src[s * part_stride + r * src_ld + c] (parts summed in order; dst dense [rows, cols]).  Writes
 * split-K weight-gradient partials and bias gradients of both trunks straight into the flat
 * gradient buffer's per-parameter views (what autograd's per-parameter accumulation did), up to
 * PHC_MAX_REDUCE_JOBS jobs per launch. */
#define PHC_MAX_REDUCE_JOBS 32
typedef struct phc_reduce_job {
  const float *src;
  float *dst;
  int64_t rows, cols, src_ld, part_stride;
  int32_t parts, accumulate;
} phc_reduce_job;
int phc_reduce_into(const phc_reduce_job *jobs, int32_t num_jobs, void *stream);

/* R19 / R21 / R22: the GEMM-operand copies of the fp32 parameters, rewritten after every optimizer
 * step in ONE launch (the reference's modules read their fp32 parameters directly; here the MFMA
 * GEMMs read f16 / bf16 copies: weights [rows, cols] at a leading dimension, and for the
 * input-gradient GEMMs their transposes [cols, rows]; fp32 bias copies use dtype PHC_DT_F32).
 * Rounding is round-to-nearest-even, as torch's copy_.  Job j: dst[r * dst_ld + c] and
 * dst_t[c * dst_t_ld + r] = src[r * src_ld + c] for r < rows, c < cols (dst or dst_t may be NULL);
 * columns of dst beyond cols are not touched (the K padding stays zero). */
#define PHC_MAX_PACK_JOBS 32
typedef struct phc_pack_job {
  const float *src;
  void *dst;
  void *dst_t;
  int64_t rows, cols, src_ld, dst_ld, dst_t_ld;
  int32_t dtype, reserved;
} phc_pack_job;
int phc_pack_weights(const phc_pack_job *jobs, int32_t num_jobs, void *stream);

/* R21: the PPO minibatch objective (clean_pufferl/core.py:298-352 with the fixed-sigma Normal
 * log-prob / entropy of pufferlib.sample_logits and PHCPolicy.bound_loss).  Forward: stats[0] =
 * loss = pg - ent_coef*ent + vf_coef*v + bound_coef*bound, stats[1..7] = pg, v, ent,
 * old_approx_kl, approx_kl, clipfrac, bound (means); row_coef [m,2] saved for the backward;
 * adv_mean_std = {mean, std} of the advantages (device, from the global statistics).
 * stats_acc (device float64 [7], nullable) += stats[1..7] (a trainer's running sums, no extra launch).
 * Backward: d loss / d mu [m,a] and d loss / d value [m] scaled by grad_loss[0] (device). */
#define PHC_PPO_STATS 7
typedef struct phc_ppo_coefs {
  float clip_coef, vf_clip_coef, vf_coef, ent_coef, bound_coef, soft_bound;
  int32_t clip_vloss;
  int32_t reserved;
} phc_ppo_coefs;
size_t phc_ppo_workspace_bytes(int64_t m);
int phc_ppo_loss_fwd(const float *mu, const float *log_sigma, const float *actions, const float *old_logprob,
                     const float *adv, const float *adv_mean_std, const float *value, const float *old_value,
                     const float *returns, int64_t m, int32_t a, const phc_ppo_coefs *coefs, float *row_coef,
                     float *stats, double *stats_acc, void *workspace, void *stream);
int phc_ppo_loss_bwd(const float *mu, const float *log_sigma, const float *actions, const float *row_coef,
                     const float *grad_loss, int64_t m, int32_t a, const phc_ppo_coefs *coefs, float *grad_mu,
                     float *grad_value, void *stream);

/* R19 + R21: the row-wise PPO minibatch tail after the twin trunks (policies/phc_policy.py:16-61
 * LayerNorm + SiLU of both trunks and the critic's value head; their backward).  Forward: h_actor
 * [rows, hidden] (the fp32 operand of the mu-head GEMM) and value [rows].  Backward: from d h_actor
 * [rows, hidden] (= dmu W_mu), dmu [rows, num_actions] and dvalue [rows] (phc_ppo_loss_bwd):
 * dy [2, rows, hidden] in dtype (f16 / bf16: the trunk backward's operand) and per-block partial
 * rows [phc_tail_blocks(rows), stride] whose column offsets phc_tail_layout returns (b_mu,
 * w_value, b_value, ln gamma [2][hidden], ln beta [2][hidden], last trunk layer bias [2][hidden],
 * stride).  hidden == 512, num_actions <= 72. */
typedef struct phc_tail_ln_args {
  const float *trunk_out;          /* [2, rows, hidden] fp32 (actor, critic) */
  const float *ln_gamma[2];        /* [hidden] each */
  const float *ln_beta[2];         /* [hidden] each */
  const float *w_value, *b_value;  /* [hidden], [1] */
  float *h_actor;                  /* [rows, hidden], written by the forward */
  float *value;                    /* [rows], written by the forward */
  int64_t rows;
  int32_t hidden;
  float ln_eps;
} phc_tail_ln_args;
int phc_tail_layout(int32_t num_actions, int32_t hidden, int32_t *offsets /* [7] */);
int32_t phc_tail_blocks(int64_t rows);
int phc_tail_ln_fwd(const phc_tail_ln_args *args, void *stream);
int phc_tail_ln_bwd(const phc_tail_ln_args *args, const float *dh_actor, const float *dmu, const float *dvalue,
                    int32_t num_actions, void *dy, int32_t dtype, float *partial, void *stream);

/* R19 + R21: the actor's mu head, nn.Linear(hidden, num_actions) in fp32
 * (policies/phc_policy.py:40-61; its autograd in clean_pufferl/core.py:298-354), fp32-class on the
 * MFMA: fwd / dgrad split every fp32 operand into three bf16 parts (six bf16 MFMA products per
 * step, fp32 sums; hidden % 32 == 0, else the fp32-input MFMA), wgrad on the fp32-input MFMA
 * (exact products); the summation order differs from a library GEMM's:
 *   fwd  : mu [rows, A] = h [rows, hidden] . w [A, hidden]^T + b [A]   (h, w 16-byte aligned, hidden % 16 == 0)
 *   dgrad: dh [rows, hidden] = dmu [rows, A] . w
 *   wgrad: partial [splits, A, hidden], partial[s] = dmu[rows_s]^T . h[rows_s] over the s-th of
 *          `splits` row chunks of ceil(rows / splits) rows (sum over s = the weight gradient).
 * A = num_actions, 1..80.  Replaces the three library GEMMs around phc_tail_ln_fwd / _bwd. */
int phc_mu_head_fwd(const float *h, const float *w, const float *b, float *mu, int64_t rows, int32_t hidden,
                    int32_t num_actions, void *stream);
int phc_mu_head_dgrad(const float *dmu, const float *w, float *dh, int64_t rows, int32_t hidden, int32_t num_actions,
                      void *stream);
int phc_mu_head_wgrad(const float *dmu, const float *h, float *partial, int64_t rows, int32_t hidden,
                      int32_t num_actions, int32_t splits, void *stream);

/* R22: the AMP discriminator's logits head (puffer_phc/policies/discriminator_policy.py:72-79:
 * Linear(hidden, 1) after the second ReLU layer; the two wide layers run on phc_twin_gemm with the
 * BIAS_RELU / RELU_GRAD epilogues) on h [rows, width] f16 / bf16 (ldh, 16-byte aligned; width
 * 8..1024, % 8), fp32 weights w [width] and bias b [1]:
 *   fwd: logits[r] = h[r] . w + b (nullable) and reward[r] = -log(max(1 - sigmoid(logits[r]), 1e-4))
 *        (nullable; the adversarial reward of clean_pufferl/core.py:229-242).
 *   bwd: from grad_logits [rows] fp32: grad_h[r, j] = grad_logits[r] * w[j] * [h[r, j] > 0] in dtype
 *        (ldg), and per-block partial rows parts [phc_disc_head_bwd_blocks(rows), 2 * width + 4] =
 *        [sum gl * h (head weight grad) | sum grad_h in fp32 (second layer bias grad) | sum gl (head
 *        bias grad) | 3 zeros], to be summed over the blocks (phc_reduce_into). */
int64_t phc_disc_head_bwd_blocks(int64_t rows);
int phc_disc_head_fwd(const void *h, int64_t ldh, int64_t rows, int32_t width, int32_t dtype, const float *w,
                      const float *b, float *logits, float *reward, void *stream);
int phc_disc_head_bwd(const void *h, int64_t ldh, int64_t rows, int32_t width, int32_t dtype, const float *w,
                      const float *grad_logits, void *grad_h, int64_t ldg, float *parts, void *stream);

/* Library version and last error (thread-local). */
int phc_version(void);
const char *phc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PHC_H_ */
