// phc_step.hip — per-step env kernels: motion state, fused obs/reward/reset (+PufferEnv
// bookkeeping, + optional in-launch re-initialisation of envs that reset), explicit env
// reset, action->PD, and the replay physics stand-in.
//
// Work decomposition (MI355X): one 32-lane half-wave per env, lane b = body b (24 of 32
// lanes active), 8 envs per 256-thread workgroup.  Per-env reductions (reward means,
// termination any/mean, power) are 5-step butterflies inside the half-wave; the only
// cross-env traffic is the per-workgroup logging row.  Each env reads its 24 rigid-body
// records and the 4 reference frame rows it blends (t and t+dt) straight from HBM and
// writes its 934-float observation row once.
#include "phc_common.h"
#include "phc_measure.h"

#include <hip/hip_ext.h>

#include <vector>

// k_env_step's minimum waves per SIMD (its register budget): 4 = at most 128 VGPRs, which with 40 KB of
// LDS per 8-env workgroup keeps 4 workgroups (16 waves) per CU; 3 let the fused kernel take 129
#ifndef PHC_ENV_WAVES
#define PHC_ENV_WAVES 4
#endif

namespace phc {

struct StepConsts {
  float dt;
  float k_pos, k_rot, k_vel, k_ang;
  float w_pos, w_rot, w_vel, w_ang;
  float power_coef;
  int use_power;
  int enable_et;
  int use_mean;
  unsigned reset_mask;
  float td[kBodies];
  float td_first;     // termination_distance[first reset body] (eval mean rule)
  float inv_nreset;   // 1 / number of reset bodies
  int reset_at_start;  // reset to motion time 0
  unsigned long long seed;
  unsigned long long *clk;  // the launch's timer slot (phc_timer_take), null when untimed
};

static StepConsts make_consts(const phc_step_params *p) {
  StepConsts c;
  c.dt = p->dt;
  c.k_pos = p->k_pos; c.k_rot = p->k_rot; c.k_vel = p->k_vel; c.k_ang = p->k_ang_vel;
  c.w_pos = p->w_pos; c.w_rot = p->w_rot; c.w_vel = p->w_vel; c.w_ang = p->w_ang_vel;
  c.power_coef = p->power_coef;
  c.use_power = p->use_power_reward;
  c.enable_et = p->enable_early_termination;
  c.use_mean = p->use_mean_termination;
  c.reset_mask = p->reset_body_mask & 0xFFFFFFu;
  int n = 0, first = -1;
  for (int b = 0; b < kBodies; ++b) {
    c.td[b] = p->termination_distance[b];
    if (c.reset_mask & (1u << b)) {
      if (first < 0) first = b;
      ++n;
    }
  }
  c.td_first = first >= 0 ? p->termination_distance[first] : 0.0f;
  c.inv_nreset = n > 0 ? 1.0f / (float)n : 0.0f;
  c.reset_at_start = p->reset_at_start;
  c.seed = p->seed;
  c.clk = nullptr;
  return c;
}

struct EnvView {
  int64_t n;
  float *rb;
  float *root;
  float *dof_state;
  const float *dof_force;
  int16_t *progress;
  int64_t *motion_ids;
  float *start;
  float *start_off;
  float *goff;
  float *obs;
  float *rew;
  float *raw;
  uint8_t *reset;
  uint8_t *term;
  uint8_t *terminals;
  uint8_t *truncs;
  uint8_t *masks;
  float *ep_ret;
  int32_t *ep_len;
  double *stats;
  uint32_t *rng;
  void *opnd;  // the fused obs operand (phc_env_buffers.obs_operand), nullable
  const float *opnd_mean, *opnd_var;
  float opnd_eps, opnd_clip;
  int opnd_ld, opnd_bf16;
};

static EnvView env_view(const phc_env_buffers *e) {
  return {e->num_envs, e->rigid_body_state, e->root_state, e->dof_state, e->dof_force, e->progress,
          e->motion_ids, e->motion_start_times, e->motion_start_offset, e->global_offset, e->obs, e->rew,
          e->reward_raw, e->reset, e->terminate, e->terminals, e->truncations, e->masks, e->episode_return,
          e->episode_length, e->stats, e->rng_counter, e->obs_operand, e->obs_norm_mean, e->obs_norm_var,
          e->obs_norm_eps, e->obs_norm_clip, e->obs_operand_ld, e->obs_operand_dtype == PHC_DT_BF16 ? 1 : 0};
}

// ------------------------------------------------------------ motion state --
__global__ __launch_bounds__(kBlock) void k_motion_state(LibView l, const int64_t *__restrict__ ids,
                                                         const float *__restrict__ times,
                                                         const float *__restrict__ offset, int64_t n,
                                                         float *__restrict__ body, float *__restrict__ dof_pos,
                                                         float *__restrict__ dof_vel) {
  const int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kGroup;
  const int b = threadIdx.x % kGroup;
  if (i >= n || b >= kBodies) return;
  const MotionScalars m = load_motion(l, ids[i]);
  const Blend bl = frame_blend(times[i], m);
  v3 off;
  if (offset) off = {offset[3 * i], offset[3 * i + 1], offset[3 * i + 2]};
  const BodyRec r = ref_body(l.frames, bl, b, offset ? &off : nullptr);
  store_body(body + (i * kBodies + b) * kRec, r);
  if (b >= 1) {
    if (dof_pos) {
      const v3 d = ref_dof_pos(l.local_rot, bl, b);
      float *q = dof_pos + i * PHC_NUM_DOF + 3 * (b - 1);
      q[0] = d.x; q[1] = d.y; q[2] = d.z;
    }
    if (dof_vel) {
      const v3 d = ref_dof_vel(l.dof_vel, bl, b);
      float *q = dof_vel + i * PHC_NUM_DOF + 3 * (b - 1);
      q[0] = d.x; q[1] = d.y; q[2] = d.z;
    }
  }
}

// ------------------------------------------------------------- env reset --
// HumanoidPHC.reset(env_ids) for one env (StateInit.Random): sample_time_interval
// (motion_lib.py:526-535), the reference state with the env's previous global offset written
// into the sim buffers (_set_env_state, humanoid_phc.py:899-929), counters cleared
// (_reset_env_tensors :745-778) and offsets cleared (_reset_ref_state_init :692-729).
// Returns this lane's new rigid-body record; the caller then computes the obs at dt + mt.
// rec_stage non-null: the rigid-body record goes to the caller's staging slot (k_env_step's per-wave
// region, written out after) instead of rigid_body_state
__device__ __forceinline__ BodyRec reset_env_state(const EnvView &e, const LibView &l, int64_t env, int lane,
                                                   const MotionScalars &m, float u, float *mt_out,
                                                   float *rec_stage = nullptr) {
  const bool active = lane < kBodies;
  const int b = active ? lane : 0;
  const float fps_step = 1.0f / 30.0f;  // motion_lib.py:532 curr_fps
  const float mt = (float)(int64_t)((u * m.len) / fps_step) * fps_step;
  const v3 go_old = {e.goff[3 * env], e.goff[3 * env + 1], e.goff[3 * env + 2]};
  const Blend bl = frame_blend(mt, m);
  const BodyRec s = ref_body(l.frames, bl, b, &go_old);
  if (active) {
    store_body(rec_stage ? rec_stage : e.rb + (env * kBodies + b) * kRec, s);
    if (b == 0 && e.root) store_body(e.root + env * kRec, s);
    if (b >= 1) {
      const v3 dp = ref_dof_pos(l.local_rot, bl, b);
      const v3 dv = ref_dof_vel(l.dof_vel, bl, b);
      float *d = e.dof_state + (env * PHC_NUM_DOF + 3 * (b - 1)) * 2;
      d[0] = dp.x; d[1] = dv.x; d[2] = dp.y; d[3] = dv.y; d[4] = dp.z; d[5] = dv.z;
    }
  }
  *mt_out = mt;
  return s;
}

__device__ __forceinline__ void reset_env_counters(const EnvView &e, int64_t env, float mt) {
  e.progress[env] = 0;
  e.reset[env] = 0;
  e.term[env] = 0;
  e.goff[3 * env] = 0.0f; e.goff[3 * env + 1] = 0.0f; e.goff[3 * env + 2] = 0.0f;
  e.start[env] = mt;
  e.start_off[env] = 0.0f;
}

// rng_val: the env's rng counter e.rng[env], read by the caller (k_env_step loads it in its first
// memory round)
__device__ __forceinline__ float reset_draw(const EnvView &e, int64_t env, unsigned long long seed,
                                            unsigned long long counter, bool at_start, uint32_t rng_val) {
  if (at_start) return 0.0f;  // StateInit.Start / flag_test: motion_times[:] = 0
  const unsigned long long ctr = e.rng ? (unsigned long long)rng_val : counter;
  return uniform01(seed, ctr, (unsigned long long)env);
}

// Observation of one env from its sim state (this lane's body) and the reference state ref1.
// the observation row of one env from its half-wave into `row` (global memory, or the workgroup's
// LDS staging rows: k_env_step)
__device__ __forceinline__ void env_obs_row(float *row, int lane, const BodyRec &s, const BodyRec &ref1, bool write) {
  const bool active = lane < kBodies;
  const int b = active ? lane : 0;
  const v3 root_p = {group_bcast(s.p.x), group_bcast(s.p.y), group_bcast(s.p.z)};
  const q4 root_r = {group_bcast(s.r.x), group_bcast(s.r.y), group_bcast(s.r.z), group_bcast(s.r.w)};
  Heading hinv, hrot;
  heading_quats(root_r, &hrot, &hinv);
  if (write && active) write_obs_body(row, b, s, root_p, hinv, hrot, ref1);
}

__device__ __forceinline__ void env_obs_ref(const EnvView &e, int64_t env, int lane, const BodyRec &s,
                                            const BodyRec &ref1, bool write) {
  env_obs_row(e.obs + env * kObs, lane, s, ref1, write);
}

// Observation of one env from its sim state and the reference at `t1` (+ offset `off`).
__device__ __forceinline__ void env_obs(const EnvView &e, const LibView &l, int64_t env, int lane,
                                        const MotionScalars &m, const BodyRec &s, float t1, v3 off, bool write) {
  const int b = lane < kBodies ? lane : 0;
  env_obs_ref(e, env, lane, s, ref_body(l.frames, frame_blend(t1, m), b, &off), write);
}

__global__ __launch_bounds__(kBlock) void k_reset_envs(EnvView e, LibView l, StepConsts c,
                                                       const uint8_t *__restrict__ mask,
                                                       const float *__restrict__ phase, unsigned long long seed,
                                                       unsigned long long counter) {
  const int64_t env = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kGroup;
  const int lane = threadIdx.x % kGroup;
  if (env >= e.n) return;
  if (!(mask ? mask[env] : e.reset[env])) return;  // uniform per half-wave
  const MotionScalars m = load_motion(l, e.motion_ids[env]);
  const float u = phase ? phase[env] : reset_draw(e, env, seed, counter, c.reset_at_start != 0, e.rng ? e.rng[env] : 0u);
  float mt;
  const BodyRec s = reset_env_state(e, l, env, lane, m, u, &mt);
  // obs of the reset env: progress 0, start = mt, offsets 0 (humanoid_phc.py:1061-1065)
  env_obs(e, l, env, lane, m, s, (float)(0 + 1) * c.dt + mt + 0.0f, v3{0.0f, 0.0f, 0.0f}, true);
  if (lane == 0) {
    reset_env_counters(e, env, mt);
    if (e.rng && !phase) e.rng[env] += 1u;
  }
}

// --------------------------------------------------------- physics stand-in --
// Triangular noise with standard deviation `sd` from one 32-bit draw (two 16-bit uniforms).
__device__ __forceinline__ float tri_noise32(uint32_t h, float sd) {
  return ((float)(h & 0xFFFFu) - (float)(h >> 16)) * (sd * 2.4494897f / 65536.0f);
}

// xorshift32 (Marsaglia's 13 / 17 / 5): the replay's per-(env, body) noise stream after one splitmix64
// seeding hash.  Round 6: the stream replaced one splitmix64 per noise pair — 9 per body, each two 64-bit
// products of quarter-rate 32-bit multiplies — which made the hashing a large part of the replay's VALU
// time.  Full-rate shifts and xors only.
__device__ __forceinline__ uint32_t xs32(uint32_t &x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

struct ReplayArgs {
  float sigma, force_scale;
  unsigned long long seed, counter;
  // R13 folded in: the action -> PD-target map (actions nullable: no PD targets written)
  const float *actions;
  float *pd;
  const float *off, *scale;
  const uint8_t *frozen;
  int clip;
};

// The replayed sim state of one (env, body): the reference record at the env's next control time
// (`s` = that blend, offset applied) plus noise keyed by (seed, counter, env, body) and, when the env
// has RNG counters, by the env's episode (rng_counter) and step (progress): no per-step host value,
// so a captured graph replays fresh noise every step.  Body b >= 1 also gets its dof velocities
// (reference + noise) and forces (noise), returned in dv / f.
// dv_ref: body b's reference dof velocities at the blend (ref_dof_vel; the caller loads them early)
__device__ __forceinline__ void replay_perturb(const EnvView &e, const ReplayArgs &r, int64_t env, int b, int prog,
                                               BodyRec &s, v3 dv_ref, v3 &dv, v3 &f, uint32_t rng_val) {
  const float sigma = r.sigma;
  unsigned long long key = r.seed ^ mix64(r.counter);
  if (e.rng) key ^= mix64(((unsigned long long)rng_val << 20) ^ (unsigned long long)(unsigned)prog ^ 0x5bd1e995ull);
  const unsigned long long base = mix64(key ^ ((unsigned long long)(env * kBodies + b) << 8));
  uint32_t x = (uint32_t)base ^ (uint32_t)(base >> 32);
  x = x ? x : 0x9E3779B9u;  // xorshift's one fixed point
  s.p.x += tri_noise32(xs32(x), sigma);
  s.p.y += tri_noise32(xs32(x), sigma);
  s.p.z += tri_noise32(xs32(x), sigma);
  q4 q = {s.r.x + tri_noise32(xs32(x), sigma), s.r.y, s.r.z, s.r.w};
  q.y += tri_noise32(xs32(x), sigma);
  q.z += tri_noise32(xs32(x), sigma);
  s.r = quat_unit_env(q);
  s.v.x += tri_noise32(xs32(x), 10.0f * sigma);
  s.v.y += tri_noise32(xs32(x), 10.0f * sigma);
  s.v.z += tri_noise32(xs32(x), 10.0f * sigma);
  s.av.x += tri_noise32(xs32(x), 20.0f * sigma);
  s.av.y += tri_noise32(xs32(x), 20.0f * sigma);
  s.av.z += tri_noise32(xs32(x), 20.0f * sigma);
  dv = {0.0f, 0.0f, 0.0f};
  f = {0.0f, 0.0f, 0.0f};
  if (b >= 1) {
    dv = dv_ref;
    dv.x = dv.x + tri_noise32(xs32(x), 10.0f * sigma);
    dv.y = dv.y + tri_noise32(xs32(x), 10.0f * sigma);
    dv.z = dv.z + tri_noise32(xs32(x), 10.0f * sigma);
    f.x = tri_noise32(xs32(x), r.force_scale);
    f.y = tri_noise32(xs32(x), r.force_scale);
    f.z = tri_noise32(xs32(x), r.force_scale);
  }
}

__device__ __forceinline__ void store_replay(const EnvView &e, int64_t env, int b, const BodyRec &s, v3 dv, v3 f) {
  store_body(e.rb + (env * kBodies + b) * kRec, s);
  if (b >= 1) {
    float *d = e.dof_state + (env * PHC_NUM_DOF + 3 * (b - 1)) * 2;
    d[1] = dv.x; d[3] = dv.y; d[5] = dv.z;
    float *fo = const_cast<float *>(e.dof_force) + env * PHC_NUM_DOF + 3 * (b - 1);
    fo[0] = f.x; fo[1] = f.y; fo[2] = f.z;
  }
}

__device__ const uint8_t kNoFrozen[PHC_NUM_DOF] = {};  // stands in for a null frozen-dof mask
__device__ const uint32_t kZeroU32 = 0;                 // stands in for a null rng counter array
// global-address-space views: a select between two pointers otherwise yields a generic pointer,
// and a flat load forces vmcnt(0) waits on every later use of any load
typedef const __attribute__((address_space(1))) uint8_t gu8;
typedef const __attribute__((address_space(1))) uint32_t gu32;

// R13 (clean_pufferl/env.py:91-93, humanoid_phc.py:1216-1226): clip(a, -1, 1) when cfg.clip_actions,
// pd = offset + scale a, frozen dofs 0
__device__ __forceinline__ float action_to_pd(float x, int d, const float *__restrict__ off,
                                              const float *__restrict__ scale, const uint8_t *__restrict__ frozen,
                                              int clip) {
  if (clip) x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
  return (frozen && frozen[d]) ? 0.0f : off[d] + scale[d] * x;
}

// the 3 PD targets of body b >= 1 (dofs 3(b-1) .. 3(b-1)+2)
__device__ __forceinline__ void map_actions(const ReplayArgs &r, int64_t env, int b) {
  if (!r.actions || b < 1) return;
  const int64_t i0 = env * PHC_NUM_DOF + 3 * (b - 1);
#pragma unroll
  for (int k = 0; k < 3; ++k) r.pd[i0 + k] = action_to_pd(r.actions[i0 + k], 3 * (b - 1) + k, r.off, r.scale, r.frozen, r.clip);
}

// --------------------------------------------------------------- env step --
// Post-physics part of HumanoidPHC.step (humanoid_phc.py:136-146):
//   progress += 1; reward with the reference at t (:1228-1303); reset at t (:1311-1333);
//   obs with the reference at t+dt (:935-959, 1061-1112); then PHCPufferEnv.step's
//   terminals/truncations/masks and episode return/length (clean_pufferl/env.py:103-140)
//   and, with AUTO, the env.reset(reset_indices) of the envs that came up for reset.

struct Outcome {
  float rew, r_pos, r_rot, r_vel, r_ang, pr;
  bool reset, terminated;
};

// reward (common.py:271-322 + power :1295-1303) and reset (common.py:326-364) of one env from
// its half-wave; every lane returns the env's totals
// pw_reg >= 0: this lane's power term already in registers (the fused replay step), else read
__device__ __forceinline__ Outcome env_reward(const EnvView &e, const StepConsts &c, int64_t ei, int lane, int prog,
                                              float t, const MotionScalars &m, const BodyRec &s,
                                              const BodyRec &ref0, float pw_reg = -1.0f) {
  const bool active = lane < kBodies;
  const int b = active ? lane : 0;
  // the means over xyz (/ 3) and over the 24 bodies (/ 24) as products with the reciprocals (1 ulp)
  // under PHC_FAST_ENV_MATH; the reward's exponentials on the hardware exp2
  constexpr float kThird = PHC_FAST_ENV_MATH ? 1.0f / 3.0f : 0.0f;
  constexpr float kInvBodies = PHC_FAST_ENV_MATH ? 1.0f / (float)kBodies : 0.0f;
  auto mean3 = [](float x) { return PHC_FAST_ENV_MATH ? x * kThird : x / 3.0f; };
  const v3 dp = vsub(ref0.p, s.p);
  float e_pos = dp.x * dp.x;
  e_pos = e_pos + dp.y * dp.y;
  e_pos = mean3(e_pos + dp.z * dp.z);
  float sin_t;
  const float ang = quat_angle_masked(quat_mul(ref0.r, quat_conj(s.r)), &sin_t);
  float e_rot = ang * ang;
  const v3 dv = vsub(ref0.v, s.v);
  float e_vel = dv.x * dv.x;
  e_vel = e_vel + dv.y * dv.y;
  e_vel = mean3(e_vel + dv.z * dv.z);
  const v3 da = vsub(ref0.av, s.av);
  float e_ang = da.x * da.x;
  e_ang = e_ang + da.y * da.y;
  e_ang = mean3(e_ang + da.z * da.z);
  // termination distance
  const v3 dd = vsub(s.p, ref0.p);
  const float dist = PHC_FAST_ENV_MATH ? fsqrt_env(dd.x * dd.x + dd.y * dd.y + dd.z * dd.z) : norm3(dd);
  const bool counted = active && ((c.reset_mask >> b) & 1u);
  float fall = (counted && dist > c.td[b]) ? 1.0f : 0.0f;
  float dsum = counted ? dist : 0.0f;
  // power: lane j < 23 owns dofs 3j..3j+2
  float pw = 0.0f;
  if (pw_reg >= 0.0f) {
    pw = pw_reg;
  } else if (lane < kBodies - 1) {
    const float *f = e.dof_force + ei * PHC_NUM_DOF + 3 * lane;
    const float *ds = e.dof_state + (ei * PHC_NUM_DOF + 3 * lane) * 2;
    pw = fabsf(f[0] * ds[1]);
    pw = pw + fabsf(f[1] * ds[3]);
    pw = pw + fabsf(f[2] * ds[5]);
  }
  if (!active) e_pos = e_rot = e_vel = e_ang = 0.0f;
  e_pos = group_sum(e_pos);
  e_rot = group_sum(e_rot);
  e_vel = group_sum(e_vel);
  e_ang = group_sum(e_ang);
  fall = group_sum(fall);
  dsum = group_sum(dsum);
  pw = group_sum(pw);

  Outcome o;
  auto mean_b = [](float x) { return PHC_FAST_ENV_MATH ? x * kInvBodies : x / (float)kBodies; };
  o.r_pos = fexp_env(-c.k_pos * mean_b(e_pos));
  o.r_rot = fexp_env(-c.k_rot * mean_b(e_rot));
  o.r_vel = fexp_env(-c.k_vel * mean_b(e_vel));
  o.r_ang = fexp_env(-c.k_ang * mean_b(e_ang));
  o.rew = c.w_pos * o.r_pos + c.w_rot * o.r_rot + c.w_vel * o.r_vel + c.w_ang * o.r_ang;
  o.pr = 0.0f;
  if (c.use_power) {
    o.pr = -c.power_coef * pw;
    if (prog <= 3) o.pr = 0.0f;
    o.rew = o.rew + o.pr;
  }
  const bool pass_time = t >= m.len;
  o.terminated = false;
  if (c.enable_et) {
    const bool fallen = c.use_mean ? (dsum * c.inv_nreset > c.td_first) : (fall > 0.0f);
    o.terminated = fallen && (prog > 1);
  }
  o.reset = pass_time || o.terminated;
  return o;
}

// lane 0: reward buffers, PHCPufferEnv bookkeeping, this env's logging row
__device__ __forceinline__ void env_bookkeeping(const EnvView &e, int64_t ei, const Outcome &o, double st_row[10]) {
  e.rew[ei] = o.rew;
  float *raw = e.raw + ei * 5;
  raw[0] = o.r_pos; raw[1] = o.r_rot; raw[2] = o.r_vel; raw[3] = o.r_ang; raw[4] = o.pr;
  const bool trunc = o.reset && !o.terminated;
  if (e.terminals) e.terminals[ei] = o.terminated;
  if (e.truncs) e.truncs[ei] = trunc;
  if (e.masks) e.masks[ei] = !trunc;
  if (e.ep_ret) {
    float ret = e.ep_ret[ei];
    int len = e.ep_len[ei];
    if (o.reset) {
      st_row[5] = ret;
      st_row[6] = len;
      st_row[7] = 1.0;
      st_row[8] = trunc ? 1.0 : 0.0;
      st_row[9] = o.terminated ? 1.0 : 0.0;
      ret = 0.0f;
      len = 0;
    }
    e.ep_ret[ei] = ret + o.rew;
    e.ep_len[ei] = len + 1;
  }
  st_row[0] = o.r_pos; st_row[1] = o.r_rot; st_row[2] = o.r_vel; st_row[3] = o.r_ang; st_row[4] = o.pr;
}

// one stats row per workgroup, summed over its envs in LDS, added to the row's old value by ONE vector
// atomic add per slot: this workgroup is the row's only writer in the launch, so the result is the
// load-add-store's bit for bit (an IEEE double add either way) — without a load of the old row at the
// kernel's start whose value (held to the end) cost a spill and a full memory round before any other load
template <int kEnvs, bool kSync = true>
__device__ __forceinline__ void flush_stats(const EnvView &e, double (*sh)[10]) {
  if (kSync) __syncthreads();
  if (threadIdx.x < 10) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kEnvs; ++j) acc += sh[j][threadIdx.x];
    (void)__builtin_amdgcn_global_atomic_fadd_f64(
        (__attribute__((address_space(1))) double *)(e.stats + (int64_t)blockIdx.x * PHC_STATS_SLOTS + threadIdx.x), acc);
  }
}

// Half-wave per env, 8 envs per workgroup: the env step after a separate physics launch (k_env_step).
// The observation rows (the kernel's largest output: 3,736 B per env) are staged in LDS and written
// out by the whole workgroup as 16-B stores: the workgroup's 8 rows are one contiguous 29,888-B
// span of obs [N, 934], so ~8 fully coalesced dwordx4 stores per thread replace 39 scattered dword
// stores per body lane.

// copy `nf` floats of LDS staging rows to global `dst` with 16-B stores (dst 16-B aligned), else 4-B
__device__ __forceinline__ void copy_rows_out(float *__restrict__ dst, const float *__restrict__ src, int nf) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int n4 = nf >> 2;
    for (int i = threadIdx.x; i < n4; i += kBlock)
      reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(src)[i];
    for (int i = (n4 << 2) + threadIdx.x; i < nf; i += kBlock) dst[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < nf; i += kBlock) dst[i] = src[i];
  }
}

// RunningNorm + rounding of the workgroup's staged obs rows into the policy's first-GEMM operand
// (phc_obs_half's expression: (x - mean) / sqrtf(var + eps), clamped, one rounding; columns past
// the 934 observations zero): 16 B per output chunk, rows of the workgroup's contiguous span
template <typename T>
__device__ __forceinline__ void operand_rows_out(const EnvView &e, const float *__restrict__ rows, int64_t env0,
                                                 int nv, int tid, int nthreads) {
  const int chunks = e.opnd_ld / 8;
  for (int i = tid; i < nv * chunks; i += nthreads) {
    const int rr = i / chunks, c0 = (i - rr * chunks) * 8;
    const float *x = rows + rr * kObs;
    T o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v = 0.0f;
      if (c0 + q < kObs) {
        v = (x[c0 + q] - e.opnd_mean[c0 + q]) / sqrtf(e.opnd_var[c0 + q] + e.opnd_eps);
        v = v < -e.opnd_clip ? -e.opnd_clip : (v > e.opnd_clip ? e.opnd_clip : v);
      }
      o[q] = (T)v;
    }
    uint4 raw;
    __builtin_memcpy(&raw, o, sizeof(raw));
    *reinterpret_cast<uint4 *>(static_cast<T *>(e.opnd) + (env0 + rr) * e.opnd_ld + c0) = raw;
  }
}

// Per-wave staging of the fused replay step (k_env_replay): each wave (2 envs) moves its envs' four
// frame rows (t and t+dt blends; 1,248 B each, 16-B aligned in the packed table) into its own LDS
// region by LDS-DMA — 10 wave-instructions of 1 KiB, fully used 64-B lines — instead of 52 scattered
// 4-B lane loads per body; the lanes read their body's records from LDS.  The same region then holds
// the envs' observation rows and replayed rigid-body records, written out by the wave as contiguous
// 16-B stores (the records were 13 scattered 4-B stores per body lane).  Wave-local: no workgroup
// barrier.  9,984 B per wave.
constexpr int kWaveEnvs = 64 / kGroup;            // 2
constexpr int kRowF = kBodies * kRec;             // 312 floats: one frame row = one env's records
constexpr int kRowChunks = kRowF / 4;             // 78 x 16 B
constexpr int kStWave = kWaveEnvs * 4 * kRowF;    // 2,496 floats per wave
constexpr int kStRec = kWaveEnvs * kObs;          // records after the wave's obs rows
constexpr int kStDma = (kWaveEnvs * 4 * kRowChunks + 63) / 64;  // 10 LDS-DMA wave-instructions
static_assert(kStRec % 4 == 0 && kStRec + kWaveEnvs * kRowF <= kStWave, "obs rows + records fit the rows region");

typedef const __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// The slot each of the observation blend's two rows is read from: its own (2, 3), or the reward blend's
// row it repeats (0, 1).  At 30 fps one control step advances one frame, so the t+dt blend's first row
// is the t blend's second one: 3 distinct rows of 4 for most envs, one 1,248-B fetch fewer.
__device__ __forceinline__ int obs_row_slot(int64_t f, int64_t r0, int64_t r1, int own) {
  return f == r1 ? 1 : (f == r0 ? 0 : own);
}

// the wave's 2 x 4 frame rows into `wreg` ([env][row][312]); fr = this lane's env's frame rows, sl2 / sl3
// the slots its observation rows are read from (a row that repeats one of the reward blend's is not fetched)
__device__ __forceinline__ void stage_frame_rows(const float *__restrict__ frames, float *wreg, const int64_t fr[4],
                                                 int sl2, int sl3, int wl) {
  int f0[4], f1[4];  // the rows of the wave's envs (lanes 0 and 32), wave-uniform
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f0[k] = __builtin_amdgcn_readlane((int)fr[k], 0);
    f1[k] = __builtin_amdgcn_readlane((int)fr[k], 32);
  }
  // which of rows 2 / 3 each env fetches (bit 2 / 3 of the mask: rows 0 and 1 always)
  const int need0 = 3 | (__builtin_amdgcn_readlane(sl2, 0) == 2 ? 4 : 0) | (__builtin_amdgcn_readlane(sl3, 0) == 3 ? 8 : 0);
  const int need1 = 3 | (__builtin_amdgcn_readlane(sl2, 32) == 2 ? 4 : 0) | (__builtin_amdgcn_readlane(sl3, 32) == 3 ? 8 : 0);
#pragma unroll
  for (int i = 0; i < kStDma; ++i) {
    const int j = i * 64 + wl;
    if (j >= kWaveEnvs * 4 * kRowChunks) break;  // the last instruction's tail lanes (EXEC-masked) move nothing
    const bool hi = j >= 4 * kRowChunks;
    const int rem = hi ? j - 4 * kRowChunks : j;
    const int rr = rem / kRowChunks, cc = rem - rr * kRowChunks;
    const int fa = rr == 0 ? f0[0] : (rr == 1 ? f0[1] : (rr == 2 ? f0[2] : f0[3]));
    const int fb = rr == 0 ? f1[0] : (rr == 1 ? f1[1] : (rr == 2 ? f1[2] : f1[3]));
    const float *src = frames + (int64_t)(hi ? fb : fa) * kRowF + cc * 4;
    if (((hi ? need1 : need0) >> rr) & 1)
      __builtin_amdgcn_global_load_lds((gvoid *)src, (lvoid *)(wreg + i * 256), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's rows have landed (wave-local region)
}

// The reset state of the envs of a wave that pass their clip's end in this step (t >= len: they reset
// whatever their reward says), by LDS-DMA into the wave's region once its frame rows are in registers:
// for each half-wave with `need`, the two frame rows of its reset blend (-> [env][2][312]), its two
// local-rotation rows ([F, 24, 4] -> kRstLr + [env][2][96]) and its two dof-velocity rows ([F, 23, 3]
// -> kRstDv + [env][2][69]): reset_env_state's loads, landing under the replay / reward arithmetic
// instead of one dependent memory round after it.  No wait (the caller waits before reading).
constexpr int kRstLr = kWaveEnvs * 2 * kRowF;                  // 1,248
constexpr int kRstDv = kRstLr + kWaveEnvs * 2 * kBodies * 4;   // 1,632
static_assert(kRstDv + kWaveEnvs * 2 * PHC_NUM_DOF <= kStWave, "reset words fit the wave's region");

__device__ __forceinline__ void stage_reset_rows(const LibView &l, float *wreg, const Blend &bR, bool need, int wl) {
  const int r00 = __builtin_amdgcn_readlane((int)bR.f0, 0), r01 = __builtin_amdgcn_readlane((int)bR.f1, 0);
  const int r10 = __builtin_amdgcn_readlane((int)bR.f0, 32), r11 = __builtin_amdgcn_readlane((int)bR.f1, 32);
  const bool n0 = __builtin_amdgcn_readlane((int)need, 0) != 0, n1 = __builtin_amdgcn_readlane((int)need, 32) != 0;
  constexpr int kRows = kWaveEnvs * 2 * kRowChunks;  // 312 chunks of 16 B
#pragma unroll
  for (int i = 0; i < (kRows + 63) / 64; ++i) {
    const int j = i * 64 + wl;
    const int h = j >= 2 * kRowChunks;
    const int rem = h ? j - 2 * kRowChunks : j;
    const int rr = rem >= kRowChunks, cc = rr ? rem - kRowChunks : rem;
    const int f = h ? (rr ? r11 : r10) : (rr ? r01 : r00);
    if (j < kRows && (h ? n1 : n0))
      __builtin_amdgcn_global_load_lds((gvoid *)(l.frames + (int64_t)f * kRowF + cc * 4), (lvoid *)(wreg + i * 256), 16,
                                       0, 0);
  }
  constexpr int kLr = kWaveEnvs * 2 * kBodies;  // 96 chunks of 16 B (one quaternion each)
#pragma unroll
  for (int i = 0; i < (kLr + 63) / 64; ++i) {
    const int j = i * 64 + wl;
    const int h = j >= 2 * kBodies;
    const int rem = h ? j - 2 * kBodies : j;
    const int rr = rem >= kBodies, bb = rr ? rem - kBodies : rem;
    const int f = h ? (rr ? r11 : r10) : (rr ? r01 : r00);
    if (j < kLr && (h ? n1 : n0))
      __builtin_amdgcn_global_load_lds((gvoid *)(l.local_rot + ((int64_t)f * kBodies + bb) * 4),
                                       (lvoid *)(wreg + kRstLr + i * 256), 16, 0, 0);
  }
  constexpr int kDv = kWaveEnvs * 2 * PHC_NUM_DOF;  // 276 dwords
#pragma unroll
  for (int i = 0; i < (kDv + 63) / 64; ++i) {
    const int j = i * 64 + wl;
    const int h = j >= 2 * PHC_NUM_DOF;
    const int rem = h ? j - 2 * PHC_NUM_DOF : j;
    const int rr = rem >= PHC_NUM_DOF, k = rr ? rem - PHC_NUM_DOF : rem;
    const int f = h ? (rr ? r11 : r10) : (rr ? r01 : r00);
    if (j < kDv && (h ? n1 : n0))
      __builtin_amdgcn_global_load_lds((gvoid *)(l.dof_vel + (int64_t)f * PHC_NUM_DOF + k),
                                       (lvoid *)(wreg + kRstDv + i * 64), 4, 0, 0);
  }
}

// reset_env_state's values of this lane's body from the staged words (its arithmetic, bit for bit): the
// record (offset: the env's previous global offset), dof position and velocity
__device__ __forceinline__ void staged_reset_values(const float *wreg, int g, int b, float t, v3 go, BodyRec &s,
                                                    v3 &dp, v3 &dv) {
  const float *rr = wreg + g * (2 * kRowF) + b * kRec;
  s = blend_body(load_body(rr), load_body(rr + kRowF), t, &go);
  if (b >= 1) {
    const float *la = wreg + kRstLr + g * (2 * kBodies * 4) + b * 4;
    const float *lc = la + kBodies * 4;
    dp = quat_to_exp_map(slerp(q4{la[0], la[1], la[2], la[3]}, q4{lc[0], lc[1], lc[2], lc[3]}, t));
    const float *da = wreg + kRstDv + g * (2 * PHC_NUM_DOF) + 3 * (b - 1);
    const float *dc = da + PHC_NUM_DOF;
    const float sb = 1.0f - t;
    dv = {sb * da[0] + t * dc[0], sb * da[1] + t * dc[1], sb * da[2] + t * dc[2]};
  }
}

// `nf` floats from the wave's LDS region to global `dst` by the wave's 64 lanes (16-B stores when
// both sides are 16-B aligned)
// the observation rows leave the wave by non-temporal stores: a streamed output (the next launch reads the
// fused half-precision operand, the row store re-reads a few MB) that otherwise evicts the frame rows and
// state the next steps read from the last-level cache (32768 envs: 89.8 -> 81.9 us, profiles/r06zn)
#ifndef PHC_ENV_NT_OBS
#define PHC_ENV_NT_OBS 1
#endif
#ifndef PHC_ENV_NT_REC
#define PHC_ENV_NT_REC 0  // the replayed rigid-body records: measurement switch (the next step's state)
#endif
template <bool NT = false>
__device__ __forceinline__ void wave_copy_out(float *__restrict__ dst, const float *src, int nf, int wl) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int n4 = nf >> 2;
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int i = wl; i < n4; i += 64) {
      const f4v v = reinterpret_cast<const f4v *>(src)[i];
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(dst) + i);
      else reinterpret_cast<f4v *>(dst)[i] = v;
    }
    for (int i = (n4 << 2) + wl; i < nf; i += 64) dst[i] = src[i];
  } else {
    for (int i = wl; i < nf; i += 64) dst[i] = src[i];
  }
}

// the same for one wave's nv <= 2 staged rows: lane l owns output chunks l, l + 64, ..., so each
// column's mean and sqrt(var + eps) are loaded / computed once per lane for both rows (same
// expression, bit-identical values)
template <typename T>
__device__ __forceinline__ void operand_rows_out_wave(const EnvView &e, const float *__restrict__ rows, int64_t env0,
                                                      int nv, int wl) {
  const int chunks = e.opnd_ld / 8;
  for (int ch = wl; ch < chunks; ch += 64) {
    const int c0 = ch * 8;
    float mv[8], dv[8];
    // unconditional loads at clamped columns, selected after: a load behind a per-column select
    // makes hipcc branch around it and wait vmcnt(0) per load (16 dependent L2 round trips)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cq = c0 + q < kObs ? c0 + q : kObs - 1;
      mv[q] = e.opnd_mean[cq];
      dv[q] = e.opnd_var[cq];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool in = c0 + q < kObs;
      mv[q] = in ? mv[q] : 0.0f;
      dv[q] = in ? sqrtf(dv[q] + e.opnd_eps) : 1.0f;
    }
    for (int rr = 0; rr < nv; ++rr) {
      const float *x = rows + rr * kObs;
      T o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = 0.0f;
        if (c0 + q < kObs) {
          v = (x[c0 + q] - mv[q]) / dv[q];
          v = v < -e.opnd_clip ? -e.opnd_clip : (v > e.opnd_clip ? e.opnd_clip : v);
        }
        o[q] = (T)v;
      }
      uint4 raw;
      __builtin_memcpy(&raw, o, sizeof(raw));
      *reinterpret_cast<uint4 *>(static_cast<T *>(e.opnd) + (env0 + rr) * e.opnd_ld + c0) = raw;
    }
  }
}

template <bool AUTO>
__global__ __launch_bounds__(kBlock, PHC_ENV_WAVES) void k_env_step(EnvView e, LibView l, StepConsts c) {
  __shared__ double sh_stats[kEnvsPerBlock][10];
  __shared__ __attribute__((aligned(16))) float sh_obs[kEnvsPerBlock * kObs];  // the workgroup's 8 obs rows
  const int g = threadIdx.x / kGroup;
  const int64_t env = (int64_t)blockIdx.x * kEnvsPerBlock + g;
  const int lane = threadIdx.x % kGroup;
  const bool valid = env < e.n;
  const int b = lane < kBodies ? lane : 0;
  const int64_t ei = valid ? env : 0;

  launch_clock_begin(c.clk);
  // per-env scalars (broadcast loads: every lane of the half-wave reads the same word); the rng
  // counter through a pointer select, so its load joins this round instead of waiting behind a
  // null check where it is used
  const uint32_t rng_val = *(e.rng ? (gu32 *)(e.rng + ei) : (gu32 *)&kZeroU32);
  const int prog = (int)e.progress[ei] + 1;
  const float st = e.start[ei];
  const float so = e.start_off[ei];
  const v3 go = {e.goff[3 * ei], e.goff[3 * ei + 1], e.goff[3 * ei + 2]};
  const MotionScalars m = load_motion(l, e.motion_ids[ei]);
  const float t = (float)prog * c.dt + st + so;
  const float t1n = (float)(prog + 1) * c.dt + st + so;  // observation time unless the env resets
  const Blend bl0 = frame_blend(t, m);
  Blend bl1 = frame_blend(t1n, m);

  // one memory round for the sim record and all four reference rows (t and t+dt)
  BodyRec s = load_body(e.rb + (ei * kBodies + b) * kRec);
  RowPair rows0 = load_rows(l.frames, bl0, b);
  RowPair rows1 = load_rows(l.frames, bl1, b);
  const BodyRec ref0 = blend_body(rows0.a, rows0.c, bl0.b, &go);
  const Outcome o = env_reward(e, c, ei, lane, prog, t, m, s, ref0);
  double st_row[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (valid && lane == 0) env_bookkeeping(e, ei, o, st_row);

  // ---- observation (and in-launch reset) ----
  v3 off1 = go;
  if (AUTO && valid && o.reset) {  // uniform per half-wave
    float mt;
    s = reset_env_state(e, l, ei, lane, m, reset_draw(e, ei, c.seed, 0ull, c.reset_at_start != 0, rng_val), &mt);
    if (lane == 0) {
      reset_env_counters(e, ei, mt);
      if (e.rng) e.rng[ei] = rng_val + 1u;
    }
    // obs of the re-initialised env: progress 0, start = mt, offsets 0 (humanoid_phc.py:1061-1065)
    bl1 = frame_blend((float)(0 + 1) * c.dt + mt + 0.0f, m);
    rows1 = load_rows(l.frames, bl1, b);
    off1 = {0.0f, 0.0f, 0.0f};
  } else if (valid && lane == 0) {
    e.progress[ei] = (int16_t)prog;
    e.reset[ei] = o.reset;
    e.term[ei] = o.terminated;
  }
  env_obs_row(sh_obs + g * kObs, lane, s, blend_body(rows1.a, rows1.c, bl1.b, &off1), valid);
  if (e.stats && lane == 0) {
#pragma unroll
    for (int k = 0; k < 10; ++k) sh_stats[g][k] = st_row[k];
  }
  __syncthreads();  // the staged rows and the stats rows are complete
  {
    const int64_t env0 = (int64_t)blockIdx.x * kEnvsPerBlock;
    const int64_t left = e.n - env0;
    const int nv = left < kEnvsPerBlock ? (int)left : kEnvsPerBlock;
    copy_rows_out(e.obs + env0 * kObs, sh_obs, nv * kObs);
    if (e.opnd) {
      if (e.opnd_bf16) operand_rows_out<__bf16>(e, sh_obs, env0, nv, threadIdx.x, kBlock);
      else operand_rows_out<_Float16>(e, sh_obs, env0, nv, threadIdx.x, kBlock);
    }
  }
  if (e.stats) flush_stats<kEnvsPerBlock, false>(e, sh_stats);
  launch_clock_end(c.clk);
}

// The fused replay step (HumanoidPHC.step with the physics stand-in, ONE launch): the action -> PD map
// (R13), the replayed sim state (k_physics_replay: the reference at t plus noise, which is exactly ref0
// below plus noise, so its frame rows are gathered once) and the post-physics step; the same values as
// k_actions_to_pd -> k_physics_replay -> k_env_step bit for bit.  kWaves waves per workgroup, each wave
// with its own LDS region (per-wave staging above) and its own stats row.
// A passing env (t >= len; it resets in this launch whatever its reward) is known from the scalars: its
// reset time is drawn before the frame rows are fetched, so the observation rows fetched are already
// those of the re-initialised env, and its reset-state words are staged while the replay and reward
// compute.  Before round 6 a resetting env fetched both after its reward, two dependent memory rounds on
// the waves that hold the launch's tail.  Only a terminated env (rare) still does.
template <bool AUTO, int kWaves>
__global__ __launch_bounds__(64 * kWaves, PHC_ENV_WAVES) void k_env_replay(EnvView e, LibView l, StepConsts c,
                                                                           ReplayArgs r) {
  constexpr int kEnvs = kWaves * kWaveEnvs;
  __shared__ double sh_stats[kEnvs][10];
  __shared__ __attribute__((aligned(16))) float sh_reg[kWaves * kStWave];  // one 2,496-float region per wave
  const int w = threadIdx.x >> 6, wl = threadIdx.x & 63;
  const int g = threadIdx.x / kGroup;
  const int gh = g & 1;  // the env's half of its wave
  const int64_t env = (int64_t)blockIdx.x * kEnvs + g;
  const int lane = threadIdx.x % kGroup;
  const bool valid = env < e.n;
  const int b = lane < kBodies ? lane : 0;
  const int64_t ei = valid ? env : 0;
  float *const wreg = sh_reg + w * kStWave;
  const int64_t env0 = (int64_t)blockIdx.x * kEnvs + w * kWaveEnvs;  // the wave's first env
  const int64_t left = e.n - env0;
  const int nv = left <= 0 ? 0 : (left < kWaveEnvs ? (int)left : kWaveEnvs);

  launch_clock_begin(c.clk);
  ENV_PHASE(0);
  // per-env scalars (broadcast loads); the rng counter through a pointer select, so its load joins this
  // round instead of waiting behind a null check where it is used
  const uint32_t rng_val = *(e.rng ? (gu32 *)(e.rng + ei) : (gu32 *)&kZeroU32);
  const int prog = (int)e.progress[ei] + 1;
  const float st = e.start[ei];
  const float so = e.start_off[ei];
  const v3 go = {e.goff[3 * ei], e.goff[3 * ei + 1], e.goff[3 * ei + 2]};
  const int64_t mid = e.motion_ids[ei];
  // R13 for the wave's envs (elementwise over their contiguous [nv, 69] action span, independent of
  // everything else): its loads issued with the scalars', its arithmetic and stores after the motion
  // scalars' loads are issued (stores ahead of them would keep them behind: a memory round more)
  constexpr int kPdIt = (kWaveEnvs * PHC_NUM_DOF + 63) / 64;
  const int cnt = nv * PHC_NUM_DOF;
  float av[kPdIt], ov[kPdIt], sv[kPdIt];
  uint8_t fv[kPdIt];
  if (r.actions) {
    const float *a = r.actions + env0 * PHC_NUM_DOF;
    // every load of the span first (clamped indices, a zero row standing in for a null frozen mask):
    // loads behind a select or a null check made hipcc wait vmcnt(0) per element
    gu8 *fz = r.frozen ? (gu8 *)r.frozen : (gu8 *)kNoFrozen;
#pragma unroll
    for (int u = 0; u < kPdIt; ++u) {
      const int i = wl + 64 * u < cnt ? wl + 64 * u : (cnt > 0 ? cnt - 1 : 0);
      const int d = i >= PHC_NUM_DOF ? i - PHC_NUM_DOF : i;
      av[u] = a[cnt > 0 ? i : 0];
      ov[u] = r.off[d];
      sv[u] = r.scale[d];
      fv[u] = fz[d];
    }
  }
  const MotionScalars m = load_motion(l, mid);
  if (r.actions) {
    float *pd = r.pd + env0 * PHC_NUM_DOF;
#pragma unroll
    for (int u = 0; u < kPdIt; ++u) {
      const int i = wl + 64 * u;
      if (i >= cnt) break;
      float x = av[u];
      if (r.clip) x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
      pd[i] = fv[u] ? 0.0f : ov[u] + sv[u] * x;  // action_to_pd's expression
    }
  }
  const float t = (float)prog * c.dt + st + so;
  const Blend bl0 = frame_blend(t, m);
  // a passing env: reset_env_state's time draw now, its observation at dt + mt (humanoid_phc.py:1061-1065)
  const bool pass = AUTO && valid && t >= m.len;  // env_reward's pass_time; uniform per half-wave
  float mt = 0.0f;
  float tobs = (float)(prog + 1) * c.dt + st + so;  // observation time unless the env resets
  if (pass) {
    const float fps_step = 1.0f / 30.0f;  // motion_lib.py:532 curr_fps
    mt = (float)(int64_t)((reset_draw(e, ei, c.seed, 0ull, c.reset_at_start != 0, rng_val) * m.len) / fps_step) *
         fps_step;
    tobs = (float)(0 + 1) * c.dt + mt + 0.0f;
  }
  Blend bl1 = frame_blend(tobs, m);
  ENV_PHASE_USE(bl1.f0);
  ENV_PHASE(1);

  // the replay's reference dof velocity rows: loaded before the row DMA's wait, in the same memory
  // round, and blended after it (ref_dof_vel's arithmetic)
  v3 dva, dvc;
  {
    const int bb = b >= 1 ? b : 1;
    const float *pa = l.dof_vel + (bl0.f0 * (kBodies - 1) + (bb - 1)) * 3;
    const float *pc = l.dof_vel + (bl0.f1 * (kBodies - 1) + (bb - 1)) * 3;
    dva = {pa[0], pa[1], pa[2]};
    dvc = {pc[0], pc[1], pc[2]};
  }
  const int64_t fr[4] = {bl0.f0, bl0.f1, bl1.f0, bl1.f1};
  const int sl2 = obs_row_slot(bl1.f0, bl0.f0, bl0.f1, 2), sl3 = obs_row_slot(bl1.f1, bl0.f0, bl0.f1, 3);
  stage_frame_rows(l.frames, wreg, fr, sl2, sl3, wl);
  ENV_PHASE(2);
  const float *rw = wreg + gh * (4 * kRowF) + b * kRec;
  const BodyRec ref0 = blend_body(load_body(rw), load_body(rw + kRowF), bl0.b, &go);
  // the observation's reference now (13 registers instead of the two rows' 26): offset 0 for a passing
  // env (a value select: a select of two addresses would put the offsets in scratch)
  const v3 off1 = {pass ? 0.0f : go.x, pass ? 0.0f : go.y, pass ? 0.0f : go.z};
  BodyRec ref1 = blend_body(load_body(rw + sl2 * kRowF), load_body(rw + sl3 * kRowF), bl1.b, &off1);
  // the region is reused below (reset words, replayed records, obs rows) by other lanes of this wave
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wave_lds_handoff();
  Blend blR = {0, 0, 0.0f};
  const bool any_pass = AUTO && __builtin_amdgcn_ballot_w64(pass) != 0;  // wave-uniform
  if (any_pass) {
    if (pass) blR = frame_blend(mt, m);
    stage_reset_rows(l, wreg, blR, pass, wl);
  }

  BodyRec s = ref0;
  v3 dv, f;
  {
    v3 dv_ref = {0.0f, 0.0f, 0.0f};
    if (b >= 1) {
      const float tb = bl0.b, sb = 1.0f - tb;
      dv_ref = {sb * dva.x + tb * dvc.x, sb * dva.y + tb * dvc.y, sb * dva.z + tb * dvc.z};
    }
    replay_perturb(e, r, ei, b, prog, s, dv_ref, dv, f, rng_val);
  }
  // dof vel / force here; the record goes out with the wave's rows at the end
  if (valid && b >= 1) {
    float *d = e.dof_state + (ei * PHC_NUM_DOF + 3 * (b - 1)) * 2;
    d[1] = dv.x; d[3] = dv.y; d[5] = dv.z;
    float *fo = const_cast<float *>(e.dof_force) + ei * PHC_NUM_DOF + 3 * (b - 1);
    fo[0] = f.x; fo[1] = f.y; fo[2] = f.z;
  }
  // power: k_env_step's lane j sums the |force x dof vel| of dofs 3j..3j+2, i.e. body j+1's
  float pw_reg;
  {
    float mine = fabsf(f.x * dv.x);
    mine = mine + fabsf(f.y * dv.y);
    mine = mine + fabsf(f.z * dv.z);
    if (lane >= kBodies) mine = 0.0f;
    pw_reg = next_lane(mine);  // lanes >= 23 (incl. 31, which reads the other env's lane 32) zeroed below
    if (lane >= kBodies - 1) pw_reg = 0.0f;
  }

  const Outcome o = env_reward(e, c, ei, lane, prog, t, m, s, ref0, pw_reg);
  ENV_PHASE_USE(o.reset);
  ENV_PHASE(3);
  if (lane == 0) {  // the env's log row straight into LDS (not 20 registers held to the end)
    double st_row[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (valid) env_bookkeeping(e, ei, o, st_row);
    if (e.stats) {
#pragma unroll
      for (int k = 0; k < 10; ++k) sh_stats[g][k] = st_row[k];
    }
  }

  // ---- in-launch reset (reset_env_state + reset_env_counters) and the observation ----
  if (any_pass) {  // the passing envs' staged words
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pass) {
      v3 dp = {0.0f, 0.0f, 0.0f}, dvr = {0.0f, 0.0f, 0.0f};
      staged_reset_values(wreg, gh, b, blR.b, go, s, dp, dvr);
      if (b >= 1 && lane < kBodies) {
        float *d = e.dof_state + (ei * PHC_NUM_DOF + 3 * (b - 1)) * 2;
        d[0] = dp.x; d[1] = dvr.x; d[2] = dp.y; d[3] = dvr.y; d[4] = dp.z; d[5] = dvr.z;
      }
      if (lane == 0 && e.root) store_body(e.root + ei * kRec, s);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the obs rows / records overwrite them
    wave_lds_handoff();
  }
  if (AUTO && valid && o.reset) {  // uniform per half-wave
    if (!pass) {  // terminated (rare): drawn and loaded now (its record is staged and written out below)
      s = reset_env_state(e, l, ei, lane, m, reset_draw(e, ei, c.seed, 0ull, c.reset_at_start != 0, rng_val), &mt,
                          wreg + kStRec + gh * kRowF + b * kRec);
      const v3 zero = {0.0f, 0.0f, 0.0f};
      ref1 = ref_body(l.frames, frame_blend((float)(0 + 1) * c.dt + mt + 0.0f, m), b, &zero);
    }
    if (lane == 0) {
      reset_env_counters(e, ei, mt);
      if (e.rng) e.rng[ei] = rng_val + 1u;
    }
  } else if (valid && lane == 0) {
    e.progress[ei] = (int16_t)prog;
    e.reset[ei] = o.reset;
    e.term[ei] = o.terminated;
  }
  if (lane < kBodies) store_body(wreg + kStRec + gh * kRowF + b * kRec, s);  // the record, written out below
  env_obs_row(wreg + gh * kObs, lane, s, ref1, valid);
  // the wave writes out its envs' rows (LDS operations of one wave complete in order: the lanes' row
  // writes above are visible to the copy once their issue order is pinned)
  wave_lds_handoff();
  ENV_PHASE(4);
  if (nv > 0) {
    wave_copy_out<PHC_ENV_NT_OBS != 0>(e.obs + env0 * kObs, wreg, nv * kObs, wl);
    wave_copy_out<PHC_ENV_NT_REC != 0>(e.rb + env0 * kRowF, wreg + kStRec, nv * kRowF, wl);
    if (e.opnd) {
      if (e.opnd_bf16) operand_rows_out_wave<__bf16>(e, wreg, env0, nv, wl);
      else operand_rows_out_wave<_Float16>(e, wreg, env0, nv, wl);
    }
  }
  ENV_PHASE(5);
  if (e.stats) {  // this wave's stats row (one per wave: no workgroup barrier), its 2 envs summed in LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wave_lds_handoff();
    if (wl < 10) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kWaveEnvs; ++j) acc += sh_stats[w * kWaveEnvs + j][wl];
      (void)__builtin_amdgcn_global_atomic_fadd_f64(
          (__attribute__((address_space(1))) double *)(e.stats + ((int64_t)blockIdx.x * kWaves + w) * PHC_STATS_SLOTS + wl),
          acc);
    }
  }
  ENV_PHASE(6);
  launch_clock_end(c.clk);
}

__global__ __launch_bounds__(kBlock) void k_physics_replay(EnvView e, LibView l, StepConsts c, ReplayArgs r) {
  const int64_t env = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kGroup;
  const int lane = threadIdx.x % kGroup;
  if (env >= e.n || lane >= kBodies) return;
  const int b = lane;
  const int prog = (int)e.progress[env] + 1;
  const float t = (float)prog * c.dt + e.start[env] + e.start_off[env];
  const MotionScalars m = load_motion(l, e.motion_ids[env]);
  const Blend bl = frame_blend(t, m);
  const v3 go = {e.goff[3 * env], e.goff[3 * env + 1], e.goff[3 * env + 2]};
  BodyRec s = ref_body(l.frames, bl, b, &go);
  v3 dv, f;
  replay_perturb(e, r, env, b, prog, s, b >= 1 ? ref_dof_vel(l.dof_vel, bl, b) : v3{0.0f, 0.0f, 0.0f}, dv, f,
                 e.rng ? e.rng[env] : 0u);
  store_replay(e, env, b, s, dv, f);
}

// --------------------------------------------------------------- actions --
__global__ __launch_bounds__(kBlock) void k_actions_to_pd(const float *__restrict__ a, float *__restrict__ pd,
                                                          int64_t total, const float *__restrict__ off,
                                                          const float *__restrict__ scale,
                                                          const uint8_t *__restrict__ frozen, int clip) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= total) return;
  pd[i] = action_to_pd(a[i], (int)(i % PHC_NUM_DOF), off, scale, frozen, clip);
}

static int grid_envs(int64_t n) { return (int)((n + kEnvsPerBlock - 1) / kEnvsPerBlock); }


static int check_lib(const phc_motion_lib *l) {
  PHC_REQUIRE(l && l->frames && l->motion_len && l->motion_dt && l->num_frames && l->length_starts,
              "motion lib: null tensor");
  PHC_REQUIRE(l->num_motions > 0, "motion lib: no motions");
  return PHC_OK;
}

static int check_env(const phc_env_buffers *e) {
  PHC_REQUIRE(e && e->num_envs > 0, "env: num_envs must be > 0");
  PHC_REQUIRE(e->rigid_body_state && e->dof_state && e->dof_force && e->progress && e->motion_ids &&
                  e->motion_start_times && e->motion_start_offset && e->global_offset && e->obs && e->rew &&
                  e->reward_raw && e->reset && e->terminate,
              "env: null buffer");
  PHC_REQUIRE((e->episode_return == nullptr) == (e->episode_length == nullptr),
              "env: episode_return and episode_length must both be set or both null");
  if (e->obs_operand) {
    PHC_REQUIRE(e->obs_norm_mean && e->obs_norm_var, "env: obs_operand needs the RunningNorm mean and var");
    PHC_REQUIRE(e->obs_operand_ld >= PHC_OBS_DIM && e->obs_operand_ld % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(e->obs_operand) & 15) == 0,
                "env: obs_operand must be 16-byte aligned with ld %% 8 == 0 and ld >= %d", PHC_OBS_DIM);
    PHC_REQUIRE(e->obs_operand_dtype == PHC_DT_F16 || e->obs_operand_dtype == PHC_DT_BF16,
                "env: obs_operand dtype must be f16 or bf16");
  }
  return PHC_OK;
}

}  // namespace phc

using namespace phc;

PHC_ENV_PHASE_COPY

// the fused replay step's workgroup shape: kReplayWaves waves (2 envs each) per workgroup, one stats row
// per wave
#ifndef PHC_REPLAY_WAVES
#define PHC_REPLAY_WAVES 1
#endif
constexpr int kReplayWaves = PHC_REPLAY_WAVES;
constexpr int kReplayEnvs = kReplayWaves * kWaveEnvs;

// stats rows: as many as whichever env kernel writes the most (k_env_replay: one per wave of 2 envs,
// k_env_step: one per 8-env workgroup)
extern "C" int64_t phc_stats_blocks(int64_t num_envs) {
  if (num_envs <= 0) return 0;
  const int64_t a = grid_envs(num_envs), b = (num_envs + kReplayEnvs - 1) / kReplayEnvs * kReplayWaves;
  return a > b ? a : b;
}

extern "C" int phc_motion_state(const phc_motion_lib *lib, const int64_t *ids, const float *times,
                                const float *offset, int64_t n, phc_ref_state *out, void *stream) {
  if (int rc = check_lib(lib)) return rc;
  PHC_REQUIRE(n >= 0, "motion_state: negative n");
  if (n == 0) return PHC_OK;
  PHC_REQUIRE(out && out->body && ids && times, "motion_state: null argument");
  hipLaunchKernelGGL(k_motion_state, dim3(grid_envs(n)), dim3(kBlock), 0, as_stream(stream), lib_view(lib), ids,
                     times, offset, n, out->body, out->dof_pos, out->dof_vel);
  return check_launch("motion_state");
}

// Kernel timer (struct and kernel side in phc_common.h): every timed launch stamps its own start and
// end into its slot of the timer's device buffer.

extern "C" phc_kernel_timer *phc_timer_create(int32_t capacity) {
  if (capacity <= 0) return nullptr;
  auto *t = new phc_kernel_timer;
  t->capacity = capacity;
  // 2 x grid words per slot: room for every slot at up to 1,024 workgroups (the rollout's largest grid)
  t->cap_words = (int64_t)capacity * 2048;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0 || hipMalloc(&t->dev, (size_t)t->cap_words * 8) != hipSuccess ||
      hipMemset(t->dev, 0, (size_t)t->cap_words * 8) != hipSuccess) {
    set_error("timer: device buffer / clock rate unavailable");
    if (t->dev) (void)hipFree(t->dev);
    delete t;
    return nullptr;
  }
  t->tick_hz = 1000.0 * (double)khz;
  return t;
}

extern "C" void phc_timer_destroy(phc_kernel_timer *t) {
  if (!t) return;
  (void)hipDeviceSynchronize();  // no launch may still stamp into the buffer
  (void)hipFree(t->dev);
  delete t;
}

// host copy of the slot words (after every launch issued so far has finished)
static bool timer_words(phc_kernel_timer *t, std::vector<unsigned long long> &w) {
  w.assign((size_t)t->used_words, 0ull);
  if (t->used_words == 0) return true;
  return hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(w.data(), t->dev, (size_t)t->used_words * 8, hipMemcpyDeviceToHost) == hipSuccess;
}

extern "C" void phc_timer_reset(phc_kernel_timer *t) {
  if (!t) return;
  std::vector<unsigned long long> w;
  const bool ok = timer_words(t, w);
  for (auto &s : t->slots) {
    unsigned long long end = 0ull;  // the slot's latest workgroup end so far
    for (int32_t g = 0; ok && s.graph && g < s.grid; ++g) end = w[(size_t)(s.off + s.grid + g)] > end ? w[(size_t)(s.off + s.grid + g)] : end;
    s.end_at_reset = ok && s.graph ? end : ~0ull;
  }
  t->base = t->slots.size();
  t->seen = 0;
}

extern "C" void phc_timer_set_period(phc_kernel_timer *t, int32_t period) {
  if (t) t->period = period > 1 ? period : 1;
}

extern "C" int64_t phc_timer_offered(const phc_kernel_timer *t) { return t ? t->seen : 0; }

// the slots that count since the last reset: the eager ones taken after it, and the graph slots
// re-stamped by a replay after it; -> (launches, work, summed ms)
static bool timer_collect(phc_kernel_timer *t, int32_t *count, double *work, double *ms, double *each = nullptr,
                          int32_t cap = 0) {
  *count = 0;
  *work = *ms = 0.0;
  std::vector<unsigned long long> w;
  if (!timer_words(t, w)) return false;
  for (size_t i = 0; i < t->slots.size(); ++i) {
    const auto &s = t->slots[i];
    unsigned long long start = ~0ull, end = 0ull;
    bool all = true;
    for (int32_t g = 0; g < s.grid; ++g) {
      const unsigned long long v0 = w[(size_t)(s.off + g)], v1 = w[(size_t)(s.off + s.grid + g)];
      all = all && v0 != 0ull && v1 != 0ull;
      start = v0 < start ? v0 : start;
      end = v1 > end ? v1 : end;
    }
    if (!all || (i < t->base && !(s.graph && end != s.end_at_reset))) continue;
    if (!all || end < start) continue;
    const double d = (double)(end - start) / t->tick_hz * 1.0e3;
    if (each && *count < cap) each[*count] = d;
    *count += 1;
    *work += s.work;
    *ms += d;
  }
  return true;
}

// per-launch ms of the counted launches, in the order they were taken (diagnostics); returns the count
extern "C" int32_t phc_timer_durations(phc_kernel_timer *t, double *out, int32_t cap) {
  int32_t c;
  double w, ms;
  return t && timer_collect(t, &c, &w, &ms, out, cap) ? c : -1;
}

extern "C" double phc_timer_work(phc_kernel_timer *t) {
  int32_t c;
  double w, ms;
  return t && timer_collect(t, &c, &w, &ms) ? w : 0.0;
}

extern "C" int32_t phc_timer_count(phc_kernel_timer *t) {
  int32_t c;
  double w, ms;
  return t && timer_collect(t, &c, &w, &ms) ? c : 0;
}

extern "C" double phc_timer_total_ms(phc_kernel_timer *t) {
  int32_t c;
  double w, ms;
  return t && timer_collect(t, &c, &w, &ms) ? ms : -1.0;
}

extern "C" int phc_env_step_timed(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                                  phc_kernel_timer *timer, void *stream) {
  if (int rc = check_env(env)) return rc;
  if (int rc = check_lib(lib)) return rc;
  PHC_REQUIRE(p && p->dt > 0.0f, "env_step: bad params");
  const dim3 block(kBlock), grid(grid_envs(env->num_envs));
  hipStream_t st = as_stream(stream);
  const EnvView ev = env_view(env);
  const LibView lv = lib_view(lib);
  StepConsts cs = make_consts(p);
  cs.clk = phc_timer_take(timer, st, grid.x, (double)env->num_envs);  // work: env-steps
  if (p->auto_reset) {
    PHC_REQUIRE(lib->local_rot && lib->dof_vel, "env_step: auto_reset needs local_rot and dof_vel");
    PHC_REQUIRE(env->rng_counter, "env_step: auto_reset needs rng_counter");
    phc_launch(k_env_step<true>, grid, block, 0, st, ev, lv, cs);
  } else {
    phc_launch(k_env_step<false>, grid, block, 0, st, ev, lv, cs);
  }
  return check_launch("env_step");
}

extern "C" int phc_env_step_replay(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                                   const phc_replay_params *rp, const phc_pd_map *pd, phc_kernel_timer *timer,
                                   void *stream) {
  if (int rc = check_env(env)) return rc;
  if (int rc = check_lib(lib)) return rc;
  PHC_REQUIRE(p && p->dt > 0.0f && rp, "env_step_replay: bad params");
  PHC_REQUIRE(lib->dof_vel, "env_step_replay: motion lib needs dof_vel");
  PHC_REQUIRE(!pd || (pd->actions && pd->pd_target && pd->offset && pd->scale), "env_step_replay: bad pd map");
  ReplayArgs ra{rp->pos_sigma, rp->force_scale, (unsigned long long)rp->seed, (unsigned long long)rp->counter,
                pd ? pd->actions : nullptr, pd ? pd->pd_target : nullptr, pd ? pd->offset : nullptr,
                pd ? pd->scale : nullptr, pd ? pd->frozen : nullptr, pd ? pd->clip : 1};
  const dim3 block(64 * kReplayWaves), grid((unsigned)((env->num_envs + kReplayEnvs - 1) / kReplayEnvs));
  hipStream_t st = as_stream(stream);
  const EnvView ev = env_view(env);
  const LibView lv = lib_view(lib);
  StepConsts cs = make_consts(p);
  cs.clk = phc_timer_take(timer, st, grid.x, (double)env->num_envs);  // work: env-steps
  if (p->auto_reset) {
    PHC_REQUIRE(lib->local_rot, "env_step_replay: auto_reset needs local_rot");
    PHC_REQUIRE(env->rng_counter, "env_step_replay: auto_reset needs rng_counter");
    phc_launch(k_env_replay<true, kReplayWaves>, grid, block, 0, st, ev, lv, cs, ra);
  } else {
    phc_launch(k_env_replay<false, kReplayWaves>, grid, block, 0, st, ev, lv, cs, ra);
  }
  return check_launch("env_step_replay");
}

extern "C" int phc_env_step(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                            void *stream) {
  return phc_env_step_timed(env, lib, p, nullptr, stream);
}

extern "C" int phc_reset_envs(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                              const uint8_t *mask, const float *phase, uint64_t seed, uint64_t counter,
                              void *stream) {
  if (int rc = check_env(env)) return rc;
  if (int rc = check_lib(lib)) return rc;
  PHC_REQUIRE(lib->local_rot && lib->dof_vel, "reset_envs: motion lib needs local_rot and dof_vel");
  PHC_REQUIRE(p && p->dt > 0.0f, "reset_envs: bad params");
  hipLaunchKernelGGL(k_reset_envs, dim3(grid_envs(env->num_envs)), dim3(kBlock), 0, as_stream(stream),
                     env_view(env), lib_view(lib), make_consts(p), mask, phase, (unsigned long long)seed,
                     (unsigned long long)counter);
  return check_launch("reset_envs");
}

extern "C" int phc_physics_replay(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_step_params *p,
                                  float pos_sigma, float force_scale, uint64_t seed, uint64_t counter,
                                  void *stream) {
  if (int rc = check_env(env)) return rc;
  if (int rc = check_lib(lib)) return rc;
  PHC_REQUIRE(lib->dof_vel, "physics_replay: motion lib needs dof_vel");
  PHC_REQUIRE(p, "physics_replay: bad params");
  ReplayArgs ra{pos_sigma, force_scale, (unsigned long long)seed, (unsigned long long)counter,
                nullptr, nullptr, nullptr, nullptr, nullptr, 1};
  hipLaunchKernelGGL(k_physics_replay, dim3(grid_envs(env->num_envs)), dim3(kBlock), 0, as_stream(stream),
                     env_view(env), lib_view(lib), make_consts(p), ra);
  return check_launch("physics_replay");
}

extern "C" int phc_actions_to_pd(const float *actions, float *pd, int64_t n, const float *offset,
                                 const float *scale, const uint8_t *frozen, int32_t clip, void *stream) {
  PHC_REQUIRE(n >= 0, "actions_to_pd: negative n");
  if (n == 0) return PHC_OK;
  PHC_REQUIRE(actions && pd && offset && scale, "actions_to_pd: null argument");
  const int64_t total = n * PHC_NUM_DOF;
  hipLaunchKernelGGL(k_actions_to_pd, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), actions, pd, total, offset, scale, frozen, (int)(clip != 0));
  return check_launch("actions_to_pd");
}
