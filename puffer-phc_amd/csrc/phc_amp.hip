// phc_amp.hip — AMP discriminator observations (R16, BASELINE config C5).
//
// One 32-lane half-wave per env, lane b = body b, as the env step.  A frame is 196 floats:
//   [0] root height | [1,7) tan-norm of the heading-local root rotation | [7,10) local root vel
//   | [10,13) local root ang vel | [13,127) tan-norm(exp_map->quat) of the 19 subset joints
//   | [127,184) their dof vel | [184,196) heading-local key-body positions (4 bodies)
// (envs/common.py:180-267 with local_root_obs, amp_root_height_obs, has_dof_subset, upright).
// A step shifts the env's 9 history frames back by one (float4 copies, last frame first) and
// writes the new current frame; an env with progress == 0 (just reset) is re-initialised from
// its sim state and the motion library instead (humanoid_phc.py:789-836).
#include "phc_common.h"

namespace phc {

constexpr int kAmp = PHC_AMP_OBS_STEP;
static_assert(kAmp % 4 == 0, "AMP frame must be float4-aligned");

// dof-subset rank of body b's joint (DOF_NAMES minus L/R_Hand, L/R_Toe: body_sets.py:42), -1 if
// excluded (and for the root, which has no dof)
__constant__ int8_t kDofRank[kBodies] = {-1, 0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8,
                                         9, 10, 11, 12, 13, 14, -1, 15, 16, 17, 18, -1};
// slot of body b in KEY_BODIES = (R_Ankle, L_Ankle, R_Wrist, L_Wrist) (body_sets.py:45), -1 if none
__constant__ int8_t kKeySlot[kBodies] = {-1, -1, -1, 1, -1, -1, -1, 0, -1, -1, -1, -1,
                                         -1, -1, -1, -1, -1, 3, -1, -1, -1, -1, 2, -1};

// build_amp_observations_smpl for one env; every lane of the half-wave calls it (the root is
// broadcast from lane 0), active lanes write their slices into `out` (and `out2` if set).
__device__ __forceinline__ void amp_frame(float *__restrict__ out, float *__restrict__ out2, int lane,
                                          const BodyRec &s, v3 dpos, v3 dvel) {
  const bool active = lane < kBodies;
  const v3 root_p = {group_bcast(s.p.x), group_bcast(s.p.y), group_bcast(s.p.z)};
  const q4 root_r = {group_bcast(s.r.x), group_bcast(s.r.y), group_bcast(s.r.z), group_bcast(s.r.w)};
  Heading hrot, hinv;
  heading_quats(root_r, &hrot, &hinv);  // calc_heading_quat_inv (torch_utils.py:396-408)
  if (!active) return;
  float v[6], buf[13];
  int at;
  if (lane == 0) {
    // root_h, tan_norm(quat_mul(heading_inv, root_rot)), local root vel / ang vel
    buf[0] = root_p.z;
    tan_norm_fast(qmul_heading_left(hinv, s.r), v);
#pragma unroll
    for (int k = 0; k < 6; ++k) buf[1 + k] = v[k];
    const v3 lv = rot_heading(hinv, s.v);
    const v3 la = rot_heading(hinv, s.av);
    buf[7] = lv.x; buf[8] = lv.y; buf[9] = lv.z;
    buf[10] = la.x; buf[11] = la.y; buf[12] = la.z;
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      out[k] = buf[k];
      if (out2) out2[k] = buf[k];
    }
  }
  const int r = kDofRank[lane];
  if (r >= 0) {
    // dof_to_obs_smpl (common.py:178-189): tan_norm(exp_map_to_quat(dof_pos triple)), then dof_vel
    tan_norm_fast(exp_map_to_quat(dpos), v);
    at = 13 + 6 * r;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      out[at + k] = v[k];
      if (out2) out2[at + k] = v[k];
    }
    at = 127 + 3 * r;
    out[at] = dvel.x; out[at + 1] = dvel.y; out[at + 2] = dvel.z;
    if (out2) { out2[at] = dvel.x; out2[at + 1] = dvel.y; out2[at + 2] = dvel.z; }
  }
  const int kslot = kKeySlot[lane];
  if (kslot >= 0) {
    const v3 lp = rot_heading(hinv, vsub(s.p, root_p));
    at = 184 + 3 * kslot;
    out[at] = lp.x; out[at + 1] = lp.y; out[at + 2] = lp.z;
    if (out2) { out2[at] = lp.x; out2[at + 1] = lp.y; out2[at + 2] = lp.z; }
  }
}

__global__ __launch_bounds__(kBlock) void k_amp_obs(const float *__restrict__ rb, const float *__restrict__ dof_state,
                                                    const int16_t *__restrict__ progress,
                                                    const int64_t *__restrict__ motion_ids,
                                                    const float *__restrict__ start, LibView l, float *amp,
                                                    float *__restrict__ demo, int steps, int64_t n, float dt,
                                                    int mode) {
  const int64_t env = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kGroup;
  const int lane = threadIdx.x % kGroup;
  if (env >= n) return;  // uniform per half-wave
  const bool init = progress[env] == 0;
  if (!init && mode == PHC_AMP_INIT) return;
  const int b = lane < kBodies ? lane : 0;
  float *a = amp + env * (int64_t)steps * kAmp;
  float *d = demo ? demo + env * (int64_t)steps * kAmp : nullptr;

  if (!init) {
    // _update_hist_amp_obs: frames [0, steps-1) -> [1, steps), last destination first.  Each lane
    // moves the same float4 slots of every frame, so a slot is always read (by this lane) before
    // this lane overwrites it: plain single-thread program order, no barrier needed.
    float4 *a4 = reinterpret_cast<float4 *>(a);
    constexpr int kF4 = kAmp / 4;
    for (int f = steps - 1; f >= 1; --f) {
      float4 t0 = a4[(f - 1) * kF4 + lane];
      float4 t1 = lane + kGroup < kF4 ? a4[(f - 1) * kF4 + lane + kGroup] : float4{0, 0, 0, 0};
      a4[f * kF4 + lane] = t0;
      if (lane + kGroup < kF4) a4[f * kF4 + lane + kGroup] = t1;
    }
  }
  // current frame from the sim state (_compute_amp_observations, humanoid_phc.py:1123-1160)
  const BodyRec s = load_body(rb + (env * kBodies + b) * kRec);
  v3 dpos = {0.0f, 0.0f, 0.0f}, dvel = {0.0f, 0.0f, 0.0f};
  if (b >= 1) {
    const float *q = dof_state + (env * PHC_NUM_DOF + 3 * (b - 1)) * 2;
    dpos = {q[0], q[2], q[4]};
    dvel = {q[1], q[3], q[5]};
  }
  amp_frame(a, init ? d : nullptr, lane, s, dpos, dvel);
  if (!init) return;

  // _init_amp_obs_ref: frame k = reference state at start - k*dt (no offset), demo = amp
  const MotionScalars m = load_motion(l, motion_ids[env]);
  const float st = start[env];
  for (int k = 1; k < steps; ++k) {
    const float tk = st + (-dt) * (float)k;  // motion_times + (-dt * (arange + 1)), fp32
    const Blend bl = frame_blend(tk, m);
    const BodyRec r = ref_body(l.frames, bl, b, nullptr);
    if (b >= 1) {
      dpos = ref_dof_pos(l.local_rot, bl, b);
      dvel = ref_dof_vel(l.dof_vel, bl, b);
    }
    amp_frame(a + k * kAmp, d ? d + k * kAmp : nullptr, lane, r, dpos, dvel);
  }
}

}  // namespace phc

using namespace phc;

extern "C" int phc_amp_obs(const phc_env_buffers *env, const phc_motion_lib *lib, const phc_amp_buffers *amp,
                           float dt, int32_t mode, void *stream) {
  PHC_REQUIRE(env && env->num_envs > 0, "amp_obs: num_envs must be > 0");
  PHC_REQUIRE(env->rigid_body_state && env->dof_state && env->progress && env->motion_ids &&
                  env->motion_start_times,
              "amp_obs: null env buffer");
  PHC_REQUIRE(lib && lib->frames && lib->local_rot && lib->dof_vel && lib->motion_len && lib->motion_dt &&
                  lib->num_frames && lib->length_starts && lib->num_motions > 0,
              "amp_obs: motion lib needs frames, local_rot and dof_vel");
  PHC_REQUIRE(amp && amp->amp_obs, "amp_obs: null amp_obs");
  PHC_REQUIRE(amp->num_steps >= 1 && amp->num_steps <= 64, "amp_obs: num_steps must be in [1, 64]");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(amp->amp_obs) & 15) == 0, "amp_obs: amp_obs must be 16-byte aligned");
  PHC_REQUIRE(mode == PHC_AMP_STEP || mode == PHC_AMP_INIT, "amp_obs: bad mode");
  PHC_REQUIRE(dt > 0.0f, "amp_obs: dt must be > 0");
  const int64_t n = env->num_envs;
  hipLaunchKernelGGL(k_amp_obs, dim3((unsigned)((n + kEnvsPerBlock - 1) / kEnvsPerBlock)), dim3(kBlock), 0,
                     as_stream(stream), env->rigid_body_state, env->dof_state, env->progress, env->motion_ids,
                     env->motion_start_times, lib_view(lib), amp->amp_obs, amp->amp_obs_demo, amp->num_steps, n,
                     dt, (int)mode);
  return check_launch("amp_obs");
}
