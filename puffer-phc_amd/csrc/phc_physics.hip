// phc_physics.hip — N3: the articulated-body physics step (replaces gym.simulate x control_freq_inv,
// puffer_phc/envs/humanoid_phc.py:129-134).
//
// Model: the SMPL humanoid of assets/smpl_humanoid.xml as a 24-body tree — a 6-DoF floating root and
// 23 ball joints (the MJCF's three hinges per body, stiffness / damping / armature per axis) — with
// one collision geom per body (sphere / capsule / box) against the ground plane.  Per substep:
//   1. forward kinematics, outward: world pose and body-coordinate twist of every body;
//   2. gravity + penalty ground contact (normal: stiffness x depth - damping x normal velocity,
//      clamped >= 0; tangential: -min(friction_damping, mu fn / |vt|) vt) as body-coordinate wrenches;
//      implicit PD torques tau = kp (target - e) - (kd + dt kp) qd, e = rotation vector of the joint;
//   3. Featherstone's articulated-body algorithm: inward pass of articulated inertias / bias forces
//      (the joint-space diagonal carries armature + dt kd + dt^2 kp, the implicit-PD term), the
//      floating root's 6x6 solve, outward pass of accelerations — all three in the W frame (world
//      orientation, reference point at each body's origin: a level hands its parent a shift only);
//   4. semi-implicit Euler: velocities, then joint / root rotations (quaternions) and root position.
// The CPU restatement is oracle/physics_oracle.py (generic 6x6 matrices, float64).
//
// Decomposition (MI355X): one 32-lane half-wave per env, lane b = body b (24 of 32 lanes), 2 envs
// per single-wave workgroup.  The tree passes run level-synchronously (depth 8 for SMPL): at level L
// the lanes of that level read their parent's (outward) or children's (inward) record from the env's
// LDS slots and write their own; the wave's LDS operations complete in issue order, so a compiler
// barrier separates the levels (phys_sync).  All per-body state stays in registers across the
// substeps; HBM is touched once per env step (read the root record, dof_state and targets; write the
// 24 rigid-body records, dof_state, dof_force).  The kernel is VALU-latency bound: about 6.1 k VALU
// wave-instructions per wave per substep at 2 waves per SIMD.
//
// Body model row (floats, PHC_BODY_MODEL_STRIDE = 80):
//   0 parent  1 level  2 num_children  3..5 children  6..8 joint offset (parent coords)  9 mass
//   10..12 com  13..18 inertia about the com (xx yy zz xy xz yz)  19..21 kp  22..24 kd  25..27 armature
//   28 num_points  32..63 contact points (x y z radius) x 8
//   64..66 / 67..69 self-collision segment end points, 70 its radius (the geom as a capsule)
//   71 self-collision mask: bit j set = this body collides with body j
#include "phc_common.h"

#include <hip/hip_ext.h>

// this file is not held to bit-exact torch rounding (its checker is a float64 restatement): let
// multiply-adds contract into FMAs and divide through the hardware reciprocal
#pragma clang fp contract(fast)

namespace phc {

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

#ifndef PHC_PHYS_EPB
#define PHC_PHYS_EPB 2  // envs per workgroup (half-waves): one wave per workgroup (measured: 8 -> 750 us, 4 -> 711 us, 2 -> 631 us per 4096-env step)
#endif
#ifndef PHC_PHYS_ABLATE
#define PHC_PHYS_ABLATE 0  // measurement builds: bit 1 FK, 2 contacts, 4 inward, 8 outward, 16 root solve skipped
#endif
#ifndef PHC_PHYS_WAVES_PER_SIMD
#define PHC_PHYS_WAVES_PER_SIMD 2  // occupancy pinned (min = max): 3 waves per SIMD measured slower at 16384 envs
#endif

#ifndef PHC_PHYS_COMPACT
#define PHC_PHYS_COMPACT 1  // self-collision: narrow phase over the compacted broad-phase hits
#endif
#ifndef PHC_PHYS_WAVESYNC
#define PHC_PHYS_WAVESYNC 1  // single-wave workgroups: LDS hand-offs ordered without the workgroup barrier
#endif

constexpr int kModel = PHC_BODY_MODEL_STRIDE;
constexpr int kPhysEnvs = PHC_PHYS_EPB;
constexpr int kPhysBlock = kPhysEnvs * kGroup;
constexpr int kSlot = 28;  // LDS floats per body: A(6, sym) B(9) M(6, sym) f(6), padded to 16 B (b128 reads)

// The hand-offs between the tree levels (and the table / pair-list / self-contact exchanges) go
// through LDS between the lanes of ONE wave (one workgroup = one wave of 2 envs): a wave's LDS
// operations are performed in issue order, so a compiler barrier suffices to order them — the
// workgroup barrier's s_waitcnt lgkmcnt(0) drain (~29 per substep) stalled the wave each time.
__device__ __forceinline__ void phys_sync() {
  if constexpr (PHC_PHYS_WAVESYNC && kPhysBlock == 64) asm volatile("" ::: "memory");
  else __syncthreads();
}
constexpr int kMaxPoints = 8;

struct PhysConsts {
  float dt;
  int nsub;
  int depth;
  float kp_scale, kd_scale, kn, cn, mu, ct, g;
  float ang_damp, max_w;
  int self_col;
  unsigned long long *clk;  // the launch's timer slot (phc_timer_take), null when untimed
};

struct M3 {
  float m[9];  // row-major
};

__device__ __forceinline__ M3 m3_quat(float x, float y, float z, float w) {
  return {{1.0f - 2.0f * (y * y + z * z), 2.0f * (x * y - z * w), 2.0f * (x * z + y * w),
           2.0f * (x * y + z * w), 1.0f - 2.0f * (x * x + z * z), 2.0f * (y * z - x * w),
           2.0f * (x * z - y * w), 2.0f * (y * z + x * w), 1.0f - 2.0f * (x * x + y * y)}};
}
__device__ __forceinline__ M3 m3_mul(const M3 &a, const M3 &b) {
  M3 o;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) o.m[3 * i + j] = a.m[3 * i] * b.m[j] + a.m[3 * i + 1] * b.m[3 + j] + a.m[3 * i + 2] * b.m[6 + j];
  return o;
}
__device__ __forceinline__ M3 m3_mul_t(const M3 &a, const M3 &b) {  // a b^T
  M3 o;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      o.m[3 * i + j] = a.m[3 * i] * b.m[3 * j] + a.m[3 * i + 1] * b.m[3 * j + 1] + a.m[3 * i + 2] * b.m[3 * j + 2];
  return o;
}
__device__ __forceinline__ M3 m3_t(const M3 &a) {
  return {{a.m[0], a.m[3], a.m[6], a.m[1], a.m[4], a.m[7], a.m[2], a.m[5], a.m[8]}};
}
__device__ __forceinline__ M3 m3_add(const M3 &a, const M3 &b) {
  M3 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) o.m[i] = a.m[i] + b.m[i];
  return o;
}
__device__ __forceinline__ M3 m3_sub(const M3 &a, const M3 &b) {
  M3 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) o.m[i] = a.m[i] - b.m[i];
  return o;
}
__device__ __forceinline__ M3 m3_skew(v3 r) { return {{0.0f, -r.z, r.y, r.z, 0.0f, -r.x, -r.y, r.x, 0.0f}}; }
__device__ __forceinline__ v3 m3_v(const M3 &a, v3 v) {
  return {a.m[0] * v.x + a.m[1] * v.y + a.m[2] * v.z, a.m[3] * v.x + a.m[4] * v.y + a.m[5] * v.z,
          a.m[6] * v.x + a.m[7] * v.y + a.m[8] * v.z};
}
__device__ __forceinline__ v3 m3_tv(const M3 &a, v3 v) {  // a^T v
  return {a.m[0] * v.x + a.m[3] * v.y + a.m[6] * v.z, a.m[1] * v.x + a.m[4] * v.y + a.m[7] * v.z,
          a.m[2] * v.x + a.m[5] * v.y + a.m[8] * v.z};
}
// inverse of a symmetric 3x3 (adjugate / determinant): the six distinct entries only
__device__ __forceinline__ M3 m3_inv_sym(const M3 &a) {
  const float *m = a.m;
  const float c0 = m[4] * m[8] - m[5] * m[5], c1 = m[5] * m[2] - m[1] * m[8], c2 = m[1] * m[5] - m[4] * m[2];
  const float id = rcp(m[0] * c0 + m[1] * c1 + m[2] * c2);
  const float i00 = c0 * id, i01 = c1 * id, i02 = c2 * id;
  const float i11 = (m[0] * m[8] - m[2] * m[2]) * id, i12 = (m[2] * m[1] - m[0] * m[5]) * id;
  const float i22 = (m[0] * m[4] - m[1] * m[1]) * id;
  return {{i00, i01, i02, i01, i11, i12, i02, i12, i22}};
}
__device__ __forceinline__ v3 cross3(v3 a, v3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// [r]x M (column j = r x M_col j) and M [r]x (row i = M_row i x r) without the skew matrix's zeros
__device__ __forceinline__ M3 skew_mul(v3 r, const M3 &a) {
  M3 o;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const v3 x = cross3(r, v3{a.m[j], a.m[3 + j], a.m[6 + j]});
    o.m[j] = x.x; o.m[3 + j] = x.y; o.m[6 + j] = x.z;
  }
  return o;
}
__device__ __forceinline__ M3 mul_skew(const M3 &a, v3 r) {
  M3 o;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const v3 x = cross3(v3{a.m[3 * i], a.m[3 * i + 1], a.m[3 * i + 2]}, r);
    o.m[3 * i] = x.x; o.m[3 * i + 1] = x.y; o.m[3 * i + 2] = x.z;
  }
  return o;
}
__device__ __forceinline__ v3 vscale(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }

__device__ __forceinline__ q4 qmul_std(q4 a, q4 b) {
  return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
          a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
__device__ __forceinline__ q4 qnormalize(q4 q) {
  const float s = rsqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return {q.x * s, q.y * s, q.z * s, q.w * s};
}
__device__ __forceinline__ q4 quat_from_rotvec(v3 e) {
  const float th = sqrtf(e.x * e.x + e.y * e.y + e.z * e.z);
  const float s = th > 1e-8f ? sinf(0.5f * th) * rcp(th) : 0.5f - th * th * (1.0f / 48.0f);
  return {e.x * s, e.y * s, e.z * s, cosf(0.5f * th)};
}
// exp of a substep's rotation increment (|e| = |omega| dt, small): series to theta^4 below 0.25 rad
// (truncation < 3e-9, below fp32 rounding), the exact form above
__device__ __forceinline__ q4 quat_exp_increment(v3 e) {
  const float t2 = e.x * e.x + e.y * e.y + e.z * e.z;
  if (t2 > 0.0625f) return quat_from_rotvec(e);
  const float s = 0.5f - t2 * (1.0f / 48.0f) + t2 * t2 * (1.0f / 3840.0f);
  const float c = 1.0f - t2 * 0.125f + t2 * t2 * (1.0f / 384.0f);
  return {e.x * s, e.y * s, e.z * s, c};
}
__device__ __forceinline__ v3 rotvec_of(q4 q) {
  if (q.w < 0.0f) q = {-q.x, -q.y, -q.z, -q.w};
  const float sn = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
  const float th = 2.0f * atan2f(sn, q.w);
  const float k = sn > 1e-8f ? th * rcp(sn) : 2.0f * rcp(fmaxf(q.w, 1e-30f));
  return {q.x * k, q.y * k, q.z * k};
}

// symmetric 3x3 products: only the upper triangle of a product known to be symmetric
struct S6 {
  float xx, yy, zz, xy, xz, yz;
};
__device__ __forceinline__ float row_col(const M3 &a, int i, const M3 &b, int j) {  // (a b)_ij
  return a.m[3 * i] * b.m[j] + a.m[3 * i + 1] * b.m[3 + j] + a.m[3 * i + 2] * b.m[6 + j];
}
__device__ __forceinline__ float col_col(const M3 &a, int i, const M3 &b, int j) {  // (a^T b)_ij
  return a.m[i] * b.m[j] + a.m[3 + i] * b.m[3 + j] + a.m[6 + i] * b.m[6 + j];
}
__device__ __forceinline__ float row_row(const M3 &a, int i, const M3 &b, int j) {  // (a b^T)_ij
  return a.m[3 * i] * b.m[3 * j] + a.m[3 * i + 1] * b.m[3 * j + 1] + a.m[3 * i + 2] * b.m[3 * j + 2];
}
__device__ __forceinline__ S6 sym_mul(const M3 &a, const M3 &b) {
  return {row_col(a, 0, b, 0), row_col(a, 1, b, 1), row_col(a, 2, b, 2), row_col(a, 0, b, 1), row_col(a, 0, b, 2),
          row_col(a, 1, b, 2)};
}
__device__ __forceinline__ S6 sym_tmul(const M3 &a, const M3 &b) {
  return {col_col(a, 0, b, 0), col_col(a, 1, b, 1), col_col(a, 2, b, 2), col_col(a, 0, b, 1), col_col(a, 0, b, 2),
          col_col(a, 1, b, 2)};
}
__device__ __forceinline__ M3 s6_full(const S6 &s) { return {{s.xx, s.xy, s.xz, s.xy, s.yy, s.yz, s.xz, s.yz, s.zz}}; }
__device__ __forceinline__ S6 s6_of(const M3 &a) { return {a.m[0], a.m[4], a.m[8], a.m[1], a.m[2], a.m[5]}; }
__device__ __forceinline__ S6 s6_sub(const S6 &a, const S6 &b) {
  return {a.xx - b.xx, a.yy - b.yy, a.zz - b.zz, a.xy - b.xy, a.xz - b.xz, a.yz - b.yz};
}
__device__ __forceinline__ S6 sandwich(const M3 &e, const S6 &s) {  // e s e^T
  const M3 t = m3_mul(e, s6_full(s));
  return {row_row(t, 0, e, 0), row_row(t, 1, e, 1), row_row(t, 2, e, 2), row_row(t, 0, e, 1), row_row(t, 0, e, 2),
          row_row(t, 1, e, 2)};
}
__device__ __forceinline__ void store_s6(const S6 &a, float *s) {
  s[0] = a.xx; s[1] = a.yy; s[2] = a.zz; s[3] = a.xy; s[4] = a.xz; s[5] = a.yz;
}

// symmetric 3x3 (xx yy zz xy xz yz) <-> full
__device__ __forceinline__ M3 sym_full(const float *s) { return {{s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]}}; }
__device__ __forceinline__ void full_sym(const M3 &a, float *s) {
  s[0] = a.m[0]; s[1] = a.m[4]; s[2] = a.m[8];
  s[3] = 0.5f * (a.m[1] + a.m[3]); s[4] = 0.5f * (a.m[2] + a.m[6]); s[5] = 0.5f * (a.m[5] + a.m[7]);
}

struct PhysView {
  int64_t n;
  float *rb;
  float *root;
  float *dof_state;
  float *dof_force;
};

// R13 folded in (phc_pd_map): with actions set, the PD targets are computed here from the actions
// (clip, offset + scale a, frozen dofs 0) and written to pd_target; else pd_target is read
struct PdArgs {
  const float *actions;
  float *pd;
  const float *off, *scale;
  const uint8_t *frozen;
  int clip;
};

// Per-block LDS: the body table with the derived constants (row stride 79 floats: lanes b = 0..23
// reading the same field hit 24 distinct banks), per env the tree-pass slots (FK record 13 / inward
// contribution 27 / acceleration 6 floats) and the self-collision records.  Each body's outward-pass
// operands K = D^-1 A, L = D^-1 B, y = D^-1 u (21 floats) stay in its lane's registers from the
// inward pass to the outward pass (209 VGPRs, still 2 waves per SIMD): held in LDS instead, the
// step ran 2-4 % slower (409 -> 400 us at 4096 envs, 1569 -> 1509 us at 16384; profiles/r06u).
constexpr int kTab = 79;  // odd: the 24 lanes reading one field hit 24 distinct banks
enum : int {
  T_PARENT = 0, T_LEVEL = 1, T_NCH = 2, T_CH = 3, T_OFF = 6, T_MASS = 9, T_COM = 10, T_A0 = 13 /* 9, full */,
  T_KP = 22, T_KD = 25, T_DEXT = 28, T_NPTS = 31, T_PTS = 32 /* 32 */, T_IC = 64 /* 6, sym */,
  T_SEG = 70 /* p0 3, p1 3, radius */, T_MASK = 77, T_OWN = 78 /* contact points the body's lane walks itself */
};
// the lanes past the bodies (kGroup - kBodies per env) walk the contact points of the many-point bodies
// beyond their first kOwnPts (launch table spr_*): a wave walks at most kSparePts points instead of kMaxPoints
constexpr int kSpare = kGroup - kBodies, kOwnPts = 2, kSparePts = 3;
// per env and body, refreshed every substep for the self-collision pass: bounding sphere, world
// segment (start, direction), radius, world angular velocity, world origin velocity, origin
constexpr int kSeg = 20;

__device__ __forceinline__ v3 ld3(const float *p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ M3 ld9(const float *p) {
  M3 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) o.m[i] = p[i];
  return o;
}

__global__ __launch_bounds__(kPhysBlock) __attribute__((amdgpu_waves_per_eu(PHC_PHYS_WAVES_PER_SIMD, PHC_PHYS_WAVES_PER_SIMD))) void k_physics_step(
    PhysView e, const float *__restrict__ model, const float *__restrict__ target, PdArgs pa, PhysConsts c) {
  __shared__ float tab[kBodies * kTab];
  __shared__ __attribute__((aligned(16))) float slots[kPhysEnvs][kBodies][kSlot];
  // the self-collision records: written and read between the outward pass of one substep and the
  // inward pass of the next (the block stays within 20 KB of LDS: 8 workgroups per CU, 2 waves per SIMD)
  __shared__ __attribute__((aligned(16))) float segw[kPhysEnvs][kBodies][kSeg];
  __shared__ float fsc[kPhysEnvs][kBodies][6];  // self-contact wrench per body (world torque, force)
  __shared__ unsigned short pairs[kBodies * (kBodies - 1) / 2];  // colliding pairs i | j << 5, i < j
#if PHC_PHYS_COMPACT
  __shared__ unsigned short hits[kPhysEnvs][kBodies * (kBodies - 1) / 2];  // this substep's broad-phase hits
#endif
  __shared__ int npairs_s;
  __shared__ int spr_b[kSpare], spr_k0[kSpare], spr_k1[kSpare];  // spare lane s: points [k0, k1) of body b (-1: none)
  __shared__ int spr_of[kBodies][2];                                 // the spare lanes walking body b's points
  __shared__ __attribute__((aligned(16))) float spw[kPhysEnvs][kSpare][8];  // their wrenches (torque, force)
  const int lane = threadIdx.x % kGroup, sub = threadIdx.x / kGroup;
  const int64_t env = (int64_t)blockIdx.x * kPhysEnvs + sub;
  const bool act = env < e.n && lane < kBodies;
  const int b = lane < kBodies ? lane : 0;
  const int64_t ev = env < e.n ? env : e.n - 1;
  float(*S)[kSlot] = slots[sub];
  launch_clock_begin(c.clk);
  const float dt = c.dt;

  // ---- body table (indices clamped: a corrupt model cannot address outside the slots)
  if (threadIdx.x < kBodies) {
    const float *md = model + threadIdx.x * kModel;
    float *t = tab + threadIdx.x * kTab;
    t[T_PARENT] = (float)min(max((int)md[0], 0), kBodies - 1);
    t[T_LEVEL] = md[1];
    t[T_NCH] = (float)min(max((int)md[2], 0), 3);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[T_CH + k] = (float)min(max((int)md[3 + k], 0), kBodies - 1);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[T_OFF + k] = md[6 + k];
    const float mass = md[9];
    t[T_MASS] = mass;
    const v3 com = ld3(md + 10);
    t[T_COM] = com.x; t[T_COM + 1] = com.y; t[T_COM + 2] = com.z;
    // spatial inertia about the origin: [[A0, m C], [m C^T, m 1]], A0 = Ic + m C C^T
    const M3 C = m3_skew(com), Ic = sym_full(md + 13), CC = m3_mul_t(C, C);
#pragma unroll
    for (int i = 0; i < 9; ++i) t[T_A0 + i] = Ic.m[i] + mass * CC.m[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float kp = md[19 + k] * c.kp_scale, kd = md[22 + k] * c.kd_scale;
      t[T_KP + k] = kp;
      t[T_KD + k] = kd;
      t[T_DEXT + k] = md[25 + k] + dt * kd + dt * dt * kp;
    }
    const int npts = min(max((int)md[28], 0), kMaxPoints);
    t[T_NPTS] = (float)npts;
    for (int k = 0; k < 4 * kMaxPoints; ++k) t[T_PTS + k] = md[32 + k];
    for (int k = 0; k < 6; ++k) t[T_IC + k] = md[13 + k];
    for (int k = 0; k < 7; ++k) t[T_SEG + k] = md[64 + k];
    t[T_MASK] = c.self_col ? md[71] : 0.0f;
  }
  phys_sync();
  // the pair list (identical for every env): body t's partners j > t at offset = the pair counts
  // of the bodies before it
  if (threadIdx.x < kBodies) {
    const int t = threadIdx.x;
    const unsigned above = ~((2u << t) - 1u);
    int off = 0;
    for (int i = 0; i < t; ++i) off += __popc((unsigned)tab[i * kTab + T_MASK] & ~((2u << i) - 1u));
    unsigned m = (unsigned)tab[t * kTab + T_MASK] & above & ((1u << kBodies) - 1u);
    while (m) {
      const int j = __builtin_ctz(m);
      m &= m - 1u;
      pairs[off++] = (unsigned short)(t | (j << 5));
    }
    if (t == kBodies - 1) npairs_s = off;
  }
  if (threadIdx.x == 0) {  // contact-point split: each spare lane takes <= kSparePts of a body's last points
    int sl = 0;
    for (int i = 0; i < kSpare; ++i) spr_b[i] = -1, spr_k0[i] = spr_k1[i] = 0;
    for (int i = 0; i < kBodies; ++i) {
      int own = (int)tab[i * kTab + T_NPTS];
      spr_of[i][0] = spr_of[i][1] = -1;
      for (int j = 0; j < 2 && own > kOwnPts && sl < kSpare; ++j, ++sl) {
        const int take = min(kSparePts, own - kOwnPts);
        spr_b[sl] = i, spr_k0[sl] = own - take, spr_k1[sl] = own;
        spr_of[i][j] = sl;
        own -= take;
      }
      tab[i * kTab + T_OWN] = (float)own;
    }
  }
  phys_sync();
  const int npairs = npairs_s;
  const float *T = tab + b * kTab;
  const int parent = (int)T[T_PARENT];
  const int level = act ? (int)T[T_LEVEL] : -1;
  const int nch = (int)T[T_NCH];
  const int ch0 = (int)T[T_CH], ch1 = (int)T[T_CH + 1], ch2 = (int)T[T_CH + 2];  // kept in registers
  // the tree passes run over the table's own depth (the host's tree_depth is only range-checked)
  int depth = 0;
  for (int i = 0; i < kBodies; ++i) depth = max(depth, (int)tab[i * kTab + T_LEVEL]);
  depth = min(depth, 15);

  // ---- state: root (lane 0) in body coordinates, joints (lanes >= 1)
  q4 r = {0.0f, 0.0f, 0.0f, 1.0f};
  v3 om = {0.0f, 0.0f, 0.0f}, tgt = {0.0f, 0.0f, 0.0f};
  v3 p0 = {0.0f, 0.0f, 0.0f}, w0 = {0.0f, 0.0f, 0.0f}, v0 = {0.0f, 0.0f, 0.0f};
  q4 q0 = {0.0f, 0.0f, 0.0f, 1.0f};
  if (act && b == 0) {
    const float *s = e.rb + ev * kBodies * kRec;
    p0 = {s[0], s[1], s[2]};
    q0 = qnormalize(q4{s[3], s[4], s[5], s[6]});
    const M3 R0 = m3_quat(q0.x, q0.y, q0.z, q0.w);
    w0 = m3_tv(R0, v3{s[10], s[11], s[12]});
    // the record holds the centre of mass's velocity (PhysX): the origin's is v_com - w x com
    v0 = vsub(m3_tv(R0, v3{s[7], s[8], s[9]}), cross3(w0, ld3(T + T_COM)));
  } else if (act) {
    const float *d = e.dof_state + (ev * PHC_NUM_DOF + 3 * (b - 1)) * 2;
    r = quat_from_rotvec(v3{d[0], d[2], d[4]});
    om = {d[1], d[3], d[5]};
    const int64_t i0 = ev * PHC_NUM_DOF + 3 * (b - 1);
    if (pa.actions) {
      float tv[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float x = pa.actions[i0 + k];
        if (pa.clip) x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
        const int d = 3 * (b - 1) + k;
        tv[k] = (pa.frozen && pa.frozen[d]) ? 0.0f : pa.off[d] + pa.scale[d] * x;
        if (env < e.n) pa.pd[i0 + k] = tv[k];
      }
      tgt = {tv[0], tv[1], tv[2]};
    } else {
      const float *t = target + i0;
      tgt = {t[0], t[1], t[2]};
    }
  }

  q4 Q = {0.0f, 0.0f, 0.0f, 1.0f};
  v3 P = {0.0f, 0.0f, 0.0f}, w = P, v = P;
  v3 rw = P;  // world offset of this body's origin from its parent's (P - P_parent)
  // outward pass: world quaternion / origin and body twist of every body
  auto kinematics = [&]() {
    for (int L = 0; L <= depth; ++L) {
      if (level == L && !(PHC_PHYS_ABLATE & 1)) {
        if (b == 0) {
          Q = q0; P = p0; w = w0; v = v0;
        } else {
          const float *ps = S[parent];
          const q4 Qp = {ps[0], ps[1], ps[2], ps[3]};
          const v3 wp = ld3(ps + 7), off = ld3(T + T_OFF);
          Q = qmul_std(Qp, r);
          rw = m3_v(m3_quat(Qp.x, Qp.y, Qp.z, Qp.w), off);
          P = vadd(ld3(ps + 4), rw);
          const M3 E = m3_quat(r.x, r.y, r.z, r.w);
          w = vadd(m3_tv(E, wp), om);
          v = m3_tv(E, vsub(ld3(ps + 10), cross3(off, wp)));
        }
        float *s = S[b];
        s[0] = Q.x; s[1] = Q.y; s[2] = Q.z; s[3] = Q.w;
        s[4] = P.x; s[5] = P.y; s[6] = P.z;
        s[7] = w.x; s[8] = w.y; s[9] = w.z;
        s[10] = v.x; s[11] = v.y; s[12] = v.z;
      }
      phys_sync();
    }
  };

  v3 applied = {0.0f, 0.0f, 0.0f};
  for (int it = 0; it < c.nsub; ++it) {
    kinematics();
    // ---- bias force pA = V x* (I V) - f_ext (gravity + ground contact), body coordinates
    v3 pt_, pb_, tau = {0.0f, 0.0f, 0.0f}, cw = {0.0f, 0.0f, 0.0f}, cv = {0.0f, 0.0f, 0.0f};
    v3 uw, mcw;  // W frame: the joint torque, mass x centre of mass
    S6 A0w, Dxw;  // W frame: rotational inertia about the origin, the joint-space diagonal R diag(d) R^T
    {
      const M3 R = m3_quat(Q.x, Q.y, Q.z, Q.w);
      const float mass = T[T_MASS];
      const v3 com = ld3(T + T_COM);
      const v3 F = m3_tv(R, v3{0.0f, 0.0f, mass * c.g});
      v3 fn_ = cross3(com, F), ff = F;
      // per-link angular damping (PhysX linear-in-omega damping): torque -d Ic w about the com
      fn_ = vsub(fn_, vscale(m3_v(sym_full(T + T_IC), w), c.ang_damp));
      // penalty self-collision over the pair list, both bodies as capsules
      if (c.self_col) {  // grid-uniform: the barriers below are reached by every wave
        float *sw = segw[sub][b];
        if (act) {
          const v3 s0 = m3_v(R, ld3(T + T_SEG)), s1 = m3_v(R, ld3(T + T_SEG + 3));
          const v3 p0w = vadd(P, s0), d1 = vsub(s1, s0);
          const float rb = T[T_SEG + 6];
          const v3 ww = m3_v(R, w), vw0 = m3_v(R, v);
          // [0, 4): bounding sphere (centre, radius) for the broad phase; then the segment (start,
          // direction), the radius, the world twist and the origin for the narrow phase
          sw[0] = p0w.x + 0.5f * d1.x; sw[1] = p0w.y + 0.5f * d1.y; sw[2] = p0w.z + 0.5f * d1.z;
          sw[3] = 0.5f * sqrtf(d1.x * d1.x + d1.y * d1.y + d1.z * d1.z) + rb;
          sw[4] = p0w.x; sw[5] = p0w.y; sw[6] = p0w.z; sw[7] = d1.x; sw[8] = d1.y; sw[9] = d1.z; sw[10] = rb;
          sw[11] = ww.x; sw[12] = ww.y; sw[13] = ww.z; sw[14] = vw0.x; sw[15] = vw0.y; sw[16] = vw0.z;
          sw[17] = P.x; sw[18] = P.y; sw[19] = P.z;
#pragma unroll
          for (int k = 0; k < 6; ++k) fsc[sub][b][k] = 0.0f;
        }
        phys_sync();
        // each of the env's 32 lanes takes every 32nd pair: broad phase on the bounding spheres,
        // narrow phase (clamped segment-segment closest points) on the overlapping ones, the
        // equal and opposite contact forces added into both bodies' LDS wrench slots (world
        // force, world torque about the body origin)
#if PHC_PHYS_COMPACT
        // broad phase over every pair, the overlapping ones compacted into the env's LDS hit list
        // (wave ballot + prefix counts, no atomics); then the narrow phase over the hits only, spread
        // over the env's lanes — one masked narrow-phase pass per 32 hits instead of one per pair
        // iteration with any hit
        int nh = 0;  // this env's hits (uniform per half-wave)
        {
          const int wl = threadIdx.x & 63;
          const unsigned long long half = (wl >> 5) ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
          const unsigned long long below = (1ull << wl) - 1ull;
          for (int q0 = 0; q0 < npairs; q0 += kGroup) {  // npairs is block-uniform: every lane runs the ballots
            const int q = q0 + lane;
            bool hit = false;
            if (env < e.n && q < npairs) {
              const int pr = pairs[q], bi = pr & 31, bj = pr >> 5;
              const float4 bsi = *reinterpret_cast<const float4 *>(segw[sub][bi]);
              const float4 bsj = *reinterpret_cast<const float4 *>(segw[sub][bj]);
              const float bx = bsj.x - bsi.x, by = bsj.y - bsi.y, bz = bsj.z - bsi.z, br = bsi.w + bsj.w;
              hit = bx * bx + by * by + bz * bz <= br * br;
            }
            const unsigned long long m = __ballot(hit) & half;
            if (hit) hits[sub][nh + __popcll(m & below)] = (unsigned short)q;
            nh += __popcll(m);
          }
        }
        phys_sync();  // the hit list is written (one wave: LDS operations in issue order)
        if (env < e.n) {
          for (int t = lane; t < nh; t += kGroup) {
            const int pr = pairs[hits[sub][t]], bi = pr & 31, bj = pr >> 5;
            const float *oi = segw[sub][bi], *oj = segw[sub][bj];
#else
        if (env < e.n) {
          for (int q = lane; q < npairs; q += kGroup) {
            const int pr = pairs[q], bi = pr & 31, bj = pr >> 5;
            const float *oi = segw[sub][bi], *oj = segw[sub][bj];
            const float4 bsi = *reinterpret_cast<const float4 *>(oi), bsj = *reinterpret_cast<const float4 *>(oj);
            const float bx = bsj.x - bsi.x, by = bsj.y - bsi.y, bz = bsj.z - bsi.z, br = bsi.w + bsj.w;
            if (bx * bx + by * by + bz * bz > br * br) continue;
#endif
            const v3 p0 = ld3(oi + 4), d1 = ld3(oi + 7), q0 = ld3(oj + 4), d2 = ld3(oj + 7);
            const float ri = oi[10], rj = oj[10];
            const v3 r0 = vsub(p0, q0);
            const float a = d1.x * d1.x + d1.y * d1.y + d1.z * d1.z, ee = d2.x * d2.x + d2.y * d2.y + d2.z * d2.z;
            const float f = d2.x * r0.x + d2.y * r0.y + d2.z * r0.z;
            float sp = 0.0f, tp = 0.0f;
            if (a > 1e-12f && ee > 1e-12f) {
              const float cc = d1.x * r0.x + d1.y * r0.y + d1.z * r0.z;
              const float bb = d1.x * d2.x + d1.y * d2.y + d1.z * d2.z;
              const float den = a * ee - bb * bb;
              sp = den > 1e-12f ? fminf(fmaxf((bb * f - cc * ee) / den, 0.0f), 1.0f) : 0.0f;
              tp = (bb * sp + f) / ee;
              if (tp < 0.0f) {
                tp = 0.0f;
                sp = fminf(fmaxf(-cc / a, 0.0f), 1.0f);
              } else if (tp > 1.0f) {
                tp = 1.0f;
                sp = fminf(fmaxf((bb - cc) / a, 0.0f), 1.0f);
              }
            } else if (a > 1e-12f) {
              sp = fminf(fmaxf(-(d1.x * r0.x + d1.y * r0.y + d1.z * r0.z) / a, 0.0f), 1.0f);
            } else if (ee > 1e-12f) {
              tp = fminf(fmaxf(f / ee, 0.0f), 1.0f);
            }
            const v3 c1 = vadd(p0, vscale(d1, sp)), c2 = vadd(q0, vscale(d2, tp));
            const v3 dd = vsub(c2, c1);
            const float dist = sqrtf(dd.x * dd.x + dd.y * dd.y + dd.z * dd.z);
            const float pen = ri + rj - dist;
            if (pen <= 0.0f) continue;
            const v3 nrm = dist > 1e-6f ? vscale(dd, 1.0f / dist) : v3{0.0f, 0.0f, 1.0f};
            const v3 x = vadd(c1, vscale(nrm, ri - 0.5f * pen));  // the contact point (mid overlap)
            const v3 xi = vsub(x, ld3(oi + 17)), xj = vsub(x, ld3(oj + 17));
            const v3 vi = vadd(ld3(oi + 14), cross3(ld3(oi + 11), xi));
            const v3 vj = vadd(ld3(oj + 14), cross3(ld3(oj + 11), xj));
            const v3 vr = vsub(vi, vj);
            const float vn = vr.x * nrm.x + vr.y * nrm.y + vr.z * nrm.z;  // approach rate
            const float fm = fmaxf(0.0f, c.kn * pen + c.cn * vn);
            const v3 Fi = vscale(nrm, -fm);  // pushes i away from j; j gets -Fi
            const v3 ti = cross3(xi, Fi), tj = cross3(xj, Fi);
            float *wi = fsc[sub][bi], *wj = fsc[sub][bj];
            atomicAdd(wi + 0, ti.x); atomicAdd(wi + 1, ti.y); atomicAdd(wi + 2, ti.z);
            atomicAdd(wi + 3, Fi.x); atomicAdd(wi + 4, Fi.y); atomicAdd(wi + 5, Fi.z);
            atomicAdd(wj + 0, -tj.x); atomicAdd(wj + 1, -tj.y); atomicAdd(wj + 2, -tj.z);
            atomicAdd(wj + 3, -Fi.x); atomicAdd(wj + 4, -Fi.y); atomicAdd(wj + 5, -Fi.z);
          }
        }
        phys_sync();
        if (act) {  // this body's accumulated contact wrench, to body coordinates
          const float *ws = fsc[sub][b];
          fn_ = vadd(fn_, m3_tv(R, ld3(ws)));
          ff = vadd(ff, m3_tv(R, ld3(ws + 3)));
        }
        phys_sync();  // segw / fsc are rewritten next substep
      }
      // penalty ground contact: this lane's body's first T_OWN points, and on a spare lane (lane >= kBodies)
      // the points [k0, k1) of the body spr_b assigns it (its pose from that body's kinematics record); the
      // spare lanes hand their wrenches to the body lanes through LDS
      const int sp = lane - kBodies;
      const bool spare = sp >= 0 && env < e.n && !(PHC_PHYS_ABLATE & 2);
      int cb = b, k0 = 0, k1 = (PHC_PHYS_ABLATE & 2) ? 0 : (int)T[T_OWN];
      M3 Rc = R;
      v3 Pc = P, wc = w, vc = v;
      if (spare) {
        cb = spr_b[sp];
        k0 = spr_k0[sp];
        k1 = cb >= 0 ? spr_k1[sp] : 0;
        cb = cb >= 0 ? cb : 0;
        const float *ks = S[cb];
        Rc = m3_quat(ks[0], ks[1], ks[2], ks[3]);
        Pc = ld3(ks + 4);
        wc = ld3(ks + 7);
        vc = ld3(ks + 10);
      }
      const float *Tc = tab + cb * kTab;
      const v3 zb = {Rc.m[6], Rc.m[7], Rc.m[8]};  // R^T z
      v3 tq = {0.0f, 0.0f, 0.0f}, fq = {0.0f, 0.0f, 0.0f};
      for (int k = k0; k < k1; ++k) {
        const float *pt = Tc + T_PTS + 4 * k;
        const v3 cp = ld3(pt);
        const float rho = pt[3];
        const float d = rho - (Pc.z + Rc.m[6] * cp.x + Rc.m[7] * cp.y + Rc.m[8] * cp.z);
        if (d > 0.0f) {
          const v3 a = vsub(cp, vscale(zb, rho));
          const v3 vw = m3_v(Rc, vadd(vc, cross3(wc, a)));
          const float fn = fmaxf(0.0f, c.kn * d - c.cn * vw.z);
          const float vt = sqrtf(vw.x * vw.x + vw.y * vw.y);
          const float kt = fminf(c.ct, c.mu * fn * rcp(fmaxf(vt, 1e-12f)));
          const v3 Fb = m3_tv(Rc, v3{-kt * vw.x, -kt * vw.y, fn});
          tq = vadd(tq, cross3(a, Fb));
          fq = vadd(fq, Fb);
        }
      }
      if (spare) {
        float *o = spw[sub][sp];
        o[0] = tq.x; o[1] = tq.y; o[2] = tq.z; o[3] = fq.x; o[4] = fq.y; o[5] = fq.z;
      }
      phys_sync();
      fn_ = vadd(fn_, tq);
      ff = vadd(ff, fq);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = spr_of[b][j];
        if (q >= 0) {
          const float *o = spw[sub][q];
          fn_ = vadd(fn_, ld3(o));
          ff = vadd(ff, ld3(o + 3));
        }
      }
      // I V = [A0 w + m com x v; m (v - com x w)]
      const v3 h = vadd(m3_v(ld9(T + T_A0), w), vscale(cross3(com, v), mass));
      const v3 l = vscale(vsub(v, cross3(com, w)), mass);
      pt_ = vsub(vadd(cross3(w, h), cross3(v, l)), fn_);
      pb_ = vsub(cross3(w, l), ff);
      if (b > 0) {
        const v3 ej = rotvec_of(r), kp = ld3(T + T_KP), kd = ld3(T + T_KD);
        tau = {kp.x * (tgt.x - ej.x) - (kd.x + dt * kp.x) * om.x, kp.y * (tgt.y - ej.y) - (kd.y + dt * kp.y) * om.y,
               kp.z * (tgt.z - ej.z) - (kd.z + dt * kp.z) * om.z};
        cw = cross3(w, om);
        cv = cross3(v, om);
      }
      // The tree passes run in the W frame: world orientation, reference point at the body's own
      // origin.  A child's quantities then reach its parent by the shift P - P_parent alone, with no
      // rotation inside the level-serial passes (body coordinates needed E (.) E^T on every articulated
      // inertia block once per level); the per-body rotations into W happen here, once per substep, all
      // lanes at once.  The joint's motion subspace is [R; 0], so its joint-space inertia
      // R^T A R + diag(d) becomes A + R diag(d) R^T for the W-frame joint acceleration R qdd.
      pt_ = m3_v(R, pt_);
      pb_ = m3_v(R, pb_);
      uw = m3_v(R, tau);
      cw = m3_v(R, cw);
      cv = m3_v(R, cv);
      A0w = sandwich(R, s6_of(ld9(T + T_A0)));
      mcw = vscale(m3_v(R, com), mass);
      const v3 dx = ld3(T + T_DEXT);
      const float *m = R.m;
      Dxw = {dx.x * m[0] * m[0] + dx.y * m[1] * m[1] + dx.z * m[2] * m[2],
             dx.x * m[3] * m[3] + dx.y * m[4] * m[4] + dx.z * m[5] * m[5],
             dx.x * m[6] * m[6] + dx.y * m[7] * m[7] + dx.z * m[8] * m[8],
             dx.x * m[0] * m[3] + dx.y * m[1] * m[4] + dx.z * m[2] * m[5],
             dx.x * m[0] * m[6] + dx.y * m[1] * m[7] + dx.z * m[2] * m[8],
             dx.x * m[3] * m[6] + dx.y * m[4] * m[7] + dx.z * m[5] * m[8]};
    }
    // articulated inertia [[A, B], [B^T, M]]: the body's own plus its children's contributions
    auto gather = [&](M3 &A, M3 &B, M3 &M) {
      const float mass = T[T_MASS];
      A = s6_full(A0w);
      B = m3_skew(mcw);
      M = {{mass, 0.0f, 0.0f, 0.0f, mass, 0.0f, 0.0f, 0.0f, mass}};
      for (int k = 0; k < nch; ++k) {
        const float *s = S[k == 0 ? ch0 : (k == 1 ? ch1 : ch2)];
        const M3 As = sym_full(s), Ms = sym_full(s + 15);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          A.m[i] += As.m[i];
          B.m[i] += s[6 + i];
          M.m[i] += Ms.m[i];
        }
        pt_ = vadd(pt_, ld3(s + 21));
        pb_ = vadd(pb_, ld3(s + 24));
      }
    };
    // ---- inward pass
    M3 oK, oL;  // this body's outward-pass operands (registers, see the LDS note above)
    v3 oy;
    for (int L = depth; L >= 1; --L) {
      if (level == L && !(PHC_PHYS_ABLATE & 4)) {
        M3 A, B, M;
        gather(A, B, M);
        M3 Ka, Lm;
        v3 y;
        {
          const M3 Dinv = m3_inv_sym(m3_add(A, s6_full(Dxw)));
          Ka = m3_mul(Dinv, A);
          Lm = m3_mul(Dinv, B);
          y = m3_v(Dinv, vsub(uw, pt_));
        }
        oK = Ka; oL = Lm; oy = y;
        // Ia = I^A - U D^-1 U^T, pa = pA + Ia c + U D^-1 u  (U = [A; B^T]); the A and M blocks are
        // symmetric, so only their upper triangles are formed
        const S6 Aa = s6_sub(s6_of(A), sym_mul(A, Ka));
        const M3 Ba = m3_sub(B, m3_mul(A, Lm));
        const S6 Ma = s6_sub(s6_of(M), sym_tmul(B, Lm));
        const v3 pat = vadd(vadd(pt_, vadd(m3_v(s6_full(Aa), cw), m3_v(Ba, cv))), m3_v(A, y));
        const v3 pab = vadd(vadd(pb_, vadd(m3_tv(Ba, cw), m3_v(s6_full(Ma), cv))), m3_tv(B, y));
        // to the parent's W frame: the shift by r = P - P_parent,
        // A_p = Aa - Ba [r]x + [r]x Ba^T - [r]x Ma [r]x, with [r]x Ba^T = -(Ba [r]x)^T
        const M3 RM = skew_mul(rw, s6_full(Ma));
        const M3 X = mul_skew(Ba, rw), Z = mul_skew(RM, rw);
        const S6 Ap = {Aa.xx - 2.0f * X.m[0] - Z.m[0], Aa.yy - 2.0f * X.m[4] - Z.m[4], Aa.zz - 2.0f * X.m[8] - Z.m[8],
                       Aa.xy - (X.m[1] + X.m[3]) - Z.m[1], Aa.xz - (X.m[2] + X.m[6]) - Z.m[2],
                       Aa.yz - (X.m[5] + X.m[7]) - Z.m[5]};
        const M3 Bp = m3_add(Ba, RM);
        const v3 Np = vadd(pat, cross3(rw, pab));
        float *s = S[b];
        store_s6(Ap, s);
#pragma unroll
        for (int i = 0; i < 9; ++i) s[6 + i] = Bp.m[i];
        store_s6(Ma, s + 15);
        s[21] = Np.x; s[22] = Np.y; s[23] = Np.z;
        s[24] = pab.x; s[25] = pab.y; s[26] = pab.z;
      }
      phys_sync();
    }
    // ---- floating root: a0 = -IA^-1 pA, IA = [[A, B], [B^T, M]], by 3x3 blocks on lane 0:
    // T = B M^-1, (A - T B^T) a_w = -pt + T pb, M a_v = -pb - B^T a_w (two closed-form symmetric
    // inverses: independent products instead of a 6x6 Cholesky's serial chain of square roots)
    v3 aw = {0.0f, 0.0f, 0.0f}, av = {0.0f, 0.0f, 0.0f};
    if (level == 0 && !(PHC_PHYS_ABLATE & 16)) {
      M3 A, B, M;
      gather(A, B, M);
      const M3 Mi = m3_inv_sym(M);
      const M3 Tm = m3_mul(B, Mi);
      const S6 Sc = s6_sub(s6_of(A), S6{row_row(Tm, 0, B, 0), row_row(Tm, 1, B, 1), row_row(Tm, 2, B, 2),
                                        row_row(Tm, 0, B, 1), row_row(Tm, 0, B, 2), row_row(Tm, 1, B, 2)});
      aw = m3_v(m3_inv_sym(s6_full(Sc)), vsub(m3_v(Tm, pb_), pt_));
      av = m3_v(Mi, vscale(vadd(pb_, m3_tv(B, aw)), -1.0f));
      float *s = S[0];
      s[0] = aw.x; s[1] = aw.y; s[2] = aw.z; s[3] = av.x; s[4] = av.y; s[5] = av.z;
    }
    phys_sync();
    // ---- outward pass: a' = X a_parent + c, qdd = y - K a'_w - L a'_v, a = a' + [qdd; 0]
    v3 qdd = {0.0f, 0.0f, 0.0f};
    for (int L = 1; L <= depth; ++L) {
      if (level == L && !(PHC_PHYS_ABLATE & 8)) {  // ablation builds only (timing breakdown)
        const float *ps = S[parent];
        const v3 apw = ld3(ps);
        aw = vadd(apw, cw);
        av = vadd(vsub(ld3(ps + 3), cross3(rw, apw)), cv);
        qdd = vsub(vsub(oy, m3_v(oK, aw)), m3_v(oL, av));  // W frame: R times the joint's qdd
        aw = vadd(aw, qdd);
        float *s = S[b];
        s[0] = aw.x; s[1] = aw.y; s[2] = aw.z; s[3] = av.x; s[4] = av.y; s[5] = av.z;
      }
      phys_sync();
    }
    // ---- semi-implicit Euler
    if (act && b > 0) {
      qdd = m3_tv(m3_quat(Q.x, Q.y, Q.z, Q.w), qdd);  // to joint (body) coordinates
      const v3 kp = ld3(T + T_KP), kd = ld3(T + T_KD);
      applied = {tau.x - dt * (kd.x + dt * kp.x) * qdd.x, tau.y - dt * (kd.y + dt * kp.y) * qdd.y,
                 tau.z - dt * (kd.z + dt * kp.z) * qdd.z};
      om = vadd(om, vscale(qdd, dt));
      const float wn2 = om.x * om.x + om.y * om.y + om.z * om.z;
      if (wn2 > c.max_w * c.max_w) om = vscale(om, c.max_w * rsqrtf(wn2));  // max_angular_velocity
      r = qnormalize(qmul_std(r, quat_exp_increment(vscale(om, dt))));
    } else if (act) {
      const M3 R0 = m3_quat(Q.x, Q.y, Q.z, Q.w);  // the root's acceleration, W frame -> body coordinates
      aw = m3_tv(R0, aw);
      av = m3_tv(R0, av);
      w0 = vadd(w0, vscale(aw, dt));
      const float wn2 = w0.x * w0.x + w0.y * w0.y + w0.z * w0.z;
      if (wn2 > c.max_w * c.max_w) w0 = vscale(w0, c.max_w * rsqrtf(wn2));
      v0 = vadd(v0, vscale(av, dt));
      p0 = vadd(p0, vscale(m3_v(R0, v0), dt));
      q0 = qnormalize(qmul_std(q0, quat_exp_increment(vscale(w0, dt))));
    }
  }
  kinematics();
  if (act) {  // no barrier follows
    const M3 R = m3_quat(Q.x, Q.y, Q.z, Q.w);
    // the centre of mass's linear velocity (PhysX's rigid-body velocity): v + w x com
    const v3 vw = m3_v(R, vadd(v, cross3(w, ld3(T + T_COM)))), ww = m3_v(R, w);
    float *o = e.rb + (env * kBodies + b) * kRec;
    o[0] = P.x; o[1] = P.y; o[2] = P.z;
    o[3] = Q.x; o[4] = Q.y; o[5] = Q.z; o[6] = Q.w;
    o[7] = vw.x; o[8] = vw.y; o[9] = vw.z;
    o[10] = ww.x; o[11] = ww.y; o[12] = ww.z;
    if (b == 0 && e.root) {
      float *rt = e.root + env * kRec;
#pragma unroll
      for (int k = 0; k < kRec; ++k) rt[k] = o[k];
    }
  }
  if (act && b > 0) {
    const v3 ej = rotvec_of(r);
    float *d = e.dof_state + (env * PHC_NUM_DOF + 3 * (b - 1)) * 2;
    d[0] = ej.x; d[1] = om.x; d[2] = ej.y; d[3] = om.y; d[4] = ej.z; d[5] = om.z;
    float *f = e.dof_force + env * PHC_NUM_DOF + 3 * (b - 1);
    f[0] = applied.x; f[1] = applied.y; f[2] = applied.z;
  }
  launch_clock_end(c.clk);
}

}  // namespace phc

using namespace phc;

static int physics_launch(const phc_env_buffers *env, const float *pd_target, const phc_pd_map *pd,
                          const float *body_model, const phc_physics_params *p, phc_kernel_timer *timer,
                          void *stream) {
  PHC_REQUIRE(env && env->num_envs > 0, "physics_step: num_envs must be > 0");
  PHC_REQUIRE(env->rigid_body_state && env->dof_state && env->dof_force, "physics_step: null env buffer");
  PHC_REQUIRE((pd_target || pd) && body_model && p, "physics_step: null target / model / params");
  PHC_REQUIRE(!pd || (pd->actions && pd->pd_target && pd->offset && pd->scale), "physics_step: bad pd map");
  PHC_REQUIRE(p->sim_dt > 0.0f && p->control_freq_inv >= 1 && p->substeps >= 1 && p->substeps <= 1024 &&
                  p->control_freq_inv <= 64,
              "physics_step: bad time stepping (sim_dt %g, control_freq_inv %d, substeps %d)", (double)p->sim_dt,
              p->control_freq_inv, p->substeps);
  PHC_REQUIRE(p->tree_depth >= 1 && p->tree_depth <= 15, "physics_step: tree_depth must be 1..15");
  PHC_REQUIRE(p->contact_stiffness >= 0.0f && p->contact_damping >= 0.0f && p->friction >= 0.0f &&
                  p->friction_damping >= 0.0f && p->angular_damping >= 0.0f && p->max_angular_velocity >= 0.0f,
              "physics_step: contact / damping coefficients must be >= 0");
  PhysConsts c;
  c.dt = p->sim_dt / (float)p->substeps;
  c.nsub = p->control_freq_inv * p->substeps;
  c.depth = p->tree_depth;
  c.kp_scale = p->kp_scale;
  c.kd_scale = p->kd_scale;
  c.kn = p->contact_stiffness;
  c.cn = p->contact_damping;
  c.mu = p->friction;
  c.ct = p->friction_damping;
  c.g = p->gravity;
  c.ang_damp = p->angular_damping;
  c.max_w = p->max_angular_velocity > 0.0f ? p->max_angular_velocity : 3.0e38f;
  c.self_col = p->self_collision;
  const PhysView v = {env->num_envs, env->rigid_body_state, env->root_state, env->dof_state,
                       const_cast<float *>(env->dof_force)};  // read-only for the env step, written here
  const int64_t blocks = (env->num_envs + kPhysEnvs - 1) / kPhysEnvs;
  c.clk = phc_timer_take(timer, as_stream(stream), blocks, (double)env->num_envs);  // work: env-steps
  const PdArgs pa{pd ? pd->actions : nullptr, pd ? pd->pd_target : nullptr, pd ? pd->offset : nullptr,
                  pd ? pd->scale : nullptr, pd ? pd->frozen : nullptr, pd ? pd->clip : 1};
  phc_launch(k_physics_step, dim3((unsigned)blocks), dim3(kPhysBlock), 0, as_stream(stream), v,
                        body_model, pd_target, pa, c);
  return check_launch("physics_step");
}

extern "C" int phc_physics_step_timed(const phc_env_buffers *env, const float *pd_target, const float *body_model,
                                      const phc_physics_params *p, phc_kernel_timer *timer, void *stream) {
  return physics_launch(env, pd_target, nullptr, body_model, p, timer, stream);
}

extern "C" int phc_physics_step_actions(const phc_env_buffers *env, const phc_pd_map *pd, const float *body_model,
                                        const phc_physics_params *p, phc_kernel_timer *timer, void *stream) {
  PHC_REQUIRE(pd, "physics_step_actions: null pd map");
  return physics_launch(env, nullptr, pd, body_model, p, timer, stream);
}

extern "C" int phc_physics_step(const phc_env_buffers *env, const float *pd_target, const float *body_model,
                                const phc_physics_params *p, void *stream) {
  return phc_physics_step_timed(env, pd_target, body_model, p, nullptr, stream);
}
