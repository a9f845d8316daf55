// phc_common.h — shared host/device plumbing of libphc_hip.so.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#include "phc.h"
#include "phc_quat.h"

namespace phc {

// The logistic sigmoid of the LayerNorm + SiLU tails (policy tail, PPO-minibatch tail, the module path's
// twin LayerNorm): PHC_FAST_SILU = 1 evaluates it from the hardware exp2 / reciprocal (1-ulp class, as the
// trunk GEMMs' fused SiLU epilogues do); 0 = expf and an IEEE division (torch's formula, ~3x the VALU work
// of these VALU-bound kernels).
#ifndef PHC_FAST_SILU
#define PHC_FAST_SILU 1
#endif
__device__ __forceinline__ float tail_sigmoid(float x) {
#if PHC_FAST_SILU
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * 1.44269504088896341f));
#else
  return 1.0f / (1.0f + expf(-x));
#endif
}
__device__ __forceinline__ float tail_silu(float x) {
#if PHC_FAST_SILU
  return x * tail_sigmoid(x);
#else
  return x / (1.0f + expf(-x));
#endif
}


// thread-local message of the last failing call (phc_last_error)
void set_error(const char *fmt, ...);
int check_launch(const char *what);

#define PHC_REQUIRE(cond, ...)        \
  do {                                \
    if (!(cond)) {                    \
      ::phc::set_error(__VA_ARGS__);  \
      return PHC_EINVAL;              \
    }                                 \
  } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace phc

// Measurement timer (phc_timer_*): a timed launch stamps itself.  Each timed launch gets a slot in the
// timer's device buffer, [2 * grid] words: word w = the start of workgroup w, word grid + w = its end
// (after every wave of it has drained its memory operations), both read from s_memrealtime (the
// constant-rate clock every CU reads alike, hipDeviceAttributeWallClockRate).  The launch's duration is
// the latest end minus the earliest start.  Plain stores, one word per workgroup each: no atomics (2,048
// waves adding to one word serialised at the memory side and lengthened a timed env step by 16 us).
// Unlike start / stop events (hipExtLaunchKernel) this works inside a captured hipGraph (events recorded
// during a capture cannot be timed on ROCm 7.2: tools/graph_timer_probe.py) and leaves the stream no idle
// time around the launch; a slot captured into a graph holds its LAST replay.
struct phc_kernel_timer {
  struct Slot {
    int64_t off;                   // first word of the slot
    int32_t grid;                  // workgroups of the launch
    bool graph;                    // taken while its stream was capturing: re-stamped by every replay
    double work;                   // the launch's algorithmic work (bytes or FLOPs)
    unsigned long long end_at_reset;
  };
  unsigned long long *dev = nullptr;
  int64_t cap_words = 0, used_words = 0;
  int32_t capacity = 0;            // slots
  std::vector<Slot> slots;
  size_t base = 0;                 // slots taken before the last reset (graph slots among them still count)
  int32_t period = 1;              // stamp every period-th launch offered (phc_timer_set_period)
  int64_t seen = 0;                // launches offered since the last reset
  double tick_hz = 1.0e8;
};

// The slot for this launch when the timer samples it (every period-th launch offered, while space
// lasts), else null: the kernel then stamps nothing.
inline unsigned long long *phc_timer_take(phc_kernel_timer *t, hipStream_t st, int64_t grid, double work) {
  if (!t || grid <= 0) return nullptr;
  if (t->seen++ % t->period != 0) return nullptr;
  if ((int32_t)t->slots.size() >= t->capacity || t->used_words + 2 * grid > t->cap_words) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool graph = hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
  phc_kernel_timer::Slot s{t->used_words, (int32_t)grid, graph, work, 0ull};
  t->slots.push_back(s);
  t->used_words += 2 * grid;
  return t->dev + s.off;
}

template <typename F, typename... Args>
inline void phc_launch(F kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, Args... args) {
  hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
}

#ifdef __HIPCC__
// kernel side of the timer: every workgroup stamps its start, and its end once all of its waves have
// drained their memory operations; clk null = untimed launch (uniform branches; every thread of the
// workgroup must reach launch_clock_end)
__device__ __forceinline__ void launch_clock_begin(unsigned long long *clk) {
  if (clk && threadIdx.x == 0) {
    const unsigned wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    clk[wg] = __builtin_amdgcn_s_memrealtime();
  }
}
__device__ __forceinline__ void launch_clock_end(unsigned long long *clk) {
  if (clk) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned g = gridDim.x * gridDim.y * gridDim.z;
      const unsigned wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
      clk[g + wg] = __builtin_amdgcn_s_memrealtime();
    }
  }
}
#endif

namespace phc {

constexpr int kBodies = PHC_NUM_BODIES;
constexpr int kRec = PHC_BODY_STRIDE;  // floats per rigid-body record
constexpr int kObs = PHC_OBS_DIM;
constexpr int kGroup = 32;             // lanes per env: one lane per body, 24 of 32 active
constexpr int kBlock = 256;            // 4 waves, 8 envs per workgroup
constexpr int kEnvsPerBlock = kBlock / kGroup;

// ---------------------------------------------------------------- records --
struct BodyRec {
  v3 p;
  q4 r;
  v3 v;
  v3 av;
};

__device__ __forceinline__ BodyRec load_body(const float *__restrict__ q) {
  BodyRec b;
  b.p = {q[0], q[1], q[2]};
  b.r = {q[3], q[4], q[5], q[6]};
  b.v = {q[7], q[8], q[9]};
  b.av = {q[10], q[11], q[12]};
  return b;
}

__device__ __forceinline__ void store_body(float *__restrict__ q, const BodyRec &b) {
  q[0] = b.p.x; q[1] = b.p.y; q[2] = b.p.z;
  q[3] = b.r.x; q[4] = b.r.y; q[5] = b.r.z; q[6] = b.r.w;
  q[7] = b.v.x; q[8] = b.v.y; q[9] = b.v.z;
  q[10] = b.av.x; q[11] = b.av.y; q[12] = b.av.z;
}

// ------------------------------------------------- motion lib (device view) --
struct LibView {
  const float *frames;
  const float *local_rot;
  const float *dof_vel;
  const float *motion_len;
  const float *motion_dt;
  const int64_t *num_frames;
  const int64_t *length_starts;
};

inline LibView lib_view(const phc_motion_lib *l) {
  return {l->frames, l->local_rot, l->dof_vel, l->motion_len, l->motion_dt, l->num_frames, l->length_starts};
}

struct MotionScalars {
  float len, dt;
  int64_t nf, start;
};

__device__ __forceinline__ MotionScalars load_motion(const LibView &l, int64_t mid) {
  return {l.motion_len[mid], l.motion_dt[mid], l.num_frames[mid], l.length_starts[mid]};
}

struct Blend {
  int64_t f0, f1;  // absolute (flat) frame rows
  float b;
};

__device__ __forceinline__ float clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

// Cross-lane hand-off through a wave's own LDS region: a lane reads what other lanes of the same wave
// wrote (or overwrites what they read).  The LDS instructions of one wave execute in issue order, so
// only the compiler could break the hand-off by moving a ds_read / ds_write across it (the two sides
// touch different addresses per lane, so nothing else orders them): a wavefront-scope fence plus the
// wave barrier pin the issue order.  No instruction is emitted.
__device__ __forceinline__ void wave_lds_handoff() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// motion_lib.py:655-665 _calc_frame_blend (bit-exact with -ffp-contract=off)
__device__ __forceinline__ Blend frame_blend(float time, const MotionScalars &m) {
  float phase = clamp01(time / m.len);
  if (time < 0.0f) time = 0.0f;
  const int64_t f0 = (int64_t)(phase * (float)(m.nf - 1));
  const int64_t f1 = f0 + 1 < m.nf - 1 ? f0 + 1 : m.nf - 1;
  const float b = clamp01((time - (float)f0 * m.dt) / m.dt);
  return {m.start + f0, m.start + f1, b};
}

// motion_lib.py:597-610: lerp of pos (+offset) / vel / ang vel, slerp of global rotation, from
// the two raw frame records of this body
__device__ __forceinline__ BodyRec blend_body(const BodyRec &a, const BodyRec &c, float t, const v3 *offset) {
  const float s = 1.0f - t;
  BodyRec o;
  o.p = {s * a.p.x + t * c.p.x, s * a.p.y + t * c.p.y, s * a.p.z + t * c.p.z};
  if (offset) o.p = vadd(o.p, *offset);
  o.v = {s * a.v.x + t * c.v.x, s * a.v.y + t * c.v.y, s * a.v.z + t * c.v.z};
  o.av = {s * a.av.x + t * c.av.x, s * a.av.y + t * c.av.y, s * a.av.z + t * c.av.z};
  o.r = slerp(a.r, c.r, t);
  return o;
}

struct RowPair {
  BodyRec a, c;
};

__device__ __forceinline__ RowPair load_rows(const float *__restrict__ frames, const Blend &bl, int body) {
  return {load_body(frames + (bl.f0 * kBodies + body) * kRec), load_body(frames + (bl.f1 * kBodies + body) * kRec)};
}

__device__ __forceinline__ BodyRec ref_body(const float *__restrict__ frames, const Blend &bl, int body,
                                            const v3 *offset) {
  const RowPair r = load_rows(frames, bl, body);
  return blend_body(r.a, r.c, bl.b, offset);
}

// dof_pos of body `body` (>=1): exp map of slerped local rotation (motion_lib.py:605-606, 670-673)
__device__ __forceinline__ v3 ref_dof_pos(const float *__restrict__ lrs, const Blend &bl, int body) {
  const float *a = lrs + (bl.f0 * kBodies + body) * 4;
  const float *c = lrs + (bl.f1 * kBodies + body) * 4;
  const q4 r = slerp(q4{a[0], a[1], a[2], a[3]}, q4{c[0], c[1], c[2], c[3]}, bl.b);
  return quat_to_exp_map(r);
}

// dof_vel of body `body` (>=1): lerp of dvs rows (motion_lib.py:603)
__device__ __forceinline__ v3 ref_dof_vel(const float *__restrict__ dvs, const Blend &bl, int body) {
  const float *a = dvs + (bl.f0 * (kBodies - 1) + (body - 1)) * 3;
  const float *c = dvs + (bl.f1 * (kBodies - 1) + (body - 1)) * 3;
  const float t = bl.b, s = 1.0f - t;
  return {s * a[0] + t * c[0], s * a[1] + t * c[1], s * a[2] + t * c[2]};
}

// -------------------------------------------------------------- group ops --
// On the 32-lane half-waves with one LDS-crossbar operation instead of five ds_bpermute round trips
// (each waited on before the next): the sum is the xor butterfly 16, 8, 4, 2, 1, its xor-16 step one
// ds_swizzle (bitmask mode: lane ^ 16 within each 32-lane group, no LDS memory access), its xor-8 / 4 /
// 2 / 1 steps DPP row rotations (once lanes i and i ^ 16 (then ^ 8, ...) hold equal values, a rotation
// by 8, 4, 2, 1 within the 16-lane row reads a lane holding the xor partner's value).  Every lane adds
// the same two values at every level (own + partner; IEEE addition commutes), so the result is the
// __shfl_xor butterfly's bit for bit and the same in all 32 lanes.  Requires every lane of the wave
// active (uniform control flow).  (v_permlane16_swap would do the xor-16 step in the VALU, but this
// compiler folds its two results into one register.)
template <int N> __device__ __forceinline__ float row_ror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + N, 0xF, 0xF, false));
}
__device__ __forceinline__ float group_sum(float v) {
  static_assert(kGroup == 32, "half-wave groups");
  constexpr int kXor16 = (0x10 << 10) | 0x1F;  // ds_swizzle bitmask mode: and 0x1F, or 0, xor 0x10
  v = v + __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), kXor16));
  v = v + row_ror<8>(v);
  v = v + row_ror<4>(v);
  v = v + row_ror<2>(v);
  v = v + row_ror<1>(v);
  return v;
}
// lane 0's value in lanes 0-31, lane 32's in lanes 32-63 (scalar reads: no LDS round trip)
__device__ __forceinline__ float group_bcast(float v) {
  const int a = __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0);
  const int b = __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32);
  return __builtin_bit_cast(float, (__lane_id() & 32) ? b : a);
}
// the next lane's value (lane i gets lane i + 1 across the whole wave: DPP wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ float next_lane(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
}

// ------------------------------------------------------------ observation --
// One body's slices of the 934-float observation (common.py:23-103 self obs with
// local_root_obs/root_height_obs/upright; common.py:107-176 imitation obs v6, time_steps 1).
// The heading rotations use the exact specialisations of phc_quat.h (rot_heading,
// qmul_heading_*, tan_norm_fast): same float32 values as the generic formulas (only the sign
// of some exact zeros can differ; checked over 40 steps x 2048 envs with tools/ab_compare.py).
// self observation slices of body b (common.py:23-103)
__device__ __forceinline__ void write_self_obs(float *__restrict__ o, int b, const BodyRec &s, v3 root_p,
                                               const Heading &hinv) {
  float t6[6];
  if (b == 0) {
    o[0] = root_p.z;
  } else {
    const v3 lp = rot_heading(hinv, vsub(s.p, root_p));
    float *d = o + 1 + 3 * (b - 1);
    d[0] = lp.x; d[1] = lp.y; d[2] = lp.z;
  }
  tan_norm_fast(qmul_heading_left(hinv, s.r), t6);
#pragma unroll
  for (int k = 0; k < 6; ++k) o[70 + 6 * b + k] = t6[k];
  v3 x = rot_heading(hinv, s.v);
  o[214 + 3 * b] = x.x; o[215 + 3 * b] = x.y; o[216 + 3 * b] = x.z;
  x = rot_heading(hinv, s.av);
  o[286 + 3 * b] = x.x; o[287 + 3 * b] = x.y; o[288 + 3 * b] = x.z;
}

// imitation (task) observation slices of body b (common.py:107-176, v6, one time step)
__device__ __forceinline__ void write_task_obs(float *__restrict__ o, int b, const BodyRec &s, v3 root_p,
                                               const Heading &hinv, const Heading &hrot, const BodyRec &ref) {
  float t6[6];
  v3 x = rot_heading(hinv, vsub(ref.p, s.p));
  o[358 + 3 * b] = x.x; o[359 + 3 * b] = x.y; o[360 + 3 * b] = x.z;
  tan_norm_fast(qmul_heading_right(qmul_heading_left(hinv, quat_mul(ref.r, quat_conj(s.r))), hrot), t6);
#pragma unroll
  for (int k = 0; k < 6; ++k) o[430 + 6 * b + k] = t6[k];
  x = rot_heading(hinv, vsub(ref.v, s.v));
  o[574 + 3 * b] = x.x; o[575 + 3 * b] = x.y; o[576 + 3 * b] = x.z;
  x = rot_heading(hinv, vsub(ref.av, s.av));
  o[646 + 3 * b] = x.x; o[647 + 3 * b] = x.y; o[648 + 3 * b] = x.z;
  x = rot_heading(hinv, vsub(ref.p, root_p));
  o[718 + 3 * b] = x.x; o[719 + 3 * b] = x.y; o[720 + 3 * b] = x.z;
  tan_norm_fast(qmul_heading_left(hinv, ref.r), t6);
#pragma unroll
  for (int k = 0; k < 6; ++k) o[790 + 6 * b + k] = t6[k];
}

__device__ __forceinline__ void write_obs_body(float *__restrict__ o, int b, const BodyRec &s, v3 root_p,
                                               const Heading &hinv, const Heading &hrot, const BodyRec &ref) {
  write_self_obs(o, b, s, root_p, hinv);
  write_task_obs(o, b, s, root_p, hinv, hrot, ref);
}

// column sums of the [rows, cols] fp32 partials (bias gradients; a template so every
// translation unit that launches it carries its own copy): 16 lanes x float4 = 64 columns per block, 16 row
// slices reduced through LDS
template <int = 0>
__global__ __launch_bounds__(256) void k_colsum(const float *__restrict__ partial, int rows, int cols,
                                                float *__restrict__ out) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, rs = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cl * 4;
  float4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  if (c < cols) {
#pragma unroll 4
    for (int r = rs; r < rows; r += 16) {
      const float4 v = *reinterpret_cast<const float4 *>(partial + (int64_t)r * cols + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[rs][cl] = acc;
  __syncthreads();
  if (rs == 0 && c < cols) {
    float4 t = red[0][cl];
    for (int k = 1; k < 16; ++k) {
      const float4 v = red[k][cl];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    *reinterpret_cast<float4 *>(out + c) = t;
  }
}

}  // namespace phc
