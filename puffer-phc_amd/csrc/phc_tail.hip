// phc_tail.hip — the row-wise part of the PPO minibatch tail after the twin trunks (R19, R21).
//
// What the reference runs between the trunks' last Linear and the mu / value heads (per
// minibatch, policies/phc_policy.py:16-61 under autograd: LayerNorm + SiLU of each trunk, the
// critic's 512 -> 1 value head; clean_pufferl/core.py:298-352 backward through them) as one
// kernel each way, around the fp32 mu-head GEMMs and the PPO objective kernels (phc_ppo.hip):
//
// k_tail_ln_fwd: per row, LayerNorm + SiLU of both trunks (one wave per row and trunk, the
//   arithmetic of phc_policy_act); the actor's h_a is written for the mu GEMM (and its weight
//   gradient), the critic's h_c is reduced on the spot into value = w_v h_c + b_v.
// k_tail_ln_bwd (persistent, one 512-thread block per CU): per row, d h_c = dvalue w_v and
//   d h_a (from the dmu W_mu GEMM) through SiLU and LayerNorm backward (recomputed from y);
//   dy is written once in the half-precision operand type of the trunk backward (the SiLU-
//   gradient GEMMs read it directly) and every column sum the tail needs — both LayerNorms'
//   gamma / beta gradients, the last trunk layer's bias gradient (sums of dy in fp32), w_v and
//   b_v, b_mu (sums of dmu) — accumulates in the lanes' registers across the block's rows: one
//   partial row per block.
// That replaces the LayerNorm kernels, the value-head GEMMs, the activation-backward + bias-
// gradient kernel and the ~25 fill / copy / add / reduction launches autograd ran between them.
#include "phc_common.h"

namespace phc {

constexpr int kTH = 512;        // hidden width
constexpr int kTC = kTH / 256;  // float4 chunks per lane in a row
constexpr int kTA = 72;         // max actions (b_mu sums: two per lane)
#ifndef PHC_TAIL_FWD_ROWS
#define PHC_TAIL_FWD_ROWS 4
#endif
constexpr int kFwdThreads = 256, kFwdRows = PHC_TAIL_FWD_ROWS;  // forward: 4 waves, 4 rows (8 row tasks)
constexpr int kBwdThreads = 512;                // backward: 8 waves, persistent

__device__ __forceinline__ float t_wave_sum(float s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// row statistics of one H-wide row held per lane (lane-strided float4 chunks), as ln_silu_row
struct LnStat {
  float mean, rstd;
};
__device__ __forceinline__ LnStat t_ln_stat(const float x[kTC][4], float eps) {
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < kTC; ++k) s += (x[k][0] + x[k][1]) + (x[k][2] + x[k][3]);
  const float mean = t_wave_sum(s) / (float)kTH;
  float v = 0.0f;
#pragma unroll
  for (int k = 0; k < kTC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = x[k][e] - mean;
      v += d * d;
    }
  return {mean, rsqrtf(t_wave_sum(v) / (float)kTH + eps)};
}

__device__ __forceinline__ int t_col(int lane, int k, int e) { return 4 * (lane + 64 * k) + e; }

__device__ __forceinline__ void t_load_row(const float *src, int lane, float x[kTC][4]) {
#pragma unroll
  for (int k = 0; k < kTC; ++k) {
    const float4 v = *reinterpret_cast<const float4 *>(src + 4 * (lane + 64 * k));
    x[k][0] = v.x; x[k][1] = v.y; x[k][2] = v.z; x[k][3] = v.w;
  }
}

// gamma / beta / w_v may be views into a flat parameter buffer: 4-byte aligned only
__device__ __forceinline__ void t_load_param(const float *p, int lane, float x[kTC][4]) {
#pragma unroll
  for (int k = 0; k < kTC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) x[k][e] = p[t_col(lane, k, e)];
}

// partial row layout (floats) of one backward block, shared with the host (phc_tail_layout)
struct TailLayout {
  int bmu, wv, bv, gamma, beta, b6, stride;
};
__host__ __device__ inline int t_align4(int x) { return (x + 3) & ~3; }
__host__ __device__ inline TailLayout tail_layout(int a, int h) {
  TailLayout l;
  l.bmu = 0;
  l.wv = t_align4(a);
  l.bv = l.wv + h;
  l.gamma = t_align4(l.bv + 1);  // [2][h]: actor, critic
  l.beta = l.gamma + 2 * h;
  l.b6 = l.beta + 2 * h;          // [2][h]: last trunk layer bias (actor, critic)
  l.stride = t_align4(l.b6 + 2 * h);
  return l;
}

// ---------------------------------------------------------------- forward --
__global__ __launch_bounds__(kFwdThreads) void k_tail_ln_fwd(phc_tail_ln_args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kWaves = kFwdThreads / 64, kTasks = 2 * kFwdRows / kWaves;
  const int64_t r0 = (int64_t)blockIdx.x * kFwdRows, M = a.rows;
  float x[kTasks][kTC][4];
#pragma unroll
  for (int t = 0; t < kTasks; ++t) {  // task q = (trunk q % 2, row q / 2): loads first
    const int q = wave + kWaves * t;
    const int64_t row = r0 + q / 2;
    if (row < M) t_load_row(a.trunk_out + ((int64_t)(q % 2) * M + row) * kTH, lane, x[t]);
  }
  // task q = wave + kWaves t belongs to trunk q % 2 = wave % 2 (kWaves even): one parameter load
  // per wave, before any store (the stores of h_actor could alias the parameter views)
  static_assert(kWaves % 2 == 0, "a wave's tasks share one trunk");
  const int grp = wave % 2;
  float gm[kTC][4], bt[kTC][4], wv[kTC][4];
  t_load_param(a.ln_gamma[grp], lane, gm);
  t_load_param(a.ln_beta[grp], lane, bt);
  if (grp == 1) t_load_param(a.w_value, lane, wv);
  const float bv = grp == 1 ? a.b_value[0] : 0.0f;
#pragma unroll
  for (int t = 0; t < kTasks; ++t) {
    const int q = wave + kWaves * t;
    const int64_t row = r0 + q / 2;
    if (row >= M) continue;
    const LnStat st = t_ln_stat(x[t], a.ln_eps);
    float h[kTC][4];
#pragma unroll
    for (int k = 0; k < kTC; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float ln = (x[t][k][e] - st.mean) * st.rstd * gm[k][e] + bt[k][e];
        h[k][e] = tail_silu(ln);
      }
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < kTC; ++k)
        *reinterpret_cast<float4 *>(a.h_actor + row * kTH + 4 * (lane + 64 * k)) =
            float4{h[k][0], h[k][1], h[k][2], h[k][3]};
    } else {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < kTC; ++k)
        s += h[k][0] * wv[k][0] + h[k][1] * wv[k][1] + h[k][2] * wv[k][2] + h[k][3] * wv[k][3];
      s = t_wave_sum(s);
      if (lane == 0) a.value[row] = s + bv;
    }
  }
}

// --------------------------------------------------------------- backward --
// LayerNorm + SiLU backward of one row held per lane (k_ln_silu_bwd's arithmetic): dh is the
// gradient of the SiLU output (critic: dh = dvalue * w_v with d w_v += dvalue * silu(ln));
// accumulates the gamma / beta / output-bias column sums of the lane's 8 columns, writes dy (T)
template <typename T, bool CRITIC>
__device__ __forceinline__ void t_ln_bwd_row(const float x[kTC][4], const float dh[kTC][4], const float gm[kTC][4],
                                             const float bt[kTC][4], float eps, float dvalue, int lane, T *dst,
                                             float pg[kTC][4], float pb[kTC][4], float p6[kTC][4],
                                             float pwv[kTC][4]) {
  const LnStat st = t_ln_stat(x, eps);
  float xh[kTC][4], dx[kTC][4];
  float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
  for (int k = 0; k < kTC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xv = (x[k][e] - st.mean) * st.rstd;
      const float ln = xv * gm[k][e] + bt[k][e];
      const float sg = tail_sigmoid(ln);
      float d = dh[k][e];
      if constexpr (CRITIC) {
        pwv[k][e] += dvalue * (ln * sg);
        d = dvalue * d;
      }
      const float dln = d * sg * (1.0f + ln * (1.0f - sg));
      pg[k][e] += dln * xv;
      pb[k][e] += dln;
      const float dd = dln * gm[k][e];
      s1 += dd;
      s2 += dd * xv;
      xh[k][e] = xv;
      dx[k][e] = dd;
    }
  s1 = t_wave_sum(s1);
  s2 = t_wave_sum(s2);
  const float m1 = s1 / (float)kTH, m2 = s2 / (float)kTH;
#pragma unroll
  for (int k = 0; k < kTC; ++k) {
    T o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = st.rstd * (dx[k][e] - m1 - xh[k][e] * m2);
      p6[k][e] += v;
      o[e] = (T)v;
    }
    uint2 raw;
    __builtin_memcpy(&raw, o, sizeof(raw));
    *reinterpret_cast<uint2 *>(dst + 4 * (lane + 64 * k)) = raw;
  }
}

template <typename T>
__global__ __launch_bounds__(kBwdThreads) void k_tail_ln_bwd(phc_tail_ln_args a, const float *__restrict__ dh_actor,
                                                            const float *__restrict__ dmu,
                                                            const float *__restrict__ dvalue, int A,
                                                            T *__restrict__ dy, float *__restrict__ partial) {
  constexpr int kWaves = kBwdThreads / 64;
  __shared__ __attribute__((aligned(16))) float red[4][kWaves][kTH];  // 64 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t M = a.rows;
  float gm[2][kTC][4], bt[2][kTC][4], wv[kTC][4];
  t_load_param(a.ln_gamma[0], lane, gm[0]);
  t_load_param(a.ln_gamma[1], lane, gm[1]);
  t_load_param(a.ln_beta[0], lane, bt[0]);
  t_load_param(a.ln_beta[1], lane, bt[1]);
  t_load_param(a.w_value, lane, wv);
  float pg[2][kTC][4], pb[2][kTC][4], p6[2][kTC][4], pwv[kTC][4];
#pragma unroll
  for (int k = 0; k < kTC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pg[0][k][e] = pg[1][k][e] = pb[0][k][e] = pb[1][k][e] = 0.0f;
      p6[0][k][e] = p6[1][k][e] = pwv[k][e] = 0.0f;
    }
  float pbmu0 = 0.0f, pbmu1 = 0.0f, pbv = 0.0f;
  // one row (both trunks) per wave at a time; the wave's next row is loaded while this one is
  // processed (its loads land during the reductions), dmu through clamped loads masked after
  struct RowIn {
    float xa[kTC][4], xc[kTC][4], da[kTC][4];
    float dv, m0, m1;
  };
  const int l0 = lane < A ? lane : A - 1, l1 = lane + 64 < A ? lane + 64 : A - 1;
  auto fetch = [&](int64_t r, RowIn &in) {
    t_load_row(a.trunk_out + r * kTH, lane, in.xa);
    t_load_row(a.trunk_out + (M + r) * kTH, lane, in.xc);
    t_load_row(dh_actor + r * kTH, lane, in.da);
    in.dv = dvalue[r];
    in.m0 = dmu[r * A + l0];
    in.m1 = dmu[r * A + l1];
  };
  const int64_t step = (int64_t)gridDim.x * kWaves;
  int64_t row = (int64_t)blockIdx.x * kWaves + wave;
  RowIn cur;
  if (row < M) fetch(row, cur);
  for (; row < M; row += step) {
    RowIn nxt;
    if (row + step < M) fetch(row + step, nxt);
    pbmu0 += lane < A ? cur.m0 : 0.0f;
    pbmu1 += lane + 64 < A ? cur.m1 : 0.0f;
    pbv += cur.dv;
    t_ln_bwd_row<T, false>(cur.xa, cur.da, gm[0], bt[0], a.ln_eps, 0.0f, lane, dy + row * kTH, pg[0], pb[0], p6[0],
                           pwv);
    t_ln_bwd_row<T, true>(cur.xc, wv, gm[1], bt[1], a.ln_eps, cur.dv, lane, dy + (M + row) * kTH, pg[1], pb[1], p6[1],
                          pwv);
    cur = nxt;
  }
  // the block's partial row (tail_layout): the 8 waves' column sums added through LDS in order
  const TailLayout L = tail_layout(A, kTH);
  float *pr = partial + (int64_t)blockIdx.x * L.stride;
  auto put = [&](int slot, const float v[kTC][4]) {
#pragma unroll
    for (int k = 0; k < kTC; ++k)
      *reinterpret_cast<float4 *>(&red[slot][wave][4 * (lane + 64 * k)]) = float4{v[k][0], v[k][1], v[k][2], v[k][3]};
  };
  auto take = [&](int slot, float *dst) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += red[slot][w][tid];
    dst[tid] = s;
  };
  put(0, pg[0]); put(1, pg[1]); put(2, pb[0]); put(3, pb[1]);
  __syncthreads();
  take(0, pr + L.gamma); take(1, pr + L.gamma + kTH); take(2, pr + L.beta); take(3, pr + L.beta + kTH);
  __syncthreads();
  put(0, p6[0]); put(1, p6[1]); put(2, pwv);
  red[3][wave][lane] = pbmu0;
  red[3][wave][64 + lane] = pbmu1;
  if (lane == 0) red[3][wave][128] = pbv;
  __syncthreads();
  take(0, pr + L.b6); take(1, pr + L.b6 + kTH); take(2, pr + L.wv);
  if (tid < A || tid == 128) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += red[3][w][tid];
    if (tid < A) pr[L.bmu + tid] = s;
    else pr[L.bv] = s;
  }
}

}  // namespace phc

using namespace phc;

extern "C" int phc_tail_layout(int32_t num_actions, int32_t hidden, int32_t *offsets) {
  PHC_REQUIRE(offsets, "tail_layout: null offsets");
  const TailLayout l = tail_layout(num_actions, hidden);
  const int v[7] = {l.bmu, l.wv, l.bv, l.gamma, l.beta, l.b6, l.stride};
  for (int i = 0; i < 7; ++i) offsets[i] = v[i];
  return PHC_OK;
}

extern "C" int32_t phc_tail_blocks(int64_t rows) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t need = (rows + kBwdThreads / 64 - 1) / (kBwdThreads / 64);
  return (int32_t)(need < cus ? need : cus);
}

static int check_tail(const phc_tail_ln_args *a) {
  PHC_REQUIRE(a, "tail_ln: null args");
  PHC_REQUIRE(a->trunk_out && a->ln_gamma[0] && a->ln_gamma[1] && a->ln_beta[0] && a->ln_beta[1] && a->w_value &&
                  a->b_value,
              "tail_ln: null argument");
  PHC_REQUIRE(a->rows > 0, "tail_ln: empty minibatch");
  PHC_REQUIRE(a->hidden == kTH, "tail_ln: hidden must be %d", kTH);
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(a->trunk_out) & 15) == 0, "tail_ln: trunk_out must be 16-byte aligned");
  return PHC_OK;
}

extern "C" int phc_tail_ln_fwd(const phc_tail_ln_args *args, void *stream) {
  if (int rc = check_tail(args)) return rc;
  PHC_REQUIRE(args->h_actor && args->value, "tail_ln_fwd: null h_actor / value");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(args->h_actor) & 15) == 0, "tail_ln_fwd: h_actor must be 16-byte aligned");
  const int64_t blocks = (args->rows + kFwdRows - 1) / kFwdRows;
  hipLaunchKernelGGL(k_tail_ln_fwd, dim3((unsigned)blocks), dim3(kFwdThreads), 0, as_stream(stream), *args);
  return check_launch("tail_ln_fwd");
}

extern "C" int phc_tail_ln_bwd(const phc_tail_ln_args *args, const float *dh_actor, const float *dmu,
                               const float *dvalue, int32_t num_actions, void *dy, int32_t dtype, float *partial,
                               void *stream) {
  if (int rc = check_tail(args)) return rc;
  PHC_REQUIRE(dh_actor && dmu && dvalue && dy && partial, "tail_ln_bwd: null argument");
  PHC_REQUIRE(num_actions >= 1 && num_actions <= kTA, "tail_ln_bwd: 1..%d actions", kTA);
  PHC_REQUIRE(dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "tail_ln_bwd: dy must be f16 or bf16");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(dy) & 7) == 0 && (reinterpret_cast<uintptr_t>(dh_actor) & 15) == 0,
              "tail_ln_bwd: dy must be 8-byte and dh_actor 16-byte aligned");
  const int blocks = phc_tail_blocks(args->rows);
  hipStream_t st = as_stream(stream);
  if (dtype == PHC_DT_F16)
    hipLaunchKernelGGL(k_tail_ln_bwd<_Float16>, dim3(blocks), dim3(kBwdThreads), 0, st, *args, dh_actor, dmu, dvalue,
                       (int)num_actions, static_cast<_Float16 *>(dy), partial);
  else
    hipLaunchKernelGGL(k_tail_ln_bwd<__bf16>, dim3(blocks), dim3(kBwdThreads), 0, st, *args, dh_actor, dmu, dvalue,
                       (int)num_actions, static_cast<__bf16 *>(dy), partial);
  return check_launch("tail_ln_bwd");
}
