// phc_mlp.hip — fused epilogues of the PHCPolicy actor/critic trunks (R19/R21).
//
// The two 6-layer SiLU trunks (policies/phc_policy.py:10-61) run side by side as "twin"
// layers: the GEMMs are plain library GEMMs (one [M,934]x[934,2x2048] GEMM for the shared
// input, then batched GEMMs over the 2 trunks), and everything between GEMMs is one of the two
// kernels below, so each activation tensor makes one HBM round trip per direction:
//   forward : pre = y + bias (kept for backward), out = silu(pre)
//   backward: g = dout * silu'(pre), bias_grad = sum over rows of g (per-block partial column
//             sums in fp32, then one reduce; deterministic, no atomics)
// A twin tensor holds G groups (trunks) of N columns for M rows, either SPLIT [M, G*N] (the
// output of the shared first GEMM) or GROUPED [G, M, N] (batched-GEMM operands); the kernels
// convert between the two on the fly.  Element types: f32 (xf32 GEMMs), f16, bf16 (GEMMs in
// reduced precision); arithmetic is fp32.
#include "phc_common.h"

#include <type_traits>

namespace phc {

constexpr int kColsPerBlock = 256;  // 64 lanes x 4 consecutive columns
constexpr int kRowsPerBlock = 64;   // 4 waves x 16 rows

template <typename T> struct Pack4 {
  T v[4];
};

template <typename T> __device__ __forceinline__ void ld4(const T *p, float o[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 v = *reinterpret_cast<const float4 *>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    const uint2 raw = *reinterpret_cast<const uint2 *>(p);
    Pack4<T> v;
    __builtin_memcpy(&v, &raw, sizeof(raw));
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (float)v.v[k];
  }
}

template <typename T> __device__ __forceinline__ void st4(T *p, const float o[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4 *>(p) = float4{o[0], o[1], o[2], o[3]};
  } else {
    Pack4<T> v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v.v[k] = (T)o[k];
    uint2 raw;
    __builtin_memcpy(&raw, &v, sizeof(raw));
    *reinterpret_cast<uint2 *>(p) = raw;
  }
}

struct TwinShape {
  int64_t m;
  int g, n;
};

// offset of logical element (row, column c = group * n + j) in a twin tensor
__device__ __forceinline__ int64_t twin_off(const TwinShape &s, int layout, int64_t row, int c) {
  if (layout == PHC_LAYOUT_SPLIT) return row * (int64_t)(s.g * s.n) + c;
  const int grp = c / s.n;
  return ((int64_t)grp * s.m + row) * s.n + (c - grp * s.n);
}

__device__ __forceinline__ float silu(float a) { return a / (1.0f + expf(-a)); }
__device__ __forceinline__ float silu_grad(float dz, float a) {
  const float sg = 1.0f / (1.0f + expf(-a));
  return dz * sg * (1.0f + a * (1.0f - sg));
}

template <typename T, typename To>
__global__ __launch_bounds__(256) void k_bias_act_fwd(const T *y, int y_layout, const float *__restrict__ bias, T *pre,
                                                      To *out, int out_layout, TwinShape s, int act) {
  const int c = blockIdx.x * kColsPerBlock + (threadIdx.x & 63) * 4;
  if (c >= s.g * s.n) return;
  float b[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (bias) {
    const float4 bv = *reinterpret_cast<const float4 *>(bias + c);
    b[0] = bv.x; b[1] = bv.y; b[2] = bv.z; b[3] = bv.w;
  }
  const int64_t r0 = (int64_t)blockIdx.y * kRowsPerBlock + (threadIdx.x >> 6);
  for (int i = 0; i < kRowsPerBlock / 4; ++i) {
    const int64_t row = r0 + 4 * i;
    if (row >= s.m) break;
    float v[4];
    const int64_t oy = twin_off(s, y_layout, row, c);
    ld4(y + oy, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] + b[k];
    if (pre) st4(pre + oy, v);
    if (act == PHC_ACT_SILU) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = silu(v[k]);
    }
    if (out) st4(out + twin_off(s, out_layout, row, c), v);
  }
}

template <typename T, typename To>
__global__ __launch_bounds__(256) void k_act_bwd(const T *dz, int dz_layout, const T *pre, int pre_layout,
                                                 const float *__restrict__ pre_bias, To *g, int g_layout,
                                                 float *__restrict__ partial, TwinShape s, int act) {
  __shared__ float red[4][kColsPerBlock];
  const int lane4 = (threadIdx.x & 63) * 4;
  const int w = threadIdx.x >> 6;
  const int c = blockIdx.x * kColsPerBlock + lane4;
  const bool col_ok = c < s.g * s.n;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float pb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (col_ok && pre_bias) {
    const float4 bv = *reinterpret_cast<const float4 *>(pre_bias + c);
    pb[0] = bv.x; pb[1] = bv.y; pb[2] = bv.z; pb[3] = bv.w;
  }
  if (col_ok) {
    const int64_t r0 = (int64_t)blockIdx.y * kRowsPerBlock + w;
    for (int i = 0; i < kRowsPerBlock / 4; ++i) {
      const int64_t row = r0 + 4 * i;
      if (row >= s.m) break;
      float d[4];
      ld4(dz + twin_off(s, dz_layout, row, c), d);
      if (act == PHC_ACT_SILU) {
        float a[4];
        ld4(pre + twin_off(s, pre_layout, row, c), a);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = silu_grad(d[k], a[k] + pb[k]);
      }
      if (g) st4(g + twin_off(s, g_layout, row, c), d);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += d[k];
    }
  }
  if (!partial) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) red[w][lane4 + k] = acc[k];
  __syncthreads();
  if (w == 0 && col_ok) {
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = ((red[0][lane4 + k] + red[1][lane4 + k]) + red[2][lane4 + k]) + red[3][lane4 + k];
    *reinterpret_cast<float4 *>(partial + (int64_t)blockIdx.y * (s.g * s.n) + c) = float4{o[0], o[1], o[2], o[3]};
  }
}

// ------------------------------------------------ LayerNorm + SiLU (twin head) --
// z = silu(LayerNorm(y) * gamma + beta) per row of a GROUPED [G, M, N] tensor with per-group
// affine parameters (the actor's and the critic's nn.LayerNorm(512) + nn.SiLU(),
// policies/phc_policy.py:16-30).  One wave per row; lane l owns the 4-element chunks
// l, l + 64, ... (coalesced 16-B accesses); row mean / rstd saved for the backward (torch's
// LayerNorm: biased variance, rsqrt(var + eps)).
constexpr int kLnMaxChunks = 4;     // N <= 1024 (4 chunks of 4 per lane)
constexpr int kLnRowsPerBlock = 64;  // backward: rows per block (16 per wave) before the column sums

template <typename T, int C>
__global__ __launch_bounds__(256) void k_ln_silu_fwd(const T *__restrict__ y, const float *__restrict__ gamma,
                                                     const float *__restrict__ beta, float *__restrict__ z,
                                                     float *__restrict__ mean_rstd, int64_t rows, int g, int n,
                                                     float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row of the [G*M] stack
  const int lane = threadIdx.x & 63;
  if (row >= rows * g) return;
  const int grp = (int)(row / rows);
  constexpr int chunks = C;  // n / 256
  float x[C][4];
  float s = 0.0f;
  #pragma unroll
  for (int k = 0; k < chunks; ++k) {
    ld4(y + row * n + 4 * (lane + 64 * k), x[k]);
    s += (x[k][0] + x[k][1]) + (x[k][2] + x[k][3]);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)n;
  float v = 0.0f;
  #pragma unroll
  for (int k = 0; k < chunks; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = x[k][e] - mean;
      v += d * d;
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const float rstd = rsqrtf(v / (float)n + eps);
  #pragma unroll
  for (int k = 0; k < chunks; ++k) {
    const int c = 4 * (lane + 64 * k);
    float gm[4], bt[4], o4[4];
    ld4(gamma + grp * n + c, gm);
    ld4(beta + grp * n + c, bt);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ln = (x[k][e] - mean) * rstd * gm[e] + bt[e];
      o4[e] = tail_silu(ln);
    }
    st4(z + row * n + c, o4);
  }
  if (lane == 0) {
    mean_rstd[2 * row] = mean;
    mean_rstd[2 * row + 1] = rstd;
  }
}

// dy = LayerNorm backward of (dz * silu'(ln)).  A block (4 waves) covers kLnRowsPerBlock rows of
// one group, two rows in flight per wave; the column sums of dln * xhat (gamma grad) and dln
// (beta grad) over those rows go to one partial row per block (LDS reduction over the waves).
template <typename T, int C>
__global__ __launch_bounds__(256) void k_ln_silu_bwd(const T *__restrict__ y, const float *__restrict__ gamma,
                                                     const float *__restrict__ beta,
                                                     const float *__restrict__ mean_rstd,
                                                     const float *__restrict__ dz, T *__restrict__ dy,
                                                     float *__restrict__ partial, int64_t rows, int n) {
  __shared__ float4 red[3][2 * C * 64];  // waves 1..3: (gamma | beta) sums per lane chunk
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t bpg = (rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock;
  const int grp = (int)(blockIdx.x / bpg);
  const int64_t r0 = (blockIdx.x - (int64_t)grp * bpg) * kLnRowsPerBlock + w * (kLnRowsPerBlock / 4);
  constexpr int chunks = C;  // n / 256
  float gm[C][4], bt[C][4], pg[C][4], pb[C][4];
  #pragma unroll
  for (int k = 0; k < chunks; ++k) {
    ld4(gamma + grp * n + 4 * (lane + 64 * k), gm[k]);
    ld4(beta + grp * n + 4 * (lane + 64 * k), bt[k]);
#pragma unroll
    for (int e = 0; e < 4; ++e) pg[k][e] = pb[k][e] = 0.0f;
  }
  for (int i = 0; i < kLnRowsPerBlock / 4; i += 2) {
    float yv[2][C][4], dv[2][C][4], mr[2][2];
    bool ok[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t r = r0 + i + h;
      ok[h] = r < rows;
      if (!ok[h]) continue;
      const int64_t row = (int64_t)grp * rows + r;
      mr[h][0] = mean_rstd[2 * row];
      mr[h][1] = mean_rstd[2 * row + 1];
      #pragma unroll
      for (int k = 0; k < chunks; ++k) {
        ld4(y + row * n + 4 * (lane + 64 * k), yv[h][k]);
        ld4(dz + row * n + 4 * (lane + 64 * k), dv[h][k]);
      }
    }
    float s1[2] = {0.0f, 0.0f}, s2[2] = {0.0f, 0.0f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!ok[h]) continue;
      #pragma unroll
      for (int k = 0; k < chunks; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (yv[h][k][e] - mr[h][0]) * mr[h][1];
          const float ln = xh * gm[k][e] + bt[k][e];
          const float sg = tail_sigmoid(ln);
          const float dln = dv[h][k][e] * sg * (1.0f + ln * (1.0f - sg));
          pg[k][e] += dln * xh;
          pb[k][e] += dln;
          const float dxh = dln * gm[k][e];
          s1[h] += dxh;
          s2[h] += dxh * xh;
          yv[h][k][e] = xh;   // keep xhat
          dv[h][k][e] = dxh;  // and d xhat
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s1[0] += __shfl_xor(s1[0], o, 64);
      s2[0] += __shfl_xor(s2[0], o, 64);
      s1[1] += __shfl_xor(s1[1], o, 64);
      s2[1] += __shfl_xor(s2[1], o, 64);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!ok[h]) continue;
      const int64_t row = (int64_t)grp * rows + r0 + i + h;
      const float m1 = s1[h] / (float)n, m2 = s2[h] / (float)n, rstd = mr[h][1];
      #pragma unroll
      for (int k = 0; k < chunks; ++k) {
        float o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = rstd * (dv[h][k][e] - m1 - yv[h][k][e] * m2);
        st4(dy + row * n + 4 * (lane + 64 * k), o4);
      }
    }
  }
  // block reduction: waves 1..3 park their sums in LDS, wave 0 adds them in wave order
  if (w > 0)
    #pragma unroll
    for (int k = 0; k < chunks; ++k) {
      red[w - 1][k * 64 + lane] = make_float4(pg[k][0], pg[k][1], pg[k][2], pg[k][3]);
      red[w - 1][(C + k) * 64 + lane] = make_float4(pb[k][0], pb[k][1], pb[k][2], pb[k][3]);
    }
  __syncthreads();
  if (w > 0) return;
  float *pr = partial + (int64_t)blockIdx.x * (2 * n);  // [bpg * G, 2n] = (gamma grad | beta grad)
  #pragma unroll
  for (int k = 0; k < chunks; ++k) {
    for (int v = 0; v < 3; ++v) {
      const float4 a = red[v][k * 64 + lane], b = red[v][(C + k) * 64 + lane];
      pg[k][0] += a.x; pg[k][1] += a.y; pg[k][2] += a.z; pg[k][3] += a.w;
      pb[k][0] += b.x; pb[k][1] += b.y; pb[k][2] += b.z; pb[k][3] += b.w;
    }
    const int c = 4 * (lane + 64 * k);
    st4(pr + c, pg[k]);
    st4(pr + n + c, pb[k]);
  }
}

// column sums of [rows, cols] partials where output columns [0, split) go to out_a and
// [split, cols) to out_b
__global__ __launch_bounds__(256) void k_colsum_strided(const float *__restrict__ partial, int rows, int cols,
                                                        float *__restrict__ out_a, float *__restrict__ out_b,
                                                        int split) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, rs = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cl * 4;
  float4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  if (c < cols) {
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
    float *o = c < split ? out_a + c : out_b + (c - split);
    o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
  }
}

static bool valid_dtype(int d) { return d == PHC_DT_F32 || d == PHC_DT_F16 || d == PHC_DT_BF16; }

static int check_twin(const void *p, int layout, int dtype, const char *what) {
  PHC_REQUIRE(p, "%s: null tensor", what);
  PHC_REQUIRE(layout == PHC_LAYOUT_SPLIT || layout == PHC_LAYOUT_GROUPED, "%s: bad layout", what);
  const uintptr_t align = dtype == PHC_DT_F32 ? 16 : 8;
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(p) & (align - 1)) == 0, "%s: misaligned", what);
  return PHC_OK;
}

static dim3 twin_grid(const TwinShape &s) {
  return dim3((unsigned)((s.g * s.n + kColsPerBlock - 1) / kColsPerBlock),
              (unsigned)((s.m + kRowsPerBlock - 1) / kRowsPerBlock));
}

// element-type pairs (input, output): equal types, or f32 GEMM outputs -> f16 / bf16 operands
template <template <typename, typename> class K, typename F>
static bool dispatch_twin(int dtype, int out_dtype, F &&launch) {
  if (dtype == out_dtype) {
    if (dtype == PHC_DT_F32) launch(K<float, float>{});
    else if (dtype == PHC_DT_F16) launch(K<_Float16, _Float16>{});
    else launch(K<__bf16, __bf16>{});
    return true;
  }
  if (dtype != PHC_DT_F32) return false;
  if (out_dtype == PHC_DT_F16) launch(K<float, _Float16>{});
  else launch(K<float, __bf16>{});
  return true;
}

template <typename T, typename To> struct ActFwd {
  using in = T;
  using out = To;
  static constexpr auto kernel = k_bias_act_fwd<T, To>;
};
template <typename T, typename To> struct ActBwd {
  using in = T;
  using out = To;
  static constexpr auto kernel = k_act_bwd<T, To>;
};

}  // namespace phc

using namespace phc;

extern "C" int phc_bias_act_fwd(const void *y, int32_t y_layout, const float *bias, void *pre, void *out,
                                int32_t out_layout, int64_t rows, int32_t groups, int32_t cols, int32_t act,
                                int32_t dtype, int32_t out_dtype, void *stream) {
  PHC_REQUIRE(rows >= 0 && groups >= 1 && cols > 0 && cols % 4 == 0, "bias_act_fwd: bad shape");
  PHC_REQUIRE(act == PHC_ACT_NONE || act == PHC_ACT_SILU, "bias_act_fwd: bad act");
  PHC_REQUIRE(valid_dtype(dtype) && valid_dtype(out_dtype) && (dtype == out_dtype || dtype == PHC_DT_F32),
              "bias_act_fwd: bad dtype pair (%d, %d)", dtype, out_dtype);
  if (rows == 0) return PHC_OK;
  if (int rc = check_twin(y, y_layout, dtype, "bias_act_fwd y")) return rc;
  PHC_REQUIRE(pre || out, "bias_act_fwd: nothing to write");
  if (out)
    if (int rc = check_twin(out, out_layout, out_dtype, "bias_act_fwd out")) return rc;
  if (pre)
    if (int rc = check_twin(pre, y_layout, dtype, "bias_act_fwd pre")) return rc;
  PHC_REQUIRE(!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0, "bias_act_fwd: misaligned bias");
  PHC_REQUIRE(!(out && out == y && (out_layout != y_layout || out_dtype != dtype)),
              "bias_act_fwd: in-place output needs the input layout and type");
  const TwinShape s{rows, groups, cols};
  hipStream_t st = as_stream(stream);
  dispatch_twin<ActFwd>(dtype, out_dtype, [&](auto k) {
    using K = decltype(k);
    hipLaunchKernelGGL(K::kernel, twin_grid(s), dim3(256), 0, st, (const typename K::in *)y, y_layout, bias,
                       (typename K::in *)pre, (typename K::out *)out, out_layout, s, act);
  });
  return check_launch("bias_act_fwd");
}

extern "C" size_t phc_act_bwd_workspace_bytes(int64_t rows, int32_t groups, int32_t cols) {
  if (rows <= 0 || groups <= 0 || cols <= 0) return 0;
  return (size_t)((rows + kRowsPerBlock - 1) / kRowsPerBlock) * (size_t)groups * (size_t)cols * sizeof(float);
}

extern "C" int phc_act_bwd(const void *grad_out, int32_t go_layout, const void *pre, int32_t pre_layout,
                           const float *pre_bias, void *grad_pre, int32_t gp_layout, float *bias_grad, int64_t rows,
                           int32_t groups, int32_t cols, int32_t act, int32_t dtype, int32_t out_dtype,
                           void *workspace, void *stream) {
  PHC_REQUIRE(rows >= 0 && groups >= 1 && cols > 0 && cols % 4 == 0, "act_bwd: bad shape");
  PHC_REQUIRE(act == PHC_ACT_NONE || act == PHC_ACT_SILU, "act_bwd: bad act");
  PHC_REQUIRE(valid_dtype(dtype) && valid_dtype(out_dtype) && (dtype == out_dtype || dtype == PHC_DT_F32),
              "act_bwd: bad dtype pair (%d, %d)", dtype, out_dtype);
  const TwinShape s{rows, groups, cols};
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    if (bias_grad) (void)hipMemsetAsync(bias_grad, 0, sizeof(float) * groups * cols, st);
    return check_launch("act_bwd");
  }
  if (int rc = check_twin(grad_out, go_layout, dtype, "act_bwd grad_out")) return rc;
  if (act == PHC_ACT_SILU)
    if (int rc = check_twin(pre, pre_layout, dtype, "act_bwd pre")) return rc;
  if (grad_pre)
    if (int rc = check_twin(grad_pre, gp_layout, out_dtype, "act_bwd grad_pre")) return rc;
  PHC_REQUIRE(!(grad_pre && (grad_pre == grad_out || grad_pre == pre) && out_dtype != dtype),
              "act_bwd: in-place grad needs the input type");
  PHC_REQUIRE(!(grad_pre && grad_pre == grad_out && gp_layout != go_layout),
              "act_bwd: in-place grad needs the grad_out layout");
  PHC_REQUIRE(grad_pre || bias_grad, "act_bwd: nothing to write");
  PHC_REQUIRE(!pre_bias || (reinterpret_cast<uintptr_t>(pre_bias) & 15) == 0, "act_bwd: misaligned pre_bias");
  float *partial = nullptr;
  const dim3 grid = twin_grid(s);
  if (bias_grad) {
    PHC_REQUIRE(workspace, "act_bwd: bias_grad needs a workspace");
    PHC_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "act_bwd: misaligned workspace");
    partial = static_cast<float *>(workspace);
  }
  dispatch_twin<ActBwd>(dtype, out_dtype, [&](auto k) {
    using K = decltype(k);
    hipLaunchKernelGGL(K::kernel, grid, dim3(256), 0, st, (const typename K::in *)grad_out, go_layout,
                       (const typename K::in *)pre, pre_layout, pre_bias, (typename K::out *)grad_pre, gp_layout,
                       partial, s, act);
  });
  if (bias_grad) {
    const int c = groups * cols;
    hipLaunchKernelGGL(k_colsum<>, dim3((unsigned)((c + 63) / 64)), dim3(256), 0, st, partial, (int)grid.y, c,
                       bias_grad);
  }
  return check_launch("act_bwd");
}

// ------------------------------------------------------------- LN + SiLU C ABI --
// instantiate for the element type and the per-lane chunk count (cols / 256)
template <template <typename, int> class K, typename F>
static void dispatch_ln(int32_t dtype, int chunks, F &&launch) {
  auto by_type = [&](auto c) {
    constexpr int C = decltype(c)::value;
    if (dtype == PHC_DT_F32) launch(K<float, C>{});
    else if (dtype == PHC_DT_F16) launch(K<_Float16, C>{});
    else launch(K<__bf16, C>{});
  };
  switch (chunks) {
    case 1: by_type(std::integral_constant<int, 1>{}); break;
    case 2: by_type(std::integral_constant<int, 2>{}); break;
    case 3: by_type(std::integral_constant<int, 3>{}); break;
    default: by_type(std::integral_constant<int, 4>{}); break;
  }
}

template <typename T, int C> struct LnFwd {
  using type = T;
  static constexpr auto kernel = k_ln_silu_fwd<T, C>;
};
template <typename T, int C> struct LnBwd {
  using type = T;
  static constexpr auto kernel = k_ln_silu_bwd<T, C>;
};

extern "C" int phc_ln_silu_fwd(const void *y, const float *gamma, const float *beta, float *z, float *mean_rstd,
                               int64_t rows, int32_t groups, int32_t cols, float eps, int32_t dtype, void *stream) {
  PHC_REQUIRE(y && gamma && beta && z && mean_rstd, "ln_silu_fwd: null argument");
  PHC_REQUIRE(rows > 0 && groups >= 1 && cols % 256 == 0 && cols / 256 <= kLnMaxChunks,
              "ln_silu_fwd: cols must be a multiple of 256 up to %d", 256 * kLnMaxChunks);
  PHC_REQUIRE(dtype == PHC_DT_F32 || dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "ln_silu_fwd: bad dtype");
  const dim3 grid((unsigned)((rows * groups + 3) / 4));
  hipStream_t st = as_stream(stream);
  dispatch_ln<LnFwd>(dtype, cols / 256, [&](auto k) {
    using T = typename decltype(k)::type;
    hipLaunchKernelGGL(decltype(k)::kernel, grid, dim3(256), 0, st, (const T *)y, gamma, beta, z, mean_rstd, rows,
                       (int)groups, (int)cols, eps);
  });
  return check_launch("ln_silu_fwd");
}

extern "C" size_t phc_ln_silu_workspace_bytes(int64_t rows, int32_t groups, int32_t cols) {
  if (rows <= 0 || groups <= 0 || cols <= 0) return 0;
  const int64_t blocks = (rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock * groups;
  return (size_t)blocks * 2 * cols * sizeof(float);
}

extern "C" int phc_ln_silu_bwd(const void *y, const float *gamma, const float *beta, const float *mean_rstd,
                               const float *dz, void *dy, float *dgamma, float *dbeta, int64_t rows, int32_t groups,
                               int32_t cols, int32_t dtype, void *workspace, void *stream) {
  PHC_REQUIRE(y && gamma && beta && mean_rstd && dz && dy && dgamma && dbeta && workspace,
              "ln_silu_bwd: null argument");
  PHC_REQUIRE(rows > 0 && groups >= 1 && cols % 256 == 0 && cols / 256 <= kLnMaxChunks, "ln_silu_bwd: bad shape");
  PHC_REQUIRE(dtype == PHC_DT_F32 || dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "ln_silu_bwd: bad dtype");
  const int64_t wpg = (rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock;  // partial rows per group
  const dim3 grid((unsigned)(wpg * groups));
  hipStream_t st = as_stream(stream);
  float *partial = static_cast<float *>(workspace);
  dispatch_ln<LnBwd>(dtype, cols / 256, [&](auto k) {
    using T = typename decltype(k)::type;
    hipLaunchKernelGGL(decltype(k)::kernel, grid, dim3(256), 0, st, (const T *)y, gamma, beta, mean_rstd, dz,
                       (T *)dy, partial, rows, (int)cols);
  });
  // per group: column sums of its wpg partial rows -> dgamma[grp], dbeta[grp]
  for (int32_t grp = 0; grp < groups; ++grp) {
    const float *pg = partial + (int64_t)grp * wpg * 2 * cols;
    hipLaunchKernelGGL(k_colsum_strided, dim3((unsigned)((2 * cols + 63) / 64)), dim3(256), 0, st, pg, (int)wpg,
                       2 * cols, dgamma + (int64_t)grp * cols, dbeta + (int64_t)grp * cols, cols);
  }
  return check_launch("ln_silu_bwd");
}
