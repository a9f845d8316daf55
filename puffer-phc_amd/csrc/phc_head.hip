// phc_head.hip — the actor's mu head in fp32 on the fp32-input MFMA (R19 / R21).
//
// The reference's mu head is nn.Linear(512, num_actions) in fp32 (policies/phc_policy.py:40-61;
// the PPO update runs it under torch autograd, clean_pufferl/core.py:298-354).  With num_actions
// = 69 its three GEMMs per minibatch are skinny (N or K = 69), so they run here as three small
// kernels on v_mfma_f32_16x16x4_f32 — exact fp32 products, fp32 accumulation, the f32 vector
// rate — instead of library GEMMs:
//   k_head_fwd   : mu[M, A]  = h[M, H] · W[A, H]^T + b          (one wave per 16 rows x 80 columns)
//   k_head_dgrad : dh[M, H]  = dmu[M, A] · W[A, H]              (one wave per 16 rows x 128 columns)
//   k_head_wgrad : part[s]   = dmu[rows_s]^T · h[rows_s]        (one wave per 80 x 32 outputs, rows
//                  split into S chunks; the caller sums the S partials, e.g. phc_reduce_into)
// Fragments come straight from global memory (the operands are L2-resident: W is 141 KB, the row
// tiles are read once).  K is walked in chunks of 16 with a permuted order inside each chunk —
// MFMA step t of chunk q feeds lane group g the index 16 q + 4 g + t on both operands — so every
// lane reads 4 consecutive K values with one 16-B load where the operand is K-contiguous.  A is at
// most 80 (5 blocks of 16).
// phc_mu_head_fwd / _dgrad launch the bf16-x3 forms below (k_head_fwd_x3 / k_head_dgrad_x3:
// three-way bf16 operand splits on v_mfma_f32_16x16x32_bf16, fp32-class products) when H % 32 == 0;
// the f32-MFMA kernels above serve the other widths (and PHC_MU_X3=0 for the input gradient).
#include "phc_common.h"
#include "phc_x3.h"

#include <algorithm>
#include <cstdlib>

namespace phc {

using hf4 = __attribute__((ext_vector_type(4))) float;
constexpr int kHeadMaxA = 80;
constexpr size_t kHeadLdsMax = 160 * 1024;  // LDS per workgroup (MI355X: 160 KB per CU)

__device__ __forceinline__ hf4 head_mfma(float a, float b, hf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// mu = h W^T + b.  Block = 4 waves = 64 rows; wave w: rows r0 + 16 w .. + 15, all 80 columns.
__global__ __launch_bounds__(256) void k_head_fwd(const float *__restrict__ h, const float *__restrict__ w,
                                                  const float *__restrict__ b, float *__restrict__ mu, int64_t M,
                                                  int H, int A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * 64 + wave * 16;
  if (r0 >= M) return;
  int64_t hr = r0 + c;
  hr = hr < M ? hr : M - 1;  // ragged last tile: clamp the read, mask the store
  const float *hp = h + hr * H + 4 * g;
  const float *wp[5];
  bool wv[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    const int a = 16 * nb + c;
    wv[nb] = a < A;
    wp[nb] = w + (int64_t)(wv[nb] ? a : 0) * H + 4 * g;
  }
  hf4 acc[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) acc[nb] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
  // chunk k0's operands are loaded one chunk ahead of its MFMAs (two register sets)
  float4 hv[2], wf[2][5];
  auto load = [&](int k0, int b) {
    hv[b] = *reinterpret_cast<const float4 *>(hp + k0);
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) wf[b][nb] = *reinterpret_cast<const float4 *>(wp[nb] + k0);
  };
  auto compute = [&](int b) {  // step-major: consecutive MFMAs write different accumulators
    float4 wv4[5];
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) wv4[nb] = wv[nb] ? wf[b][nb] : float4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(hv[b].x, wv4[nb].x, acc[nb]);
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(hv[b].y, wv4[nb].y, acc[nb]);
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(hv[b].z, wv4[nb].z, acc[nb]);
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(hv[b].w, wv4[nb].w, acc[nb]);
  };
  load(0, 0);
  for (int k0 = 0; k0 < H; k0 += 32) {  // H % 16 == 0: the second half-step may be absent
    if (k0 + 16 < H) load(k0 + 16, 1);
    compute(0);
    if (k0 + 16 >= H) break;
    if (k0 + 32 < H) load(k0 + 32, 0);
    compute(1);
  }
  // lane: column a = 16 nb + c, rows r0 + 4 g + e
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    const int a = 16 * nb + c;
    if (a >= A) continue;
    const float bias = b[a];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = r0 + 4 * g + e;
      if (row < M) mu[row * A + a] = acc[nb][e] + bias;
    }
  }
}

// dh = dmu W.  Block = 4 waves = 16 rows x 512 columns; wave w: columns 128 w .. + 127 (8 blocks),
// blockIdx.y walks further 512-column panels when H > 512.  K = A in chunks of 16 (zero past A).
__global__ __launch_bounds__(256) void k_head_dgrad(const float *__restrict__ dmu, const float *__restrict__ w,
                                                    float *__restrict__ dh, int64_t M, int H, int A) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const int c0 = blockIdx.y * 512 + wave * 128;
  if (c0 >= H) return;
  int64_t ar = r0 + c;
  ar = ar < M ? ar : M - 1;
  const float *ap = dmu + ar * A;
  hf4 acc[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) acc[nb] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
  // the lane's whole dmu fragment (k = 16 q + 4 g + t, q < 5) up front; W one chunk ahead
  // loads are unconditional (clamped addresses) and masked after they land: a select around a
  // load makes the compiler branch and drain the load queue per element
  float av[5][4];
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 16 * q + 4 * g + t;
      av[q][t] = ap[k < A ? k : A - 1];
    }
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (16 * q + 4 * g + t >= A) av[q][t] = 0.0f;  // the matching W rows are zeroed too
  int colc[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) colc[nb] = c0 + 16 * nb + c < H ? 16 * nb : H - 1 - c0 - c;
  float bw[2][4][8];
  auto load = [&](int q, int b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 16 * q + 4 * g + t;
      const float *wr = w + (int64_t)(k < A ? k : A - 1) * H + c0 + c;
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) bw[b][t][nb] = wr[colc[nb]];
    }
  };
  auto compute = [&](int q, int b) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[nb] = head_mfma(av[q][t], bw[b][t][nb], acc[nb]);
  };
  const int nq = (A + 15) / 16;
  load(0, 0);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    if (q >= nq) break;
    if (q + 1 < nq) load(q + 1, (q + 1) & 1);
    compute(q, q & 1);
  }
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) {
    const int col = c0 + 16 * nb + c;
    if (col >= H) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = r0 + 4 * g + e;
      if (row < M) dh[row * H + col] = acc[nb][e];
    }
  }
}

// part[s] = dmu[rows_s]^T h[rows_s] for the s-th chunk of rows_per_split rows (the last chunk
// ragged).  Block (blockIdx.x = column panel of 128, blockIdx.y = s) = 4 waves; wave w: all 80
// output rows (a) x columns 128 x + 32 w .. + 31 (2 blocks).  K = rows in chunks of 16.
__global__ __launch_bounds__(256) void k_head_wgrad(const float *__restrict__ dmu, const float *__restrict__ h,
                                                    float *__restrict__ part, int64_t M, int H, int A,
                                                    int64_t rows_per_split) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int c0 = blockIdx.x * 128 + wave * 32;
  const int64_t s = blockIdx.y, rb = s * rows_per_split;
  const int64_t re = rb + rows_per_split < M ? rb + rows_per_split : M;
  hf4 acc[5][2];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
  const bool colv[2] = {c0 + c < H, c0 + 16 + c < H};
  float av[2][4][5], bv[2][4][2];  // one 16-row chunk's fragments, loaded a chunk ahead
  int ac[5];  // clamped dmu columns (masked after the load), see k_head_dgrad
#pragma unroll
  for (int i = 0; i < 5; ++i) ac[i] = 16 * i + c < A ? 16 * i + c : A - 1;
  const int hc[2] = {colv[0] ? c0 + c : H - 1, colv[1] ? c0 + 16 + c : H - 1};
  auto load = [&](int64_t k0, int b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t row = k0 + 4 * g + t;
      const bool rv = row < re;
      const float *arow = dmu + (rv ? row : rb) * A;
      const float *hrow = h + (rv ? row : rb) * H;
#pragma unroll
      for (int i = 0; i < 5; ++i) av[b][t][i] = arow[ac[i]];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[b][t][j] = hrow[hc[j]];
#pragma unroll
      for (int i = 0; i < 5; ++i)
        if (!rv || 16 * i + c >= A) av[b][t][i] = 0.0f;
    }
  };
  auto compute = [&](int b) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = head_mfma(av[b][t][i], bv[b][t][j], acc[i][j]);
  };
  if (rb < re) load(rb, 0);
  for (int64_t k0 = rb; k0 < re; k0 += 32) {
    if (k0 + 16 < re) load(k0 + 16, 1);
    compute(0);
    if (k0 + 16 >= re) break;
    if (k0 + 32 < re) load(k0 + 32, 0);
    compute(1);
  }
  // lane: output row a = 16 i + 4 g + e, column c0 + 16 j + c
  float *out = part + s * (int64_t)A * H;
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int a = 16 * i + 4 * g + e;
      if (a >= A) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (colv[j]) out[(int64_t)a * H + c0 + 16 * j + c] = acc[i][j][e];
    }
}

// ---- W staged in LDS once per workgroup (persistent over row tiles) ------------------------------
// Forward: W as [A][H + 4] fp32 in LDS (row stride 16 B off a multiple of 256 B, so the 16 lanes of
// a ds_read_b128 group, 16 consecutive rows a at the same k, hit 16 distinct 16-B bank slots);
// every wave then reads its B fragments from LDS instead of re-reading W from L2 per 16 rows.
constexpr int kHeadFwdWaves = 8;  // LDS-staged forward: 2 waves per SIMD

__global__ __launch_bounds__(kHeadFwdWaves * 64) void k_head_fwd_lds(const float *__restrict__ h, const float *__restrict__ w,
                                                      const float *__restrict__ b, float *__restrict__ mu, int64_t M,
                                                      int H, int A) {
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [A][H + 4]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int ld = H + 4;
  for (int i = threadIdx.x; i < A * (H / 4); i += blockDim.x) {
    const int a = i / (H / 4), k4 = i - a * (H / 4);
    *reinterpret_cast<float4 *>(&wl[a * ld + 4 * k4]) = *reinterpret_cast<const float4 *>(w + (int64_t)a * H + 4 * k4);
  }
  __syncthreads();
  int arow[5];
  bool av[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    av[nb] = 16 * nb + c < A;
    arow[nb] = (av[nb] ? 16 * nb + c : 0) * ld + 4 * g;
  }
  float bias[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) bias[nb] = av[nb] ? b[16 * nb + c] : 0.0f;
  const int64_t tiles = (M + 15) / 16;
  for (int64_t t = (int64_t)blockIdx.x * kHeadFwdWaves + wave; t < tiles; t += (int64_t)gridDim.x * kHeadFwdWaves) {
    const int64_t r0 = t * 16;
    int64_t hr = r0 + c;
    hr = hr < M ? hr : M - 1;
    const float *hp = h + hr * H + 4 * g;
    hf4 acc[5];
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) acc[nb] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
    float4 hv[2];
    hv[0] = *reinterpret_cast<const float4 *>(hp);
    for (int k0 = 0; k0 < H; k0 += 32) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int kk = k0 + 16 * half;
        if (kk >= H) break;
        if (kk + 16 < H) hv[half ^ 1] = *reinterpret_cast<const float4 *>(hp + kk + 16);
        float4 wv[5];
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          wv[nb] = *reinterpret_cast<const float4 *>(&wl[arow[nb] + kk]);
          if (!av[nb]) wv[nb] = float4{0.0f, 0.0f, 0.0f, 0.0f};
        }
        const float4 x = hv[half];
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(x.x, wv[nb].x, acc[nb]);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(x.y, wv[nb].y, acc[nb]);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(x.z, wv[nb].z, acc[nb]);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) acc[nb] = head_mfma(x.w, wv[nb].w, acc[nb]);
      }
    }
#pragma unroll
    for (int nb = 0; nb < 5; ++nb) {
      const int a = 16 * nb + c;
      if (a >= A) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = r0 + 4 * g + e;
        if (row < M) mu[row * A + a] = acc[nb][e] + bias[nb];
      }
    }
  }
}

// ---- forward / input gradient on the bf16 MFMA with three-way operand splits ------------------
// (split3 / mma_x3_n: phc_x3.h).  Six bf16 MFMAs (16 cycles each) per 32-deep step against eight
// 32-cycle v_mfma_f32_16x16x4f32 per 32 K: the launches become bound by their HBM traffic (h / dh:
// 64 MB per 32768-row minibatch) instead of the fp32 matrix rate.
using b8 = x3b8;

// mu = h W^T + b.  W is split once per workgroup into three bf16 planes in LDS, 128 K at a time
// ([80][128 + 8] per plane, rows past A zero); every wave owns one 16-row tile and keeps its
// accumulators across the K chunks.  Lane (g, c): h row / W row c, K = k0 + 8 g .. + 7 of each
// 32-deep step (the same K order on both operands); kX3FwdDepth steps of h are in flight per wave,
// the first ones issued before the W staging.  Requires H % 32 == 0.
#ifndef PHC_HEAD_FWD_WAVES
#define PHC_HEAD_FWD_WAVES 8
#endif
constexpr int kX3FwdWaves = PHC_HEAD_FWD_WAVES;
constexpr int kX3FwdDepth = 4;  // 32-deep steps of h in flight per wave
constexpr int kX3FwdKC = 128, kX3FwdKP = kX3FwdKC + 8;

__global__ __launch_bounds__(kX3FwdWaves * 64) void k_head_fwd_x3(const float *__restrict__ h, const float *__restrict__ w,
                                                                 const float *__restrict__ b, float *__restrict__ mu,
                                                                 int64_t M, int H, int A) {
  __shared__ __attribute__((aligned(16))) __bf16 pl[3][kHeadMaxA * kX3FwdKP];
  constexpr int D = kX3FwdDepth;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int64_t r0 = ((int64_t)blockIdx.x * kX3FwdWaves + wave) * 16;
  const bool live = r0 < M;  // uniform per wave; dead waves still stage W
  int64_t hr = r0 + c;
  hr = hr < M ? hr : M - 1;  // ragged last tile: clamp the read, mask the store
  const float *hp = h + hr * H + 8 * g;
  float4 ring[D][2];
  auto fetch = [&](int d, int kk) {
    ring[d][0] = *reinterpret_cast<const float4 *>(hp + kk);
    ring[d][1] = *reinterpret_cast<const float4 *>(hp + kk + 4);
  };
  if (live) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (32 * d < H) fetch(d, 32 * d);
  }
  hf4 acc[5];
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) acc[nb] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int kc = 0; kc < H; kc += kX3FwdKC) {
    const int kn = H - kc < kX3FwdKC ? H - kc : kX3FwdKC;
    if (kc) __syncthreads();  // the previous chunk's planes are no longer read
    // stage W[:, kc : kc + kn] split into the planes: 4 consecutive K per thread item, 8 in flight
    const int items = kHeadMaxA * (kn / 4);  // all 80 rows (zero past A)
    for (int base = threadIdx.x; base < items; base += 8 * kX3FwdWaves * 64) {
      float4 tmp[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kX3FwdWaves * 64, a = i / (kn / 4), k4 = i - a * (kn / 4);
        tmp[u] = (i < items && a < A) ? *reinterpret_cast<const float4 *>(w + (int64_t)a * H + kc + 4 * k4)
                                      : float4{0.0f, 0.0f, 0.0f, 0.0f};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kX3FwdWaves * 64, a = i / (kn / 4), k4 = i - a * (kn / 4);
        if (i >= items) break;
        const float v[4] = {tmp[u].x, tmp[u].y, tmp[u].z, tmp[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const __bf16 hi = (__bf16)v[j];
          float r = v[j] - (float)hi;
          const __bf16 mi = (__bf16)r;
          r -= (float)mi;
          const int o = a * kX3FwdKP + 4 * k4 + j;
          pl[0][o] = hi;
          pl[1][o] = mi;
          pl[2][o] = (__bf16)r;
        }
      }
    }
    __syncthreads();
    if (!live) continue;
    for (int k0 = kc; k0 < kc + kn; k0 += 32 * D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int kk = k0 + 32 * d;
        if (kk >= kc + kn) break;
        X3 xs;
        split3(ring[d][0], ring[d][1], xs);
        if (kk + 32 * D < H) fetch(d, kk + 32 * D);
        X3 ws[5];
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          const int off = (16 * nb + c) * kX3FwdKP + (kk - kc) + 8 * g;
          ws[nb].h = *reinterpret_cast<const b8 *>(&pl[0][off]);
          ws[nb].m = *reinterpret_cast<const b8 *>(&pl[1][off]);
          ws[nb].l = *reinterpret_cast<const b8 *>(&pl[2][off]);
        }
        mma_x3_n<5>(&xs, ws, acc, true);  // blocks past A multiply zero planes
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int nb = 0; nb < 5; ++nb) {
    const int a = 16 * nb + c;
    if (a >= A) continue;
    const float bias = b[a];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = r0 + 4 * g + e;
      if (row < M) mu[row * A + a] = acc[nb][e] + bias;
    }
  }
}

// dh = dmu W.  Workgroup = 8 waves = 512 rows x one 128-column panel (blockIdx.y); the panel's W
// columns are split once into three bf16 planes in LDS, transposed to [column][K] (K = actions,
// zero past A, padded to 96 + 8) so a lane's 8 consecutive K values are one 16-B read; wave tile =
// 64 rows (4 row blocks) x 128 columns (8 column blocks), 32 accumulators.
constexpr int kX3DgradKP = 104;
// waves per workgroup (64 rows each): the panel's W split is shared by kX3DgradWaves x 64 rows
// (8: 33.9 vs 35.8 us per 32768-row minibatch with 4, profiles/r05_round5b_experiments.txt §15)
#ifndef PHC_HEAD_DGRAD_WAVES
#define PHC_HEAD_DGRAD_WAVES 8
#endif
constexpr int kX3DgradWaves = PHC_HEAD_DGRAD_WAVES, kX3DgradThreads = 64 * kX3DgradWaves;

__global__ __launch_bounds__(kX3DgradThreads, 8 / kX3DgradWaves) void k_head_dgrad_x3(const float *__restrict__ dmu,
                                                                                     const float *__restrict__ w,
                                                                                     float *__restrict__ dh, int64_t M,
                                                                                     int H, int A) {
  __shared__ __attribute__((aligned(16))) __bf16 pl[3][128 * kX3DgradKP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.y * 128;
  const int nq = (A + 31) / 32;  // 32-deep K steps (uniform)
  constexpr int kU = 4096 / kX3DgradThreads;  // loads in flight per thread (16 at 4 waves)
  for (int base = threadIdx.x; base < 32 * nq * 128; base += kU * kX3DgradThreads) {
    float tmp[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = base + kX3DgradThreads * u, k = i >> 7, n = i & 127;
      tmp[u] = (k < A && n0 + n < H) ? w[(int64_t)k * H + n0 + n] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = base + kX3DgradThreads * u, k = i >> 7, n = i & 127;
      if (i >= 32 * nq * 128) break;
      const __bf16 hi = (__bf16)tmp[u];
      float r = tmp[u] - (float)hi;
      const __bf16 mi = (__bf16)r;
      r -= (float)mi;
      pl[0][n * kX3DgradKP + k] = hi;
      pl[1][n * kX3DgradKP + k] = mi;
      pl[2][n * kX3DgradKP + k] = (__bf16)r;
    }
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * (64 * kX3DgradWaves) + wave * 64;
  if (r0 >= M) return;  // after the barrier
  const float *ap[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    int64_t ar = r0 + 16 * rb + c;
    ar = ar < M ? ar : M - 1;
    ap[rb] = dmu + ar * A;
  }
  // computed transposed, dh^T = W^T dmu^T: lane (g, c) then holds 4 consecutive dh columns
  // 16 nb + 4 g .. + 3 of row 16 rb + c, stored as one float4
  hf4 acc[4][8];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) acc[rb][nb] = hf4{0.0f, 0.0f, 0.0f, 0.0f};
  // dmu fragments of step q (clamped loads, masked after landing); step q + 1's loads are issued
  // into the same registers once step q's split has consumed them, so they land during its MFMAs
  float v[4][8];
  auto load = [&](int q) {
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * q + 8 * g + j;
        v[rb][j] = ap[rb][k < A ? k : A - 1];
      }
  };
  load(0);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (q >= nq) break;
    X3 as[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = 32 * q + 8 * g + j < A ? v[rb][j] : 0.0f;
      split3(float4{x[0], x[1], x[2], x[3]}, float4{x[4], x[5], x[6], x[7]}, as[rb]);
    }
    if (q + 1 < nq) load(q + 1);
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int off = (16 * nb + c) * kX3DgradKP + 32 * q + 8 * g;
      X3 ws;
      ws.h = *reinterpret_cast<const b8 *>(&pl[0][off]);
      ws.m = *reinterpret_cast<const b8 *>(&pl[1][off]);
      ws.l = *reinterpret_cast<const b8 *>(&pl[2][off]);
      hf4 cc[4] = {acc[0][nb], acc[1][nb], acc[2][nb], acc[3][nb]};
      mma_x3_n<4>(&ws, as, cc, true);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb][nb] = cc[rb];
    }
  }
  const bool vec = (H & 3) == 0;  // uniform
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int64_t row = r0 + 16 * rb + c;
    if (row >= M) continue;
    float *out = dh + row * H;
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int col = n0 + 16 * nb + 4 * g;
      if (vec && col + 3 < H) {
        *reinterpret_cast<float4 *>(out + col) = float4{acc[rb][nb][0], acc[rb][nb][1], acc[rb][nb][2], acc[rb][nb][3]};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < H) out[col + e] = acc[rb][nb][e];
      }
    }
  }
}

static int head_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}

static int check_head(const void *x, const void *w, int64_t M, int H, int A) {
  PHC_REQUIRE(x && w, "mu_head: null operand");
  PHC_REQUIRE(M > 0 && H > 0 && A >= 1 && A <= kHeadMaxA, "mu_head: bad shape (rows %lld, hidden %d, actions %d <= %d)",
              (long long)M, H, A, kHeadMaxA);
  return PHC_OK;
}

}  // namespace phc

using namespace phc;

extern "C" int phc_mu_head_fwd(const float *h, const float *w, const float *b, float *mu, int64_t rows, int32_t hidden,
                               int32_t num_actions, void *stream) {
  if (int rc = check_head(h, w, rows, hidden, num_actions)) return rc;
  PHC_REQUIRE(b && mu, "mu_head_fwd: null bias / output");
  PHC_REQUIRE(hidden % 16 == 0, "mu_head_fwd: hidden must be a multiple of 16");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(h) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0,
              "mu_head_fwd: h and w must be 16-byte aligned");
  const size_t lds = (size_t)num_actions * (hidden + 4) * sizeof(float);
  if (hidden % 32 == 0) {  // bf16 x3 MFMA: W planes in LDS, one 16-row tile per wave
    const int64_t blocks = (rows + 16 * kX3FwdWaves - 1) / (16 * kX3FwdWaves);
    PHC_REQUIRE(blocks <= 0x7fffffff, "mu_head_fwd: too many rows");
    hipLaunchKernelGGL(k_head_fwd_x3, dim3((unsigned)blocks), dim3(kX3FwdWaves * 64), 0, as_stream(stream), h, w, b, mu,
                       rows, (int)hidden, (int)num_actions);
  } else if (lds <= kHeadLdsMax) {  // W staged in LDS, persistent over 16-row tiles
    static bool attr = [] {
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_head_fwd_lds),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHeadLdsMax);
      return true;
    }();
    (void)attr;
    const int64_t tiles = (rows + 15) / 16;
    const int64_t blocks = std::min<int64_t>((tiles + kHeadFwdWaves - 1) / kHeadFwdWaves, head_cus());
    hipLaunchKernelGGL(k_head_fwd_lds, dim3((unsigned)blocks), dim3(kHeadFwdWaves * 64), lds, as_stream(stream), h, w, b, mu, rows,
                       (int)hidden, (int)num_actions);
  } else {
    const int64_t blocks = (rows + 63) / 64;
    hipLaunchKernelGGL(k_head_fwd, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), h, w, b, mu, rows,
                       (int)hidden, (int)num_actions);
  }
  return check_launch("mu_head_fwd");
}

extern "C" int phc_mu_head_dgrad(const float *dmu, const float *w, float *dh, int64_t rows, int32_t hidden,
                                 int32_t num_actions, void *stream) {
  if (int rc = check_head(dmu, w, rows, hidden, num_actions)) return rc;
  PHC_REQUIRE(dh, "mu_head_dgrad: null output");
  static const bool x3 = [] {
    const char *e = getenv("PHC_MU_X3");
    return !(e && atoi(e) == 0);
  }();
  if (x3) {  // bf16 x3 MFMA, 512 rows x 128 columns per workgroup
    const int64_t per = 64 * kX3DgradWaves;
    const dim3 grid((unsigned)((rows + per - 1) / per), (unsigned)((hidden + 127) / 128));
    hipLaunchKernelGGL(k_head_dgrad_x3, grid, dim3(kX3DgradThreads), 0, as_stream(stream), dmu, w, dh, rows, (int)hidden,
                       (int)num_actions);
    return check_launch("mu_head_dgrad");
  }
  const dim3 grid((unsigned)((rows + 15) / 16), (unsigned)((hidden + 511) / 512));
  hipLaunchKernelGGL(k_head_dgrad, grid, dim3(256), 0, as_stream(stream), dmu, w, dh, rows, (int)hidden,
                     (int)num_actions);
  return check_launch("mu_head_dgrad");
}

extern "C" int phc_mu_head_wgrad(const float *dmu, const float *h, float *partial, int64_t rows, int32_t hidden,
                                 int32_t num_actions, int32_t splits, void *stream) {
  if (int rc = check_head(dmu, h, rows, hidden, num_actions)) return rc;
  PHC_REQUIRE(partial, "mu_head_wgrad: null partials");
  PHC_REQUIRE(splits >= 1 && splits <= 65535, "mu_head_wgrad: 1..65535 splits");
  const int64_t per = (rows + splits - 1) / splits;
  const dim3 grid((unsigned)((hidden + 127) / 128), (unsigned)splits);
  hipLaunchKernelGGL(k_head_wgrad, grid, dim3(256), 0, as_stream(stream), dmu, h, partial, rows, (int)hidden,
                     (int)num_actions, per);
  return check_launch("mu_head_wgrad");
}
