// phc_disc.hip — the AMP discriminator's logits head (R22) around the MFMA GEMMs.
//
// DiscriminatorPolicy.discriminate (puffer_phc/policies/discriminator_policy.py:72-79) is
// RunningNorm -> Linear(1960, 1024) + ReLU -> Linear(1024, H) + ReLU -> Linear(H, 1).  The two
// wide layers run on phc_twin_gemm (BIAS_RELU forward, RELU_GRAD backward); the H -> 1 layer is a
// dot product per row, done here on the last activation h [rows, H] (f16 / bf16, as the GEMM
// epilogue wrote it) with fp32 weights and accumulation:
//   phc_disc_head_fwd : logit = h . w + b, and optionally the adversarial reward of
//                       clean_pufferl/core.py:229-242, -log(max(1 - 1 / (1 + exp(-logit)), 1e-4))
//   phc_disc_head_bwd : from d loss / d logit (gl, the BCE-with-logits gradient autograd hands
//                       back): g = gl * w * [h > 0] (the input gradient of the second ReLU layer,
//                       rounded once into the next GEMM's operand type) and per-block fp32 partial
//                       rows of dW_head = sum gl * h, db_layer2 = sum g, db_head = sum gl.
// One wave per row (lane l owns columns 8 (l + 64 c), c < H / 512), several rows per wave.
#include "phc_common.h"

namespace phc {

constexpr int kDiscRowsPerBlock = 32;  // 4 waves x 8 rows

template <typename T> __device__ __forceinline__ void disc_load8(const T *p, float v[8]) {
  const uint4 raw = *reinterpret_cast<const uint4 *>(p);
  T h[8];
  __builtin_memcpy(h, &raw, sizeof(raw));
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)h[e];
}

__device__ __forceinline__ float disc_wave_sum(float s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

template <typename T, int NC>
__global__ __launch_bounds__(256) void k_disc_head_fwd(const T *__restrict__ h, int64_t ldh, int64_t rows, int width,
                                                       const float *__restrict__ w, const float *__restrict__ b,
                                                       float *__restrict__ logits, float *__restrict__ reward) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wv[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = (lane + 64 * c) * 8 + e;
      wv[c][e] = col < width ? w[col] : 0.0f;
    }
  const float bias = b[0];
  const int64_t r0 = (int64_t)blockIdx.x * kDiscRowsPerBlock + wave * (kDiscRowsPerBlock / 4);
  for (int rr = 0; rr < kDiscRowsPerBlock / 4; ++rr) {
    const int64_t r = r0 + rr;
    if (r >= rows) break;
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 8;
      if (col < width) {
        float v[8];
        disc_load8(h + r * ldh + col, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[e] * wv[c][e];
      }
    }
    s = disc_wave_sum(s);
    if (lane == 0) {
      const float l = s + bias;
      if (logits) logits[r] = l;
      if (reward) {
        const float prob = 1.0f / (1.0f + expf(-l));
        const float q = 1.0f - prob;
        // torch.maximum(1 - prob, 1e-4) propagates a NaN (a diverged discriminator stays visible)
        reward[r] = -logf(q != q ? q : (q > 1.0e-4f ? q : 1.0e-4f));
      }
    }
  }
}

// partial row of block k (stride 2 width + 4, 16-byte rows): [dW_head (width) | db_layer2 (width) |
// db_head (1) | 3 zeros], summed by the caller
template <typename T, int NC>
__global__ __launch_bounds__(256) void k_disc_head_bwd(const T *__restrict__ h, int64_t ldh, int64_t rows, int width,
                                                       const float *__restrict__ w, const float *__restrict__ gl,
                                                       T *__restrict__ g, int64_t ldg, float *__restrict__ parts) {
  __shared__ float red[4][2 * 64 * 8 * NC + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wv[NC][8], dw[NC][8], db[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = (lane + 64 * c) * 8 + e;
      wv[c][e] = col < width ? w[col] : 0.0f;
      dw[c][e] = 0.0f;
      db[c][e] = 0.0f;
    }
  float dbh = 0.0f;
  const int64_t r0 = (int64_t)blockIdx.x * kDiscRowsPerBlock + wave * (kDiscRowsPerBlock / 4);
  for (int rr = 0; rr < kDiscRowsPerBlock / 4; ++rr) {
    const int64_t r = r0 + rr;
    if (r >= rows) break;
    const float gr = gl[r];
    dbh += gr;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 8;
      if (col < width) {
        float v[8];
        disc_load8(h + r * ldh + col, v);
        T o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = v[e] > 0.0f ? gr * wv[c][e] : 0.0f;
          o[e] = (T)gv;
          dw[c][e] += gr * v[e];
          db[c][e] += gv;
        }
        uint4 raw;
        __builtin_memcpy(&raw, o, sizeof(raw));
        *reinterpret_cast<uint4 *>(g + r * ldg + col) = raw;
      }
    }
  }
  // the 4 waves' partials through LDS, one row per block
  constexpr int W = 64 * 8 * NC;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = (lane + 64 * c) * 8 + e;
      red[wave][col] = dw[c][e];
      red[wave][W + col] = db[c][e];
    }
  if (lane == 0) red[wave][2 * W] = dbh;
  __syncthreads();
  float *out = parts + (int64_t)blockIdx.x * (2 * width + 4);
  for (int j = threadIdx.x; j < 2 * width + 4; j += 256) {
    if (j > 2 * width) {
      out[j] = 0.0f;
      continue;
    }
    const int src = j < width ? j : (j < 2 * width ? W + (j - width) : 2 * W);
    out[j] = red[0][src] + red[1][src] + red[2][src] + red[3][src];
  }
}

template <typename T>
static void launch_head(bool fwd, int64_t blocks, hipStream_t st, const void *h, int64_t ldh, int64_t rows, int width,
                        const float *w, const float *b, float *logits, float *reward, const float *gl, void *g,
                        int64_t ldg, float *parts) {
  const T *ht = static_cast<const T *>(h);
  T *gt = static_cast<T *>(g);
  const dim3 grid((unsigned)blocks), block(256);
  if (fwd) {
    if (width <= 512)
      hipLaunchKernelGGL((k_disc_head_fwd<T, 1>), grid, block, 0, st, ht, ldh, rows, width, w, b, logits, reward);
    else
      hipLaunchKernelGGL((k_disc_head_fwd<T, 2>), grid, block, 0, st, ht, ldh, rows, width, w, b, logits, reward);
  } else {
    if (width <= 512)
      hipLaunchKernelGGL((k_disc_head_bwd<T, 1>), grid, block, 0, st, ht, ldh, rows, width, w, gl, gt, ldg, parts);
    else
      hipLaunchKernelGGL((k_disc_head_bwd<T, 2>), grid, block, 0, st, ht, ldh, rows, width, w, gl, gt, ldg, parts);
  }
}

static int head_checks(const void *h, int64_t ldh, int64_t rows, int32_t width, int32_t dtype) {
  PHC_REQUIRE(h, "disc_head: null activation");
  PHC_REQUIRE(rows >= 0 && width >= 8 && width <= 1024 && width % 8 == 0, "disc_head: width must be 8..1024 and a multiple of 8");
  PHC_REQUIRE(ldh >= width && ldh % 8 == 0, "disc_head: ldh must cover the width and be a multiple of 8");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(h) & 15) == 0, "disc_head: activation must be 16-byte aligned");
  PHC_REQUIRE(dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "disc_head: dtype must be f16 or bf16");
  return PHC_OK;
}

}  // namespace phc

using namespace phc;

extern "C" int64_t phc_disc_head_bwd_blocks(int64_t rows) {
  return rows <= 0 ? 0 : (rows + kDiscRowsPerBlock - 1) / kDiscRowsPerBlock;
}

extern "C" int phc_disc_head_fwd(const void *h, int64_t ldh, int64_t rows, int32_t width, int32_t dtype,
                                 const float *w, const float *b, float *logits, float *reward, void *stream) {
  const int rc = head_checks(h, ldh, rows, width, dtype);
  if (rc != PHC_OK) return rc;
  PHC_REQUIRE(w && b && (logits || reward), "disc_head_fwd: null argument");
  if (rows == 0) return PHC_OK;
  const int64_t blocks = phc_disc_head_bwd_blocks(rows);
  PHC_REQUIRE(blocks < (1ll << 31), "disc_head_fwd: too many rows");
  if (dtype == PHC_DT_F16)
    launch_head<_Float16>(true, blocks, as_stream(stream), h, ldh, rows, width, w, b, logits, reward, nullptr,
                          nullptr, 0, nullptr);
  else
    launch_head<__bf16>(true, blocks, as_stream(stream), h, ldh, rows, width, w, b, logits, reward, nullptr,
                        nullptr, 0, nullptr);
  return check_launch("disc_head_fwd");
}

extern "C" int phc_disc_head_bwd(const void *h, int64_t ldh, int64_t rows, int32_t width, int32_t dtype,
                                 const float *w, const float *grad_logits, void *grad_h, int64_t ldg, float *parts,
                                 void *stream) {
  const int rc = head_checks(h, ldh, rows, width, dtype);
  if (rc != PHC_OK) return rc;
  PHC_REQUIRE(w && grad_logits && grad_h && parts, "disc_head_bwd: null argument");
  PHC_REQUIRE(ldg >= width && ldg % 8 == 0 && (reinterpret_cast<uintptr_t>(grad_h) & 15) == 0,
              "disc_head_bwd: grad_h must be 16-byte aligned with ldg >= width, % 8");
  if (rows == 0) return PHC_OK;
  const int64_t blocks = phc_disc_head_bwd_blocks(rows);
  PHC_REQUIRE(blocks < (1ll << 31), "disc_head_bwd: too many rows");
  if (dtype == PHC_DT_F16)
    launch_head<_Float16>(false, blocks, as_stream(stream), h, ldh, rows, width, w, nullptr, nullptr, nullptr,
                          grad_logits, grad_h, ldg, parts);
  else
    launch_head<__bf16>(false, blocks, as_stream(stream), h, ldh, rows, width, w, nullptr, nullptr, nullptr,
                        grad_logits, grad_h, ldg, parts);
  return check_launch("disc_head_bwd");
}
