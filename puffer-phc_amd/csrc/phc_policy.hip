// phc_policy.hip — the PHCPolicy pieces around the twin-trunk GEMMs (R17, R19).
//
// phc_obs_half: RunningNorm forward (policies/running_norm.py:15-20: clamp((x - mean) /
//   sqrt(var + eps), -clip, clip)) of float32 observation rows — optionally gathered through a
//   row index (the trainer's env-major minibatch order, clean_pufferl/structs.py:146-160) —
//   rounded once into the f16 / bf16 operand of the first trunk GEMM, zero-padded to its
//   K % 64 == 0 width.  One pass replaces normalize + cast + pad (+ gather).
//
// phc_policy_act: the rollout's inference tail after the trunks (policies/phc_policy.py:40-61,
//   discriminator_policy.py:55-67, pufferlib sample_logits): per row, LayerNorm + SiLU of both
//   trunks' last Linear outputs, mu = W_mu h_actor + b_mu (512 -> 69), value = w_v h_critic + b_v,
//   action = mu + std * noise (std = exp(sigma), clamped to 1e-6 in deterministic mode),
//   logprob = sum_j Normal(mu, std).log_prob(action) — one launch instead of a LayerNorm kernel,
//   two GEMMs and ~20 elementwise / reduction launches.  Rows are independent; a 320-thread
//   block owns kActRows = 8 rows (512 blocks at 4096 rows, two or more per CU): LayerNorm one
//   row per wave (64 lanes x H/64 values, every row's loads issued before the first reduction),
//   the actor's h rows kept in LDS; thread (half, group, action) accumulates 4 rows x 1 action
//   of mu over one half of k in fp32, its W_mu row read as float4 straight from L2 (no staging
//   barriers), the two halves added through LDS.
#include "phc_common.h"
#include "phc_x3.h"

#include <cstdlib>

namespace phc {

// ----------------------------------------------------------------- obs_half --
template <typename T>
__global__ __launch_bounds__(256) void k_obs_half(const float *__restrict__ obs, const int64_t *__restrict__ rows,
                                                  int64_t m, int d, int ldo, const float *__restrict__ mean,
                                                  const float *__restrict__ var, float eps, float clip,
                                                  T *__restrict__ out) {
  const int chunks = ldo / 8;  // 8 outputs (16 B) per thread; m * chunks < 2^31 (host check)
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int)m * chunks) return;
  const int r = i / chunks;
  const int c0 = (i - r * chunks) * 8;
  const int64_t src = rows ? rows[r] : r;
  const float *x = obs + src * d;
  float xv[8], mv[8], vv[8];
  if (c0 + 8 <= d && (((uintptr_t)(x + c0)) & 7) == 0) {  // 8-byte aligned run: float2 loads
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float2 t = *reinterpret_cast<const float2 *>(x + c0 + e);
      xv[e] = t.x; xv[e + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = c0 + e < d ? x[c0 + e] : 0.0f;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mv[e] = c0 + e < d ? mean[c0 + e] : 0.0f;
    vv[e] = c0 + e < d ? var[c0 + e] : 1.0f;
  }
  T o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v = 0.0f;
    if (c0 + e < d) {
      v = (xv[e] - mv[e]) / sqrtf(vv[e] + eps);  // same expression as k_rms_normalize
      v = v < -clip ? -clip : (v > clip ? clip : v);
    }
    o[e] = (T)v;
  }
  uint4 raw;
  __builtin_memcpy(&raw, o, sizeof(raw));
  *reinterpret_cast<uint4 *>(out + (int64_t)r * ldo + c0) = raw;
}

// Row-per-wave form (ld_out <= 64 * 8 * NC: 1024 for the policy's 934-wide obs, 2048 for the
// 1960-wide AMP obs): lane l owns output chunks l + 64 c, c < NC (8 columns each) of every row its
// wave visits, so the per-column mean and sqrt(var + eps) are loaded and computed
// once per lane instead of once per element; rows_per_wave rows per wave, loads of two rows in
// flight.  Same expression as k_rms_normalize / the generic form: bit-identical outputs.
template <typename T, int NC>
__global__ __launch_bounds__(256) void k_obs_half_rows(const float *__restrict__ obs, const int64_t *__restrict__ rows,
                                                       int64_t m, int d, int ldo, const float *__restrict__ mean,
                                                       const float *__restrict__ var, float eps, float clip,
                                                       int rows_per_wave, T *__restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunks = ldo / 8;
  float mv[NC][8], dv[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = (lane + 64 * c) * 8 + e;
      const bool in = col < d;
      mv[c][e] = in ? mean[col] : 0.0f;
      dv[c][e] = in ? sqrtf(var[col] + eps) : 1.0f;
    }
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * rows_per_wave;
  // rows in groups of G: every load of a group is issued before the first is consumed
  constexpr int G = NC <= 2 ? 4 : 2;
  for (int rr0 = 0; rr0 < rows_per_wave; rr0 += G) {
    float xv[G][NC][8];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t r = row0 + rr0 + u;
      const bool live = rr0 + u < rows_per_wave && r < m;
      const float *x = obs + (live ? (rows ? rows[r] : r) : 0) * d;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int c0 = (lane + 64 * c) * 8;
        if (live && c0 + 8 <= d && (((uintptr_t)(x + c0)) & 7) == 0) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const float2 t = *reinterpret_cast<const float2 *>(x + c0 + e);
            xv[u][c][e] = t.x; xv[u][c][e + 1] = t.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) xv[u][c][e] = live && c0 + e < d ? x[c0 + e] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t r = row0 + rr0 + u;
      if (rr0 + u >= rows_per_wave || r >= m) break;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ch >= chunks) continue;
        const int c0 = ch * 8;
        T o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = 0.0f;
          if (c0 + e < d) {
            v = (xv[u][c][e] - mv[c][e]) / dv[c][e];  // same expression as k_rms_normalize
            v = v < -clip ? -clip : (v > clip ? clip : v);
          }
          o[e] = (T)v;
        }
        uint4 raw;
        __builtin_memcpy(&raw, o, sizeof(raw));
        *reinterpret_cast<uint4 *>(out + r * ldo + c0) = raw;
      }
    }
  }
}

// --------------------------------------------------------------- policy_act --
#ifndef PHC_ACT_ROWS
#define PHC_ACT_ROWS 8
#endif
constexpr int kActRows = PHC_ACT_ROWS;  // rows per block
constexpr int kActMaxA = 72;     // actions supported (PHC_NUM_DOF + 3)
constexpr int kActThreads = 320; // 2 k halves x 2 row groups x up to 72 actions (288), 5 waves
constexpr int kActTasks = (2 * kActRows + kActThreads / 64 - 1) / (kActThreads / 64);  // LN rows per wave
static_assert(2 * (kActRows / 4) * kActMaxA <= kActThreads, "one (k half, row group, action) per thread");
static_assert(4 * kActMaxA <= kActThreads && (kActRows / 2) * kActMaxA <= kActThreads, "transposed-W mu head threads");

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// LayerNorm + SiLU of one H-wide row held as C x 4 values per lane (lane-strided float4 chunks),
// the same arithmetic as k_ln_silu_fwd
template <int C>
__device__ __forceinline__ void ln_silu_row(float x[C][4], const float *__restrict__ gamma,
                                            const float *__restrict__ beta, int lane, float eps) {
  constexpr int H = C * 256;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < C; ++k) s += (x[k][0] + x[k][1]) + (x[k][2] + x[k][3]);
  const float mean = wave_sum(s) / (float)H;
  float v = 0.0f;
#pragma unroll
  for (int k = 0; k < C; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float dd = x[k][e] - mean;
      v += dd * dd;
    }
  const float rstd = rsqrtf(wave_sum(v) / (float)H + eps);
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int c = 4 * (lane + 64 * k);
    // gamma / beta may be views into a flat parameter buffer: 4-byte alignment only
    const float g4[4] = {gamma[c], gamma[c + 1], gamma[c + 2], gamma[c + 3]};
    const float b4[4] = {beta[c], beta[c + 1], beta[c + 2], beta[c + 3]};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ln = (x[k][e] - mean) * rstd * g4[e] + b4[e];
      x[k][e] = tail_silu(ln);
    }
  }
}

// The mu head, sample and log_prob from the transposed W_mu: thread (kq, j) accumulates all kActRows
// rows of action j over the k quarter kq — per k step one dword of W^T row k (the 4 x A threads of a
// step read one contiguous run of every W^T row: coalesced, where w_mu's rows put 64 lanes on 64
// lines) and one broadcast float4 of each h row from LDS; the quarters are summed in a fixed order.
#ifndef PHC_ACT_WT_UNROLL
#define PHC_ACT_WT_UNROLL 2  // 4-deep k steps per unrolled group (measured: 2 -> 25.0 us, 8 -> 26.8 us, 16 -> 27.1 us per 4096-row launch)
#endif
template <int H>
__device__ __forceinline__ void act_tail_wt(const phc_policy_act_args &a, float (*hs)[H], float (*part)[kActMaxA],
                                            int64_t r0, int tid) {
  __shared__ float quarter[4][kActRows][kActMaxA];
  const int A = a.num_actions;
  constexpr int KQ = H / 4;
  if (tid < 4 * A) {
    const int kq = tid / A, j = tid % A;
    float acc[kActRows];
#pragma unroll
    for (int r = 0; r < kActRows; ++r) acc[r] = 0.0f;
    const int64_t ld = a.ld_w_mu_t;
    const float *wt = a.w_mu_t + (int64_t)(kq * KQ) * ld + j;
#pragma unroll PHC_ACT_WT_UNROLL
    for (int kk = 0; kk < KQ; kk += 4) {
      const float w0 = wt[(kk + 0) * ld], w1 = wt[(kk + 1) * ld], w2 = wt[(kk + 2) * ld], w3 = wt[(kk + 3) * ld];
#pragma unroll
      for (int r = 0; r < kActRows; ++r) {
        const float4 h = *reinterpret_cast<const float4 *>(&hs[r][kq * KQ + kk]);
        acc[r] += h.x * w0;
        acc[r] += h.y * w1;
        acc[r] += h.z * w2;
        acc[r] += h.w * w3;
      }
    }
#pragma unroll
    for (int r = 0; r < kActRows; ++r) quarter[kq][r][j] = acc[r];
  }
  __syncthreads();
  // thread (g, j): rows 2g, 2g + 1 of action j
  const float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
  if (tid < (kActRows / 2) * A) {
    const int g = tid / A, j = tid % A;
    float sd = expf(a.log_sigma[j]);
    sd = sd > a.std_max ? a.std_max : sd;
    const float bj = a.b_mu[j];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = 2 * g + u;
      const int64_t row = r0 + rr;
      float lp = 0.0f;
      if (row < a.rows) {
        const float mu = ((quarter[0][rr][j] + quarter[1][rr][j]) + (quarter[2][rr][j] + quarter[3][rr][j])) + bj;
        const float act = mu + sd * a.noise[row * A + j];
        const float d = act - mu;
        lp = -(d * d) / (2.0f * (sd * sd)) - logf(sd) - kLogSqrt2Pi;
        a.actions[row * A + j] = act;
        if (a.mu) a.mu[row * A + j] = mu;
      }
      part[rr][j] = lp;
    }
  }
  __syncthreads();
  if (tid < kActRows && r0 + tid < a.rows) {
    float s = 0.0f;
    for (int jj = 0; jj < A; ++jj) s += part[tid][jj];
    a.logprob[r0 + tid] = s;
  }
}

template <int C>
__global__ __launch_bounds__(kActThreads) void k_policy_act(phc_policy_act_args a) {
  constexpr int H = C * 256;
  constexpr int kWaves = kActThreads / 64;
  __shared__ __attribute__((aligned(16))) float hs[kActRows][H];
  __shared__ float part[kActRows][kActMaxA];  // the second k half's mu partials, then log_prob terms
  __shared__ float red[kActRows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kActRows;
  const int A = a.num_actions;
  const float *y = a.trunk_out;

  // LayerNorm + SiLU: task q = (trunk, row) of the block, one wave per task; all of a wave's
  // row loads are issued before its first reduction
  float x[kActTasks][C][4];
#pragma unroll
  for (int t = 0; t < kActTasks; ++t) {
    const int q = wave + kWaves * t;
    const int grp = q / kActRows;
    const int64_t row = r0 + q % kActRows;
    if (q < 2 * kActRows && row < a.rows) {
      const float *src = y + ((int64_t)grp * a.rows + row) * H;
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const float4 v = *reinterpret_cast<const float4 *>(src + 4 * (lane + 64 * k));
        x[t][k][0] = v.x; x[t][k][1] = v.y; x[t][k][2] = v.z; x[t][k][3] = v.w;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < kActTasks; ++t) {
    const int q = wave + kWaves * t;
    const int grp = q / kActRows, rr = q % kActRows;
    if (q >= 2 * kActRows || r0 + rr >= a.rows) continue;
    ln_silu_row<C>(x[t], a.ln_gamma[grp], a.ln_beta[grp], lane, a.ln_eps);
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < C; ++k)
        *reinterpret_cast<float4 *>(&hs[rr][4 * (lane + 64 * k)]) =
            float4{x[t][k][0], x[t][k][1], x[t][k][2], x[t][k][3]};
    } else {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const float *w = a.w_value + 4 * (lane + 64 * k);
        s += x[t][k][0] * w[0] + x[t][k][1] * w[1] + x[t][k][2] * w[2] + x[t][k][3] * w[3];
      }
      s = wave_sum(s);
      if (lane == 0) red[rr] = s + a.b_value[0];
    }
  }
  __syncthreads();
  if (tid < kActRows && r0 + tid < a.rows) a.value[r0 + tid] = red[tid];
  if (a.w_mu_t) {
    act_tail_wt<H>(a, hs, part, r0, tid);
    return;
  }

  // mu head: thread (kh, g, j) owns rows 4g..4g+3 of action j over k in [kh H/2, (kh+1) H/2);
  // per 4-deep k step one float4 of its W_mu row (L2) and one broadcast float4 of each h row
  constexpr int kGroups = kActRows / 4;
  const int kh = tid / (kGroups * A), g = (tid / A) % kGroups, j = tid % A;
  const bool active = tid < 2 * kGroups * A;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (active) {
    const float *w = a.w_mu + (int64_t)j * H + kh * (H / 2);
    const float *h0 = &hs[4 * g][kh * (H / 2)];
    auto step = [&](int kk, float4 wv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float4 h = *reinterpret_cast<const float4 *>(h0 + r * H + kk);
        acc[r] += h.x * wv.x;
        acc[r] += h.y * wv.y;
        acc[r] += h.z * wv.z;
        acc[r] += h.w * wv.w;
      }
    };
    if ((reinterpret_cast<uintptr_t>(a.w_mu) & 15) == 0) {  // the aligned copy: one dwordx4 per step
#pragma unroll 8
      for (int kk = 0; kk < H / 2; kk += 4) step(kk, *reinterpret_cast<const float4 *>(w + kk));
    } else {  // a view into a flat parameter buffer: 4-byte alignment only
#pragma unroll 8
      for (int kk = 0; kk < H / 2; kk += 4) step(kk, float4{w[kk], w[kk + 1], w[kk + 2], w[kk + 3]});
    }
    if (kh == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) part[4 * g + r][j] = acc[r];
    }
  }
  __syncthreads();
  // action / logprob: the Normal's log_prob terms per (row, action), summed per row in a fixed
  // order (deterministic: a captured rollout graph and the eager step give identical bits)
  const float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
  float lp[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (active && kh == 0) {
    float sd = expf(a.log_sigma[j]);
    sd = sd > a.std_max ? a.std_max : sd;
    const float bj = a.b_mu[j];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * g + r;
      const int64_t row = r0 + rr;
      if (row >= a.rows) break;
      const float mu = (acc[r] + part[rr][j]) + bj;
      const float act = mu + sd * a.noise[row * A + j];
      const float d = act - mu;
      lp[r] = -(d * d) / (2.0f * (sd * sd)) - logf(sd) - kLogSqrt2Pi;
      a.actions[row * A + j] = act;
      if (a.mu) a.mu[row * A + j] = mu;
    }
  }
  __syncthreads();  // every mu partial has been read
  if (active && kh == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) part[4 * g + r][j] = lp[r];
  }
  __syncthreads();
  if (tid < kActRows && r0 + tid < a.rows) {
    float s = 0.0f;
    for (int jj = 0; jj < A; ++jj) s += part[tid][jj];
    a.logprob[r0 + tid] = s;
  }
}

// ------------------------------------------------------- policy_act, MFMA form --
// 16 rows per 512-thread workgroup (256 workgroups at 4096 rows: one per CU).  LayerNorm + SiLU as
// above (one (trunk, row) task per wave, 4 tasks per wave), the actor's h rows kept in LDS as fp32;
// then the mu head on the bf16 MFMA with three-way operand splits (phc_x3.h: fp32-class products):
// wave w takes the K slice [w H/8, (w + 1) H/8) of all 16 rows x 80 action columns (5 blocks of 16;
// columns past A multiply zeros), its W_mu fragments (lane (g, c): action 16 nb + c, 8 consecutive
// K) issued right after the trunk rows and LayerNorm parameters so they land during the LayerNorm,
// and split in registers (no staging of W); the 8 K-slice partials are added through LDS in a fixed
// order, then the Normal sample and log_prob as above.  Replaces the fp32-FMA head of k_policy_act
// (per-thread LDS broadcast reads + W row loads): 4096 rows 18.8-21.3 us standalone vs 24.6-29.0,
// 20.3-22.3 us vs 28.5 us inside the PPO rollout (tools/act_probe.py, profiles/r05r / r05s traces).
// PHC_ACT_X3=0 selects k_policy_act.
constexpr int kAx3Rows = 16, kAx3Waves = 8, kAx3Threads = kAx3Waves * 64, kAx3NB = kActMaxA / 16 + 1;
static_assert(kAx3NB * 16 >= kActMaxA, "action blocks cover every action");
static_assert(2 * kAx3Rows % kAx3Waves == 0, "LayerNorm tasks split evenly over the waves");

template <int C>
__global__ __launch_bounds__(kAx3Threads) void k_policy_act_x3(phc_policy_act_args a) {
  constexpr int H = C * 256, KW = H / kAx3Waves, KS = KW / 32, HP = H + 4, NB = kAx3NB;
  // K steps whose W fragments load before the LayerNorm
  constexpr int KPRE = C >= 3 ? 1 : (KS < 2 ? KS : 2);
  constexpr int kTasks = 2 * kAx3Rows / kAx3Waves;
  static_assert(KW % 32 == 0, "each wave's K slice is whole 32-deep MFMA steps");
  __shared__ __attribute__((aligned(16))) float hs[kAx3Rows][HP];  // +4 floats: conflict-free A reads
  __shared__ __attribute__((aligned(16))) float part[kAx3Waves][kAx3Rows][NB * 16];
  __shared__ float lpt[kAx3Rows][kActMaxA];
  __shared__ float red[kAx3Rows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * kAx3Rows;
  const int A = a.num_actions;
  const int kw0 = wave * KW;

  // W_mu fragments: rows clamped to A - 1 (loads stay in bounds), zeroed past A after they land
  const bool wvec = (reinterpret_cast<uintptr_t>(a.w_mu) & 15) == 0;  // uniform
  auto load_w = [&](int s, float4 (&wf)[NB][2]) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int act = 16 * nb + c;
      const float *wp = a.w_mu + (int64_t)(act < A ? act : A - 1) * H + kw0 + 32 * s + 8 * g;
      if (wvec) {
        wf[nb][0] = *reinterpret_cast<const float4 *>(wp);
        wf[nb][1] = *reinterpret_cast<const float4 *>(wp + 4);
      } else {
        wf[nb][0] = float4{wp[0], wp[1], wp[2], wp[3]};
        wf[nb][1] = float4{wp[4], wp[5], wp[6], wp[7]};
      }
    }
  };

  // load order = wait order (vmcnt counts in issue order): the trunk rows first, then the LayerNorm
  // parameters of both trunks (a wave's tasks span both) and w_value, then what is needed only after
  // the LayerNorm (W_mu fragments, the sampling inputs).
  // LayerNorm + SiLU: task q = (trunk, row), q = wave + kAx3Waves t; rows past the end leave zeros
  float x[kTasks][C][4];
#pragma unroll
  for (int t = 0; t < kTasks; ++t) {
    const int q = wave + kAx3Waves * t;
    const int grp = q / kAx3Rows;
    const int64_t row = r0 + q % kAx3Rows;
    if (row < a.rows) {
      const float *src = a.trunk_out + ((int64_t)grp * a.rows + row) * H;
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const float4 v = *reinterpret_cast<const float4 *>(src + 4 * (lane + 64 * k));
        x[t][k][0] = v.x; x[t][k][1] = v.y; x[t][k][2] = v.z; x[t][k][3] = v.w;
      }
    }
  }
  float gm[2][C][4], bt[2][C][4], wv[C][4];
#pragma unroll
  for (int k = 0; k < C; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = 4 * (lane + 64 * k) + e;  // parameter views may be 4-byte aligned only
      gm[0][k][e] = a.ln_gamma[0][col];
      gm[1][k][e] = a.ln_gamma[1][col];
      bt[0][k][e] = a.ln_beta[0][col];
      bt[1][k][e] = a.ln_beta[1][col];
      wv[k][e] = a.w_value[col];
    }
  const float bv = a.b_value[0];
  float4 wpre[KPRE][NB][2];
#pragma unroll
  for (int s = 0; s < KPRE; ++s) load_w(s, wpre[s]);
  // the sampling phase's inputs: thread item u = (row, action) i = tid + kAx3Threads u
  constexpr int kItems = (kAx3Rows * kActMaxA + kAx3Threads - 1) / kAx3Threads;
  float nz[kItems], lsg[kItems], bmu[kItems];
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = tid + kAx3Threads * u, rr = i / A, j = i - rr * A;
    const int64_t row = r0 + rr;
    const bool ok = i < kAx3Rows * A && row < a.rows;
    nz[u] = ok ? a.noise[row * A + j] : 0.0f;
    lsg[u] = ok ? a.log_sigma[j] : 0.0f;
    bmu[u] = ok ? a.b_mu[j] : 0.0f;
  }

#pragma unroll
  for (int t = 0; t < kTasks; ++t) {
    const int q = wave + kAx3Waves * t;
    const int grp = q / kAx3Rows, rr = q % kAx3Rows;  // grp: compile-time per t (kAx3Waves | kAx3Rows)
    if (r0 + rr >= a.rows) {
      if (grp == 0) {
#pragma unroll
        for (int k = 0; k < C; ++k) *reinterpret_cast<float4 *>(&hs[rr][4 * (lane + 64 * k)]) = float4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      continue;
    }
    // ln_silu_row's arithmetic with the parameters in registers
    float sm = 0.0f;
#pragma unroll
    for (int k = 0; k < C; ++k) sm += (x[t][k][0] + x[t][k][1]) + (x[t][k][2] + x[t][k][3]);
    const float mean = wave_sum(sm) / (float)H;
    float vr = 0.0f;
#pragma unroll
    for (int k = 0; k < C; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dd = x[t][k][e] - mean;
        vr += dd * dd;
      }
    const float rstd = rsqrtf(wave_sum(vr) / (float)H + a.ln_eps);
#pragma unroll
    for (int k = 0; k < C; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float ln = (x[t][k][e] - mean) * rstd * gm[grp][k][e] + bt[grp][k][e];
        x[t][k][e] = tail_silu(ln);
      }
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < C; ++k)
        *reinterpret_cast<float4 *>(&hs[rr][4 * (lane + 64 * k)]) = float4{x[t][k][0], x[t][k][1], x[t][k][2], x[t][k][3]};
    } else {
      float sv = 0.0f;
#pragma unroll
      for (int k = 0; k < C; ++k)
        sv += x[t][k][0] * wv[k][0] + x[t][k][1] * wv[k][1] + x[t][k][2] * wv[k][2] + x[t][k][3] * wv[k][3];
      sv = wave_sum(sv);
      if (lane == 0) red[rr] = sv + bv;
    }
  }
  __syncthreads();

  // mu partial over this wave's K slice: A = h rows (lane (g, c): row c, K 8 g .. + 7 of the step)
  x3f4 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = x3f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    float4 wl[NB][2];
    if (s >= KPRE) load_w(s, wl);
    const float4(&wf)[NB][2] = s < KPRE ? wpre[s < KPRE ? s : 0] : wl;
    X3 xs, ws[NB];
    const float *hp = &hs[c][kw0 + 32 * s + 8 * g];
    split3(*reinterpret_cast<const float4 *>(hp), *reinterpret_cast<const float4 *>(hp + 4), xs);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const bool live = 16 * nb + c < A;
      const float4 z4{0.0f, 0.0f, 0.0f, 0.0f};
      split3(live ? wf[nb][0] : z4, live ? wf[nb][1] : z4, ws[nb]);
    }
    mma_x3_n<NB>(&xs, ws, acc, true);
  }
  // lane (g, c) holds rows 4 g + e of action column 16 nb + c
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int e = 0; e < 4; ++e) part[wave][4 * g + e][16 * nb + c] = acc[nb][e];
  __syncthreads();

  // the 8 partials in a fixed order, + b_mu; sample and the Normal's log_prob terms
  const float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
#pragma unroll
  for (int u = 0; u < kItems; ++u) {
    const int i = tid + kAx3Threads * u;
    if (i >= kAx3Rows * A) break;
    const int rr = i / A, j = i - rr * A;
    const int64_t row = r0 + rr;
    float lp = 0.0f;
    if (row < a.rows) {
      const float s = ((part[0][rr][j] + part[1][rr][j]) + (part[2][rr][j] + part[3][rr][j])) +
                      ((part[4][rr][j] + part[5][rr][j]) + (part[6][rr][j] + part[7][rr][j]));
      const float mu = s + bmu[u];
      float sd = expf(lsg[u]);
      sd = sd > a.std_max ? a.std_max : sd;
      const float act = mu + sd * nz[u];
      const float d = act - mu;
      lp = -(d * d) / (2.0f * (sd * sd)) - logf(sd) - kLogSqrt2Pi;
      a.actions[row * A + j] = act;
      if (a.mu) a.mu[row * A + j] = mu;
    }
    lpt[rr][j] = lp;
  }
  __syncthreads();
  if (tid < kAx3Rows && r0 + tid < a.rows) {
    float s = 0.0f;
    for (int jj = 0; jj < A; ++jj) s += lpt[tid][jj];
    a.logprob[r0 + tid] = s;
    a.value[r0 + tid] = red[tid];
  }
}

}  // namespace phc

using namespace phc;

extern "C" int phc_obs_half(const float *obs, const int64_t *rows, int64_t m, int32_t d, const float *mean,
                            const float *var, float eps, float clip, void *out, int32_t ld_out, int32_t dtype,
                            void *stream) {
  PHC_REQUIRE(m >= 0 && d > 0 && ld_out >= d && ld_out % 8 == 0, "obs_half: bad shape (ld_out >= d, ld_out %% 8 == 0)");
  if (m == 0) return PHC_OK;
  PHC_REQUIRE(obs && mean && var && out, "obs_half: null argument");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(out) & 15) == 0, "obs_half: out must be 16-byte aligned");
  PHC_REQUIRE(dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "obs_half: dtype must be f16 or bf16");
  hipStream_t st = as_stream(stream);
  if (ld_out <= 2048) {  // row-per-wave form
    static const int rpw_forced = [] {  // tuning aid
      const char *e = getenv("PHC_OBS_RPW");
      return e ? atoi(e) : 0;
    }();
    // rows per wave: the per-column statistics are loaded once per wave, so a wave takes several rows
    // (4096-row rollout operand: 1 / 2 / 4 rows per wave measured 33.4 / 23.1 / 21.2 us)
    const int rpw = rpw_forced > 0 ? rpw_forced : (m >= 65536 ? 8 : (m >= 2048 ? 4 : 1));
    const int64_t blocks = (m + 4 * rpw - 1) / (4 * rpw);
    PHC_REQUIRE(blocks < (1ll << 31), "obs_half: too many rows");
    const dim3 grid((unsigned)blocks);
    if (dtype == PHC_DT_F16) {
      if (ld_out <= 1024)
        hipLaunchKernelGGL((k_obs_half_rows<_Float16, 2>), grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out,
                           mean, var, eps, clip, rpw, static_cast<_Float16 *>(out));
      else
        hipLaunchKernelGGL((k_obs_half_rows<_Float16, 4>), grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out,
                           mean, var, eps, clip, rpw, static_cast<_Float16 *>(out));
    } else {
      if (ld_out <= 1024)
        hipLaunchKernelGGL((k_obs_half_rows<__bf16, 2>), grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out,
                           mean, var, eps, clip, rpw, static_cast<__bf16 *>(out));
      else
        hipLaunchKernelGGL((k_obs_half_rows<__bf16, 4>), grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out,
                           mean, var, eps, clip, rpw, static_cast<__bf16 *>(out));
    }
    return check_launch("obs_half");
  }
  const int64_t threads = m * (ld_out / 8);
  PHC_REQUIRE(threads < (1ll << 31) - 256, "obs_half: too many rows");
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (dtype == PHC_DT_F16)
    hipLaunchKernelGGL(k_obs_half<_Float16>, grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out, mean, var,
                       eps, clip, static_cast<_Float16 *>(out));
  else
    hipLaunchKernelGGL(k_obs_half<__bf16>, grid, dim3(256), 0, st, obs, rows, m, (int)d, (int)ld_out, mean, var,
                       eps, clip, static_cast<__bf16 *>(out));
  return check_launch("obs_half");
}

extern "C" int phc_policy_act(const phc_policy_act_args *args, void *stream) {
  PHC_REQUIRE(args, "policy_act: null args");
  const phc_policy_act_args &a = *args;
  PHC_REQUIRE(a.trunk_out && a.ln_gamma[0] && a.ln_beta[0] && a.ln_gamma[1] && a.ln_beta[1] && a.w_mu && a.b_mu && a.w_value && a.b_value && a.log_sigma &&
                  a.noise && a.actions && a.logprob && a.value,
              "policy_act: null argument");
  PHC_REQUIRE(a.rows >= 0, "policy_act: bad rows");
  PHC_REQUIRE(a.hidden == 256 || a.hidden == 512 || a.hidden == 768 || a.hidden == 1024,
              "policy_act: hidden must be 256, 512, 768 or 1024");
  PHC_REQUIRE(a.num_actions >= 1 && a.num_actions <= kActMaxA, "policy_act: 1..%d actions", kActMaxA);
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(a.trunk_out) & 15) == 0, "policy_act: trunk_out must be 16-byte aligned");
  PHC_REQUIRE(!a.w_mu_t || (a.ld_w_mu_t >= a.num_actions && a.ld_w_mu_t % 4 == 0 &&
                            (reinterpret_cast<uintptr_t>(a.w_mu_t) & 15) == 0),
              "policy_act: w_mu_t must be 16-byte aligned with ld_w_mu_t >= num_actions, ld_w_mu_t %% 4 == 0");
  if (a.rows == 0) return PHC_OK;
  hipStream_t st = as_stream(stream);
  static const bool x3 = [] {  // A/B aid: PHC_ACT_X3=0 selects the fp32-FMA head (k_policy_act)
    const char *e = getenv("PHC_ACT_X3");
    return !(e && atoi(e) == 0);
  }();
  if (x3) {
    const dim3 gx((unsigned)((a.rows + kAx3Rows - 1) / kAx3Rows));
    switch (a.hidden / 256) {
      case 1: hipLaunchKernelGGL(k_policy_act_x3<1>, gx, dim3(kAx3Threads), 0, st, a); break;
      case 2: hipLaunchKernelGGL(k_policy_act_x3<2>, gx, dim3(kAx3Threads), 0, st, a); break;
      case 3: hipLaunchKernelGGL(k_policy_act_x3<3>, gx, dim3(kAx3Threads), 0, st, a); break;
      default: hipLaunchKernelGGL(k_policy_act_x3<4>, gx, dim3(kAx3Threads), 0, st, a); break;
    }
    return check_launch("policy_act");
  }
  const dim3 grid((unsigned)((a.rows + kActRows - 1) / kActRows));
  switch (a.hidden / 256) {
    case 1: hipLaunchKernelGGL(k_policy_act<1>, grid, dim3(kActThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_policy_act<2>, grid, dim3(kActThreads), 0, st, a); break;
    case 3: hipLaunchKernelGGL(k_policy_act<3>, grid, dim3(kActThreads), 0, st, a); break;
    default: hipLaunchKernelGGL(k_policy_act<4>, grid, dim3(kActThreads), 0, st, a); break;
  }
  return check_launch("policy_act");
}

