// phc_ppo.hip — the PPO minibatch objective (R21) as two kernels instead of ~60 small torch ops.
//
// clean_pufferl/core.py:298-352 (+ policies/phc_policy.py bound loss, pufferlib sample_logits
// log-prob / entropy of the fixed-sigma Normal): per row r with mu[r, :], action a[r, :]
//   lp     = sum_j ( -(a - mu)^2 / (2 sigma^2) - log sigma - log sqrt(2 pi) )
//   ratio  = exp(lp - lp_old);  A = (adv - mean) / (std + 1e-8)
//   pg     = mean_r max(-A ratio, -A clamp(ratio, 1 - c, 1 + c))
//   v      = mean_r max((v - R)^2, (v_old + clamp(v - v_old, -vc, vc) - R)^2)   (clip_vloss)
//   ent    = mean_r sum_j (0.5 + log sqrt(2 pi) + log sigma)
//   bound  = mean_{r,j} (mu > b) (mu - b)^2 + (mu < -b) (mu + b)^2
//   loss   = pg - ent_coef ent + vf_coef v + bound_coef bound
// plus the logged statistics (old_approx_kl, approx_kl, clipfrac).  The forward saves two
// per-row coefficients (d pg / d lp, d v / d value); the backward forms d loss / d mu and
// d loss / d value from them.  torch.maximum's tie rule (gradient split evenly) and clamp's
// inclusive bounds are reproduced.  Statistics reduce through per-block partials (no atomics).
#include "phc_common.h"

namespace phc {

constexpr int kPpoBlock = 256;
constexpr int kPpoWaveRows = 16;                          // k_ppo_fwd: rows per wave
constexpr int kPpoRows = kPpoWaveRows * kPpoBlock / 64;   // k_ppo_fwd: rows per block
constexpr int kPpoStats = PHC_PPO_STATS;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))

struct PpoArgs {
  const float *mu, *log_sigma, *actions, *old_logprob, *adv, *adv_mean_std, *value, *old_value, *returns;
  int64_t m;
  int a;
  phc_ppo_coefs c;
};

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// d max(x, y) / dx and / dy with torch.maximum's rule: ties split the gradient evenly
__device__ __forceinline__ void dmax(float x, float y, float *gx, float *gy) {
  if (x > y) { *gx = 1.0f; *gy = 0.0f; }
  else if (x < y) { *gx = 0.0f; *gy = 1.0f; }
  else { *gx = 0.5f; *gy = 0.5f; }
}

// one wave per kPpoWaveRows rows: the per-action log-prob / bound terms of a row are formed with
// the actions across the lanes (coalesced row reads) and summed by a butterfly; lane i keeps row
// i's sums, then lanes 0..kPpoWaveRows-1 finish their rows
__device__ __forceinline__ float ppo_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kPpoBlock) void k_ppo_fwd(PpoArgs p, float *__restrict__ row_coef,
                                                       float *__restrict__ partial) {
  __shared__ float red[kPpoStats][kPpoBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t rbase = (int64_t)blockIdx.x * kPpoRows + wv * kPpoWaveRows;
  const int64_t r = rbase + lane;
  // per-action constants of the fixed-sigma Normal (std = exp(sigma), phc_policy.py decode_actions;
  // Normal.log_prob / entropy use scale.log())
  float var[2], ls[2];
  bool act_ok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = lane + 64 * h;
    act_ok[h] = j < p.a;
    const float sg = act_ok[h] ? expf(p.log_sigma[j]) : 1.0f;
    ls[h] = logf(sg);
    var[h] = sg * sg;
  }
  const float ent = ppo_wave_sum((act_ok[0] ? 0.5f + kLogSqrt2Pi + ls[0] : 0.0f) +
                                 (act_ok[1] ? 0.5f + kLogSqrt2Pi + ls[1] : 0.0f));
  const float b = p.c.soft_bound;
  float lp = 0.0f, bound = 0.0f;
  // every load of the wave's rows first, unconditionally (clamped indices, masked below): a load
  // behind a per-row condition makes hipcc branch around it and wait vmcnt(0) per row
  float mv[kPpoWaveRows][2], av[kPpoWaveRows][2];
#pragma unroll
  for (int i = 0; i < kPpoWaveRows; ++i) {
    const int64_t row = rbase + i < p.m ? rbase + i : p.m - 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = act_ok[h] ? lane + 64 * h : 0;
      mv[i][h] = p.mu[row * p.a + j];
      av[i][h] = p.actions[row * p.a + j];
    }
  }
  const int64_t rr = r < p.m ? r : p.m - 1;  // this lane's row of the tail below (lanes < kPpoWaveRows)
  const float r_old_lp = p.old_logprob[rr], r_adv = p.adv[rr], r_v = p.value[rr], r_ret = p.returns[rr];
  const float r_old_v = p.old_value[rr];
#pragma unroll
  for (int i = 0; i < kPpoWaveRows; ++i) {
    const int64_t row = rbase + i;
    const bool row_ok = row < p.m;  // wave-uniform
    float tl = 0.0f, tb = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!act_ok[h] || !row_ok) continue;
      const float m = mv[i][h];
      const float d = av[i][h] - m;
      tl += -(d * d) / (2.0f * var[h]) - ls[h] - kLogSqrt2Pi;
      tb += m > b ? (m - b) * (m - b) : (m < -b ? (m + b) * (m + b) : 0.0f);
    }
    tl = ppo_wave_sum(tl);
    tb = ppo_wave_sum(tb);
    if (lane == i) {
      lp = tl;
      bound = tb;
    }
  }
  float s[kPpoStats];
#pragma unroll
  for (int k = 0; k < kPpoStats; ++k) s[k] = 0.0f;
  if (lane < kPpoWaveRows && r < p.m) {
    const float logratio = lp - r_old_lp;
    const float ratio = expf(logratio);
    const float A = (r_adv - p.adv_mean_std[0]) / (p.adv_mean_std[1] + 1e-8f);
    const float lo = 1.0f - p.c.clip_coef, hi = 1.0f + p.c.clip_coef;
    const float t1 = -A * ratio, t2 = -A * clampf(ratio, lo, hi);
    float g1, g2;
    dmax(t1, t2, &g1, &g2);
    const float inside = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
    const float dpg_dratio = -A * g1 + -A * inside * g2;  // per row, before the 1/M of the mean
    const float v = r_v, ret = r_ret;
    float vl, dv;
    if (p.c.clip_vloss) {
      const float vu = (v - ret) * (v - ret);
      const float dvv = v - r_old_v;
      const float vcl = r_old_v + clampf(dvv, -p.c.vf_clip_coef, p.c.vf_clip_coef);
      const float vc = (vcl - ret) * (vcl - ret);
      float gu, gc;
      dmax(vu, vc, &gu, &gc);
      const float in_v = (dvv >= -p.c.vf_clip_coef && dvv <= p.c.vf_clip_coef) ? 1.0f : 0.0f;
      vl = vu > vc ? vu : vc;
      dv = gu * 2.0f * (v - ret) + gc * 2.0f * (vcl - ret) * in_v;
    } else {
      vl = (v - ret) * (v - ret);
      dv = 2.0f * (v - ret);
    }
    row_coef[2 * r] = dpg_dratio * ratio;  // d pg_row / d lp
    row_coef[2 * r + 1] = dv;              // d v_row / d value
    s[0] = t1 > t2 ? t1 : t2;
    s[1] = vl;
    s[2] = ent;
    s[3] = -logratio;
    s[4] = (ratio - 1.0f) - logratio;
    s[5] = fabsf(ratio - 1.0f) > p.c.clip_coef ? 1.0f : 0.0f;
    s[6] = bound;
  }
  // block reduction: wave sums by butterfly, then the 4 wave partials
#pragma unroll
  for (int k = 0; k < kPpoStats; ++k) {
    const float v = ppo_wave_sum(s[k]);
    if (lane == 0) red[k][wv] = v;
  }
  __syncthreads();
  if (threadIdx.x < kPpoStats) {
    const int k = threadIdx.x;
    partial[(int64_t)blockIdx.x * kPpoStats + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
}

// stats[0] = loss, then pg, v, ent, old_approx_kl, approx_kl, clipfrac, bound (means): 256
// threads accumulate strided block partials in double, then one wave adds the 256 sums in order
__global__ __launch_bounds__(256) void k_ppo_reduce(const float *__restrict__ partial, int blocks, int64_t m, int a,
                                                    phc_ppo_coefs c, float *__restrict__ stats,
                                                    double *__restrict__ stats_acc) {
  __shared__ double red[kPpoStats][256];
  double acc[kPpoStats];
#pragma unroll
  for (int k = 0; k < kPpoStats; ++k) acc[k] = 0.0;
  for (int i = threadIdx.x; i < blocks; i += 256)
#pragma unroll
    for (int k = 0; k < kPpoStats; ++k) acc[k] += partial[(int64_t)i * kPpoStats + k];
#pragma unroll
  for (int k = 0; k < kPpoStats; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int k = threadIdx.x;
  float mean = 0.0f;
  if (k < kPpoStats) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += red[k][i];
    mean = (float)(k == 6 ? t / ((double)m * a) : t / (double)m);
    stats[1 + k] = mean;
    if (stats_acc) stats_acc[k] += (double)mean;  // the trainer's running sum over minibatches
  }
  const float pg = __shfl(mean, 0, 64), v = __shfl(mean, 1, 64), ent = __shfl(mean, 2, 64),
              bound = __shfl(mean, 6, 64);
  if (k == 0) stats[0] = pg - c.ent_coef * ent + c.vf_coef * v + c.bound_coef * bound;
}

__global__ __launch_bounds__(kPpoBlock) void k_ppo_bwd(PpoArgs p, const float *__restrict__ row_coef,
                                                       const float *__restrict__ grad_loss, float *__restrict__ gmu,
                                                       float *__restrict__ gvalue) {
  const int64_t i = (int64_t)blockIdx.x * kPpoBlock + threadIdx.x;  // element of [m, a]
  const float gl = grad_loss[0];
  const float inv_m = 1.0f / (float)p.m;
  if (i < p.m * p.a) {
    const int64_t r = i / p.a;
    const int j = (int)(i - r * p.a);
    const float sg = expf(p.log_sigma[j]);
    const float var = sg * sg;
    const float mu = p.mu[i];
    const float d = p.actions[i] - mu;
    const float b = p.c.soft_bound;
    const float db = mu > b ? 2.0f * (mu - b) : (mu < -b ? 2.0f * (mu + b) : 0.0f);
    gmu[i] = gl * (row_coef[2 * r] * inv_m * (d / var) +
                   p.c.bound_coef * db * (1.0f / ((float)p.m * (float)p.a)));
  }
  if (i < p.m) gvalue[i] = gl * p.c.vf_coef * row_coef[2 * i + 1] * inv_m;
}

static int check_ppo(const PpoArgs &p) {
  PHC_REQUIRE(p.m > 0 && p.a > 0, "ppo_loss: empty minibatch");
  PHC_REQUIRE(p.mu && p.log_sigma && p.actions && p.old_logprob && p.adv && p.adv_mean_std && p.value &&
                  p.old_value && p.returns,
              "ppo_loss: null input");
  return PHC_OK;
}

}  // namespace phc

using namespace phc;

extern "C" size_t phc_ppo_workspace_bytes(int64_t m) {
  return m <= 0 ? 0 : (size_t)((m + kPpoRows - 1) / kPpoRows) * kPpoStats * sizeof(float);
}

extern "C" int phc_ppo_loss_fwd(const float *mu, const float *log_sigma, const float *actions,
                                const float *old_logprob, const float *adv, const float *adv_mean_std,
                                const float *value, const float *old_value, const float *returns, int64_t m,
                                int32_t a, const phc_ppo_coefs *coefs, float *row_coef, float *stats,
                                double *stats_acc, void *workspace, void *stream) {
  PHC_REQUIRE(coefs && row_coef && stats && workspace, "ppo_loss_fwd: null output/workspace");
  const PpoArgs p{mu, log_sigma, actions, old_logprob, adv, adv_mean_std, value, old_value, returns, m, a, *coefs};
  if (int rc = check_ppo(p)) return rc;
  const int blocks = (int)((m + kPpoRows - 1) / kPpoRows);
  float *partial = static_cast<float *>(workspace);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_ppo_fwd, dim3(blocks), dim3(kPpoBlock), 0, st, p, row_coef, partial);
  hipLaunchKernelGGL(k_ppo_reduce, dim3(1), dim3(256), 0, st, partial, blocks, m, (int)a, *coefs, stats, stats_acc);
  return check_launch("ppo_loss_fwd");
}

extern "C" int phc_ppo_loss_bwd(const float *mu, const float *log_sigma, const float *actions,
                                const float *row_coef, const float *grad_loss, int64_t m, int32_t a,
                                const phc_ppo_coefs *coefs, float *grad_mu, float *grad_value, void *stream) {
  PHC_REQUIRE(coefs && row_coef && grad_loss && grad_mu && grad_value && mu && log_sigma && actions,
              "ppo_loss_bwd: null argument");
  PHC_REQUIRE(m > 0 && a > 0, "ppo_loss_bwd: empty minibatch");
  PpoArgs p{};
  p.mu = mu;
  p.log_sigma = log_sigma;
  p.actions = actions;
  p.m = m;
  p.a = a;
  p.c = *coefs;
  const int64_t n = m * a;
  hipLaunchKernelGGL(k_ppo_bwd, dim3((unsigned)((n + kPpoBlock - 1) / kPpoBlock)), dim3(kPpoBlock), 0,
                     as_stream(stream), p, row_coef, grad_loss, grad_mu, grad_value);
  return check_launch("ppo_loss_bwd");
}
