// phc_optim.hip — the PPO minibatch update tail (R21) on flat fp32 buffers: gradient
// unscaling + per-parameter norms + global-norm clipping + Adam, with the loss-scale update.
//
// Reference (clean_pufferl/core.py:360-372): loss.backward(); clip_grad_norm_(params,
// max_grad_norm); optimizer.step() with torch.optim.Adam(lr, eps=1e-5) (betas 0.9 / 0.999); the
// logged "before clip" gradient norm is the sum of per-parameter norms.  With fp16 operands the
// loss is scaled first and the update follows torch.amp.GradScaler: gradients unscaled by 1/S,
// the step skipped (and S halved) when any gradient is inf / nan, S doubled after 2000 clean
// steps.  Here: the parameters, gradients and Adam moments are each ONE flat buffer, so the tail
// is three launches (segment partial sums, a one-block finish that also advances the Adam step
// and the scaler, the Adam update) instead of torch's multi-tensor norm / clip / unscale / Adam
// launches.  Reductions run in a fixed order (no atomics): results are deterministic.
#include "phc_common.h"

namespace phc {

constexpr int kOptBlock = 256;

// partial sums of squares (double) and a non-finite flag per block of the flat gradient; the
// block table maps block i -> [start, end) inside one parameter segment
__global__ __launch_bounds__(kOptBlock) void k_grad_partials(const float *__restrict__ g,
                                                             const int64_t *__restrict__ blk_range,
                                                             double *__restrict__ part_sq,
                                                             int *__restrict__ part_bad) {
  __shared__ double red[kOptBlock / 64];
  __shared__ int bad_s[kOptBlock / 64];
  const int64_t s = blk_range[2 * blockIdx.x], e = blk_range[2 * blockIdx.x + 1];
  double acc = 0.0;
  int bad = 0;
  for (int64_t i = s + threadIdx.x; i < e; i += kOptBlock) {
    const float v = g[i];
    bad |= !__builtin_isfinite(v);
    acc += (double)v * (double)v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    acc += __shfl_xor(acc, o, 64);
    bad |= __shfl_xor(bad, o, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[w] = acc;
    bad_s[w] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part_sq[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
    part_bad[blockIdx.x] = bad_s[0] | bad_s[1] | bad_s[2] | bad_s[3];
  }
}

// one wave: per-segment norms (segment j owns blocks [seg_blk[j], seg_blk[j+1])), clip
// coefficient, skip decision, loss-scale update, Adam step / bias corrections -> st
__global__ __launch_bounds__(64) void k_opt_finish(const double *__restrict__ part_sq, const int *__restrict__ part_bad,
                                                   const int32_t *__restrict__ seg_blk, int nseg,
                                                   phc_adam_params hp, phc_opt_state *__restrict__ st,
                                                   float *__restrict__ norm_out) {
  const int lane = threadIdx.x;
  const float inv = hp.use_loss_scale ? 1.0f / st->loss_scale : 1.0f;
  double tot = 0.0, norm_sum = 0.0;
  int bad = 0;
  for (int j = lane; j < nseg; j += 64) {  // segment sums in block order
    double sq = 0.0;
    for (int b = seg_blk[j]; b < seg_blk[j + 1]; ++b) {
      sq += part_sq[b];
      bad |= part_bad[b];
    }
    tot += sq;
    norm_sum += sqrt(sq) * (double)inv;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    tot += __shfl_xor(tot, o, 64);
    norm_sum += __shfl_xor(norm_sum, o, 64);
    bad |= __shfl_xor(bad, o, 64);
  }
  if (lane != 0) return;
  // clip_grad_norm_: coefficient from the global norm of the (unscaled) gradients
  const float total_norm = (float)(sqrt(tot) * (double)inv);
  float clip = hp.max_norm / (total_norm + 1e-6f);
  clip = clip < 1.0f ? clip : 1.0f;
  int skip = 0;
  if (hp.use_loss_scale) {  // torch.amp.GradScaler.update
    if (bad) {
      skip = 1;
      st->loss_scale *= hp.backoff_factor;
      st->growth_tracker = 0;
    } else if (++st->growth_tracker == hp.growth_interval) {
      st->loss_scale *= hp.growth_factor;
      st->growth_tracker = 0;
    }
    st->skipped += skip;
  }
  if (!skip) st->step += 1;
  const double t = (double)st->step;
  const double bc1 = 1.0 - pow((double)hp.beta1, t), bc2 = 1.0 - pow((double)hp.beta2, t);
  st->grad_mul = inv * clip;
  st->step_size = (float)((double)hp.lr / bc1);
  st->bc2_sqrt = (float)sqrt(bc2);
  st->skip = skip;
  if (norm_out) {
    norm_out[0] = (float)norm_sum;
    norm_out[1] = total_norm;
  }
}

// torch.optim.Adam (fused form): m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
// p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps), on g = grad * grad_mul
__global__ __launch_bounds__(kOptBlock) void k_adam(float *__restrict__ p, const float *__restrict__ g,
                                                    float *__restrict__ m, float *__restrict__ v, int64_t n,
                                                    phc_adam_params hp, const phc_opt_state *__restrict__ st) {
  if (st->skip) return;
  const float gm = st->grad_mul, ss = st->step_size, bc2s = st->bc2_sqrt;
  const float b1 = hp.beta1, b2 = hp.beta2, eps = hp.eps;
  const int64_t stride = (int64_t)gridDim.x * kOptBlock * 4;
  for (int64_t i = ((int64_t)blockIdx.x * kOptBlock + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 pv = *reinterpret_cast<float4 *>(p + i);
      const float4 gv = *reinterpret_cast<const float4 *>(g + i);
      float4 mv = *reinterpret_cast<float4 *>(m + i);
      float4 vv = *reinterpret_cast<float4 *>(v + i);
      float *pp = &pv.x, *mm = &mv.x, *vq = &vv.x;
      const float *gg = &gv.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gk = gg[k] * gm;
        mm[k] = b1 * mm[k] + (1.0f - b1) * gk;
        vq[k] = b2 * vq[k] + (1.0f - b2) * gk * gk;
        pp[k] -= ss * mm[k] / (sqrtf(vq[k]) / bc2s + eps);
      }
      *reinterpret_cast<float4 *>(p + i) = pv;
      *reinterpret_cast<float4 *>(m + i) = mv;
      *reinterpret_cast<float4 *>(v + i) = vv;
    } else {
      for (int64_t j = i; j < n; ++j) {
        const float gk = g[j] * gm;
        m[j] = b1 * m[j] + (1.0f - b1) * gk;
        v[j] = b2 * v[j] + (1.0f - b2) * gk * gk;
        p[j] -= ss * m[j] / (sqrtf(v[j]) / bc2s + eps);
      }
    }
  }
}

}  // namespace phc

using namespace phc;

extern "C" int64_t phc_opt_block_elems(void) { return 16384; }

extern "C" int phc_opt_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                            const int64_t *blk_range, int32_t nblk, const int32_t *seg_blk, int32_t nseg,
                            const phc_adam_params *hp, phc_opt_state *state, float *norm_out, void *workspace,
                            void *stream) {
  PHC_REQUIRE(param && grad && exp_avg && exp_avg_sq && blk_range && seg_blk && hp && state && workspace,
              "opt_step: null argument");
  PHC_REQUIRE(n > 0 && nblk > 0 && nseg > 0, "opt_step: empty parameter set");
  PHC_REQUIRE(((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0,
              "opt_step: flat buffers must be 16-byte aligned");
  PHC_REQUIRE(!hp->use_loss_scale || hp->growth_interval > 0, "opt_step: bad loss-scale growth interval");
  hipStream_t st = as_stream(stream);
  double *part_sq = static_cast<double *>(workspace);
  int *part_bad = reinterpret_cast<int *>(part_sq + nblk);
  hipLaunchKernelGGL(k_grad_partials, dim3((unsigned)nblk), dim3(kOptBlock), 0, st, grad, blk_range, part_sq,
                     part_bad);
  hipLaunchKernelGGL(k_opt_finish, dim3(1), dim3(64), 0, st, part_sq, part_bad, seg_blk, (int)nseg, *hp, state,
                     norm_out);
  const int64_t quads = (n + 3) / 4;
  const int64_t blocks = std::min<int64_t>((quads + kOptBlock - 1) / kOptBlock, 4096);
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(kOptBlock), 0, st, param, grad, exp_avg, exp_avg_sq, n,
                     *hp, state);
  return check_launch("opt_step");
}

extern "C" size_t phc_opt_workspace_bytes(int32_t nblk) {
  return nblk <= 0 ? 0 : (size_t)nblk * (sizeof(double) + sizeof(int)) + 16;
}
