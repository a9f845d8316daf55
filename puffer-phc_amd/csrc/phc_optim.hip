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
// With p0 (the initial parameters) the block also sums (p - p0)^2 for the L2-init
// regulariser the reference logs every minibatch (core.py:352-359), on the parameters before
// this step's update, as the reference evaluates it.
__global__ __launch_bounds__(kOptBlock) void k_grad_partials(const float *__restrict__ g,
                                                             const int64_t *__restrict__ blk_range,
                                                             double *__restrict__ part_sq,
                                                             int *__restrict__ part_bad,
                                                             const float *__restrict__ p,
                                                             const float *__restrict__ p0,
                                                             double *__restrict__ part_l2) {
  __shared__ double red[kOptBlock / 64], red_l2[kOptBlock / 64];
  __shared__ int bad_s[kOptBlock / 64];
  const int64_t s = blk_range[2 * blockIdx.x], e = blk_range[2 * blockIdx.x + 1];
  double acc = 0.0, l2 = 0.0;
  int bad = 0;
  // scalar head up to a 16-B boundary, float4 body (16-B loads: the pass is HBM-bound over the 3
  // flat buffers), scalar tail; a fixed per-thread order, so the result stays deterministic
  auto one = [&](int64_t i) {
    const float v = g[i];
    bad |= !__builtin_isfinite(v);
    acc += (double)v * (double)v;
    if (p0) {
      const double d = (double)p[i] - (double)p0[i];
      l2 += d * d;
    }
  };
  auto four = [&](const float4 v, const float4 a, const float4 b) {
    bad |= !__builtin_isfinite(v.x) | !__builtin_isfinite(v.y) | !__builtin_isfinite(v.z) | !__builtin_isfinite(v.w);
    acc += ((double)v.x * (double)v.x + (double)v.y * (double)v.y) + ((double)v.z * (double)v.z + (double)v.w * (double)v.w);
    if (p0) {
      const double d0 = (double)a.x - (double)b.x, d1 = (double)a.y - (double)b.y;
      const double d2 = (double)a.z - (double)b.z, d3 = (double)a.w - (double)b.w;
      l2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  };
  const bool aligned = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(p) |
                         reinterpret_cast<uintptr_t>(p0)) & 15) == 0;  // uniform
  int64_t vs = aligned ? (s + 3) & ~(int64_t)3 : e;
  vs = vs < e ? vs : e;
  const int64_t ve = aligned ? vs + ((e - vs) & ~(int64_t)3) : vs;
  for (int64_t t = s + threadIdx.x; t < vs; t += kOptBlock) one(t);  // < 4 elements when aligned
  int64_t i = vs + 4 * (int64_t)threadIdx.x;
  if (p0) {  // uniform: no select around the loads (it would serialise them)
    // four 16-B loads per buffer in flight (12 per thread); the chunks are summed in the thread's
    // address order whatever the unroll, so the partials do not depend on it
    for (; i + 12 * kOptBlock < ve; i += 16 * kOptBlock) {
      float4 v[4], a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = *reinterpret_cast<const float4 *>(g + i + 4 * u * kOptBlock);
        a[u] = *reinterpret_cast<const float4 *>(p + i + 4 * u * kOptBlock);
        b[u] = *reinterpret_cast<const float4 *>(p0 + i + 4 * u * kOptBlock);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) four(v[u], a[u], b[u]);
    }
    for (; i < ve; i += 4 * kOptBlock)
      four(*reinterpret_cast<const float4 *>(g + i), *reinterpret_cast<const float4 *>(p + i),
           *reinterpret_cast<const float4 *>(p0 + i));
  } else {
    // the gradient alone: four 16-B loads per thread in flight (two left the pass latency-bound at
    // a quarter of HBM); the chunks are still summed in the thread's address order
    const float4 z4{0.0f, 0.0f, 0.0f, 0.0f};
    for (; i + 12 * kOptBlock < ve; i += 16 * kOptBlock) {
      const float4 v0 = *reinterpret_cast<const float4 *>(g + i);
      const float4 v1 = *reinterpret_cast<const float4 *>(g + i + 4 * kOptBlock);
      const float4 v2 = *reinterpret_cast<const float4 *>(g + i + 8 * kOptBlock);
      const float4 v3 = *reinterpret_cast<const float4 *>(g + i + 12 * kOptBlock);
      four(v0, z4, z4);
      four(v1, z4, z4);
      four(v2, z4, z4);
      four(v3, z4, z4);
    }
    for (; i < ve; i += 4 * kOptBlock) four(*reinterpret_cast<const float4 *>(g + i), z4, z4);
  }
  for (int64_t t = ve + threadIdx.x; t < e; t += kOptBlock) one(t);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    acc += __shfl_xor(acc, o, 64);
    l2 += __shfl_xor(l2, o, 64);
    bad |= __shfl_xor(bad, o, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[w] = acc;
    red_l2[w] = l2;
    bad_s[w] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part_sq[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
    part_bad[blockIdx.x] = bad_s[0] | bad_s[1] | bad_s[2] | bad_s[3];
    if (p0) part_l2[blockIdx.x] = ((red_l2[0] + red_l2[1]) + red_l2[2]) + red_l2[3];
  }
}

// per-segment norms (segment j owns blocks [seg_blk[j], seg_blk[j+1])), clip coefficient, skip
// decision, loss-scale update, Adam step / bias corrections -> st.  One 1024-thread block: wave w
// takes segments w, w + 16, ...; its lanes stride over the segment's block partials and reduce by
// butterfly, the 16 wave totals are added in wave order (a fixed order: deterministic)
constexpr int kFinThreads = 1024, kFinWaves = kFinThreads / 64;
__global__ __launch_bounds__(kFinThreads) void k_opt_finish(const double *__restrict__ part_sq,
                                                            const int *__restrict__ part_bad,
                                                            const double *__restrict__ part_l2,
                                                            const int64_t *__restrict__ blk_range,
                                                            const int32_t *__restrict__ seg_blk, int nseg,
                                                            phc_adam_params hp, phc_opt_state *__restrict__ st,
                                                            float *__restrict__ norm_out,
                                                            double *__restrict__ norm_acc) {
  __shared__ double s_tot[kFinWaves], s_norm[kFinWaves], s_l2[kFinWaves];
  __shared__ int s_bad[kFinWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float inv = hp.use_loss_scale ? 1.0f / st->loss_scale : 1.0f;
  double tot = 0.0, norm_sum = 0.0, l2 = 0.0;
  int bad = 0;
  for (int j = wave; j < nseg; j += kFinWaves) {
    double sq = 0.0, dl = 0.0;
    int bd = 0;
    for (int b = seg_blk[j] + lane; b < seg_blk[j + 1]; b += 64) {
      sq += part_sq[b];
      bd |= part_bad[b];
      if (part_l2) dl += part_l2[b];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      sq += __shfl_xor(sq, o, 64);
      dl += __shfl_xor(dl, o, 64);
      bd |= __shfl_xor(bd, o, 64);
    }
    tot += sq;
    norm_sum += sqrt(sq) * (double)inv;
    bad |= bd;
    if (part_l2 && seg_blk[j + 1] > seg_blk[j]) {  // mean over the parameter's elements
      const int64_t n = blk_range[2 * (seg_blk[j + 1] - 1) + 1] - blk_range[2 * seg_blk[j]];
      l2 += dl / (double)n;
    }
  }
  if (lane == 0) {
    s_tot[wave] = tot;
    s_norm[wave] = norm_sum;
    s_l2[wave] = l2;
    s_bad[wave] = bad;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  tot = norm_sum = l2 = 0.0;
  bad = 0;
  for (int w = 0; w < kFinWaves; ++w) {
    tot += s_tot[w];
    norm_sum += s_norm[w];
    l2 += s_l2[w];
    bad |= s_bad[w];
  }
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
  const float lr = hp.lr_from_state ? st->lr : hp.lr;
  st->step_size = (float)((double)lr / bc1);
  st->bc2_sqrt = (float)sqrt(bc2);
  st->skip = skip;
  if (norm_out) {
    norm_out[0] = (float)norm_sum;
    norm_out[1] = total_norm;
    if (part_l2) norm_out[2] = (float)l2;
    if (norm_acc) {  // the trainer's running sums of the logged row, as `acc += norm_out` would add them
      norm_acc[0] += (double)norm_out[0];
      norm_acc[1] += (double)norm_out[1];
      norm_acc[2] += (double)norm_out[2];
    }
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

// ---------------------------------------------------------------- reduce_into --
// dst[r, c] (+)= sum_{s < parts} src[s * part_stride + r * src_ld + c], parts summed in order:
// split-K weight-gradient partials (and plain strided copies) written straight into a flat
// gradient buffer's per-parameter views, many jobs per launch.
struct ReduceJobs {
  phc_reduce_job j[PHC_MAX_REDUCE_JOBS];
  int64_t first_block[PHC_MAX_REDUCE_JOBS + 1];
  int n;
};
constexpr int kRedThreads = 256, kRedPerThread = 4;

constexpr int kRedManyParts = 8;  // jobs with more parts split them over the block's 4 waves

__host__ __device__ inline int64_t red_elems_per_block(const phc_reduce_job &j) {
  return j.parts > kRedManyParts ? 64 : kRedThreads * kRedPerThread;
}

__global__ __launch_bounds__(kRedThreads) void k_reduce_into(ReduceJobs js) {
  int q = 0;
  while (q + 1 < js.n && (int64_t)blockIdx.x >= js.first_block[q + 1]) ++q;
  const phc_reduce_job &job = js.j[q];
  const int64_t total = job.rows * job.cols;
  if (job.parts > kRedManyParts) {  // uniform per block
    // many parts (fine split-K): one element per lane, the parts split into 4 contiguous ranges,
    // one per wave, each summed with 8 independent running sums (8 loads in flight per lane), the
    // 4 wave sums combined through LDS in a fixed order: deterministic, 4x shorter load chains
    __shared__ float red[kRedThreads / 64][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = ((int64_t)blockIdx.x - js.first_block[q]) * 64 + lane;
    const int per = (job.parts + 3) / 4, s0 = w * per, s1 = s0 + per < job.parts ? s0 + per : job.parts;
    float a8[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (i < total) {
      const int64_t r = i / job.cols, c = i - r * job.cols;
      const float *src = job.src + r * job.src_ld + c;
      int s = s0;
      // 16 loads in flight, added in the same order as 8 per step (bit-equal to that form)
      for (; s + 16 <= s1; s += 16) {
        float v[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) v[l] = src[(int64_t)(s + l) * job.part_stride];
#pragma unroll
        for (int l = 0; l < 8; ++l) a8[l] += v[l];
#pragma unroll
        for (int l = 0; l < 8; ++l) a8[l] += v[8 + l];
      }
      for (; s + 8 <= s1; s += 8) {
#pragma unroll
        for (int l = 0; l < 8; ++l) a8[l] += src[(int64_t)(s + l) * job.part_stride];
      }
      for (int l = 0; s + l < s1; ++l) a8[l] += src[(int64_t)(s + l) * job.part_stride];
    }
    red[w][lane] = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
    __syncthreads();
    if (w == 0 && i < total) {
      const float acc = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
      if (job.accumulate) job.dst[i] += acc;
      else job.dst[i] = acc;
    }
    return;
  }
  // few parts: every part of the thread's kRedPerThread elements loaded at clamped indices in one
  // memory round (a bounds break or a part loop with loads behind it serialised them), then summed
  // in part order as before
  const int64_t base = ((int64_t)blockIdx.x - js.first_block[q]) * kRedThreads * kRedPerThread + threadIdx.x;
  const int P = job.parts;
  float v[kRedPerThread][kRedManyParts], dv[kRedPerThread];
#pragma unroll
  for (int u = 0; u < kRedPerThread; ++u) {
    int64_t i = base + (int64_t)u * kRedThreads;
    i = i < total ? i : total - 1;
    const int64_t r = i / job.cols, c = i - r * job.cols;
    const float *src = job.src + r * job.src_ld + c;
#pragma unroll
    for (int sp = 0; sp < kRedManyParts; ++sp) v[u][sp] = src[(int64_t)(sp < P ? sp : P - 1) * job.part_stride];
    dv[u] = job.dst[i];  // read even when not accumulating: one round with the parts
  }
#pragma unroll
  for (int u = 0; u < kRedPerThread; ++u) {
    const int64_t i = base + (int64_t)u * kRedThreads;
    if (i >= total) break;
    float acc = v[u][0];
#pragma unroll
    for (int sp = 1; sp < kRedManyParts; ++sp)
      if (sp < P) acc += v[u][sp];
    job.dst[i] = job.accumulate ? dv[u] + acc : acc;
  }
}

// --------------------------------------------------------------- pack_weights --
// GEMM-operand refresh after an optimizer step: 64 x 64 tiles of every fp32 parameter staged
// through LDS (coalesced row reads), written converted row-wise (dst) and column-wise (dst_t: the
// transpose, coalesced along the source's rows).  One launch for all of a policy's operands.
struct PackJobs {
  phc_pack_job j[PHC_MAX_PACK_JOBS];
  int64_t first_block[PHC_MAX_PACK_JOBS + 1];
  int64_t tiles_c[PHC_MAX_PACK_JOBS];
  int n;
};
constexpr int kPackTile = 64, kPackThreads = 256;

__device__ __forceinline__ void pack_store(void *base, int64_t idx, int32_t dt, float v) {
  if (dt == PHC_DT_F16) static_cast<_Float16 *>(base)[idx] = (_Float16)v;  // RNE conversions
  else if (dt == PHC_DT_BF16) static_cast<__bf16 *>(base)[idx] = (__bf16)v;
  else static_cast<float *>(base)[idx] = v;
}

// 4 consecutive values at element idx (8-B aligned for half types, 16-B for fp32), or one by one
__device__ __forceinline__ void pack_store4(void *base, int64_t idx, int32_t dt, const float v[4], bool vec) {
  if (vec && dt == PHC_DT_F16) {
    _Float16 h[4] = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
    uint2 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    *reinterpret_cast<uint2 *>(static_cast<_Float16 *>(base) + idx) = raw;
  } else if (vec && dt == PHC_DT_BF16) {
    __bf16 h[4] = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    uint2 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    *reinterpret_cast<uint2 *>(static_cast<__bf16 *>(base) + idx) = raw;
  } else if (vec) {
    *reinterpret_cast<float4 *>(static_cast<float *>(base) + idx) = float4{v[0], v[1], v[2], v[3]};
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) pack_store(base, idx + q, dt, v[q]);
  }
}

// 64 x 64 tile per block: thread t owns columns 4 (t % 16) .. +3 of rows t / 16 + 16 i (16-B source
// loads, 8-B half stores), and for the transpose 4 consecutive tile rows of one column
__global__ __launch_bounds__(kPackThreads) void k_pack_weights(PackJobs js) {
  __shared__ float tile[kPackTile][kPackTile + 1];
  int q = 0;
  while (q + 1 < js.n && (int64_t)blockIdx.x >= js.first_block[q + 1]) ++q;
  const phc_pack_job &job = js.j[q];
  const int64_t t = (int64_t)blockIdx.x - js.first_block[q];
  const int64_t r0 = (t / js.tiles_c[q]) * kPackTile, c0 = (t % js.tiles_c[q]) * kPackTile;
  const int cq = (threadIdx.x & 15) * 4, rq = threadIdx.x >> 4;
  const int esz = job.dtype == PHC_DT_F32 ? 4 : 2;
  const bool src_vec = (job.src_ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(job.src) & 15) == 0);
  const bool dst_vec = job.dst && ((job.dst_ld * esz) % (4 * esz) == 0) &&
                       ((reinterpret_cast<uintptr_t>(job.dst) & (4 * esz - 1)) == 0);
#pragma unroll
  for (int i = 0; i < kPackTile / 16; ++i) {
    const int rr = rq + 16 * i;
    const int64_t r = r0 + rr, c = c0 + cq;
    float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool row_in = r < job.rows;
    const bool full = row_in && c + 3 < job.cols;
    if (full && src_vec) {
      const float4 x = *reinterpret_cast<const float4 *>(job.src + r * job.src_ld + c);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else if (row_in) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < job.cols) v[k] = job.src[r * job.src_ld + c + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rr][cq + k] = v[k];
    if (job.dst && row_in) {
      if (full) {
        pack_store4(job.dst, r * job.dst_ld + c, job.dtype, v, dst_vec);
      } else {
        for (int k = 0; k < 4; ++k)
          if (c + k < job.cols) pack_store(job.dst, r * job.dst_ld + c + k, job.dtype, v[k]);
      }
    }
  }
  if (!job.dst_t) return;
  __syncthreads();
  const bool t_vec = ((job.dst_t_ld * esz) % (4 * esz) == 0) &&
                     ((reinterpret_cast<uintptr_t>(job.dst_t) & (4 * esz - 1)) == 0);
#pragma unroll
  for (int i = 0; i < kPackTile / 16; ++i) {  // dst_t row c0 + cc, columns r0 + rq4 .. +3
    const int cc = (threadIdx.x >> 4) + 16 * i, rq4 = (threadIdx.x & 15) * 4;
    const int64_t c = c0 + cc, r = r0 + rq4;
    if (c >= job.cols) continue;
    const float v[4] = {tile[rq4][cc], tile[rq4 + 1][cc], tile[rq4 + 2][cc], tile[rq4 + 3][cc]};
    if (r + 3 < job.rows) {
      pack_store4(job.dst_t, c * job.dst_t_ld + r, job.dtype, v, t_vec);
    } else {
      for (int k = 0; k < 4; ++k)
        if (r + k < job.rows) pack_store(job.dst_t, c * job.dst_t_ld + r + k, job.dtype, v[k]);
    }
  }
}

// ------------------------------------------------- Adam + GEMM-operand copies (phc_opt_step_operands) --
// k_adam's arithmetic (same expression order: bit-identical parameters and moments) over a job table:
// tile jobs take a 64 x 64 tile of one parameter per workgroup (thread t: 4 consecutive columns of rows
// t / 16 + 16 i) and write the updated values converted row-wise (dst) and, through the LDS tile,
// transposed (dst_t) — what phc_pack_weights would write from the same fp32 values; flat jobs take
// 4,096 consecutive elements per workgroup.
__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, float gm, float ss, float bc2s, float b1,
                                         float b2, float eps) {
  const float gk = g * gm;
  m = b1 * m + (1.0f - b1) * gk;
  v = b2 * v + (1.0f - b2) * gk * gk;
  p -= ss * m / (sqrtf(v) / bc2s + eps);
}

constexpr int kAdamFlatElems = 4096;

__global__ __launch_bounds__(kPackThreads) void k_adam_ops(float *__restrict__ p, const float *__restrict__ g,
                                                           float *__restrict__ m, float *__restrict__ v,
                                                           const phc_adam_job *__restrict__ jobs, int njobs,
                                                           phc_adam_params hp, const phc_opt_state *__restrict__ st) {
  __shared__ float tile[kPackTile][kPackTile + 1];
  if (st->skip) return;
  // this workgroup's job: every thread tests one job's first block (one memory round, njobs <= 256)
  const int flag = (int)threadIdx.x < njobs && jobs[threadIdx.x].first_block <= (int64_t)blockIdx.x;
  const int q = __syncthreads_count(flag) - 1;
  const phc_adam_job &job = jobs[q];
  const int64_t t = (int64_t)blockIdx.x - job.first_block;
  const float gm = st->grad_mul, ss = st->step_size, bc2s = st->bc2_sqrt;
  const float b1 = hp.beta1, b2 = hp.beta2, eps = hp.eps;
  if (job.kind == PHC_ADAM_FLAT) {
    const int64_t e0 = job.off + t * kAdamFlatElems, e1 = job.off + job.rows;
#pragma unroll 4
    for (int k = 0; k < kAdamFlatElems / kPackThreads; ++k) {
      const int64_t e = e0 + threadIdx.x + (int64_t)k * kPackThreads;
      if (e < e1) {
        float pe = p[e], me = m[e], ve = v[e];
        adam_one(pe, g[e], me, ve, gm, ss, bc2s, b1, b2, eps);
        p[e] = pe; m[e] = me; v[e] = ve;
      }
    }
    return;
  }
  const int64_t r0 = (t / job.tiles_c) * kPackTile, c0 = (t % job.tiles_c) * kPackTile;
  const int cq = (threadIdx.x & 15) * 4, rq = threadIdx.x >> 4;
  const int esz = job.dtype == PHC_DT_F32 ? 4 : 2;
  // 16-B accesses when every tile row starts 16-B aligned (FlatGrads aligns each parameter's slice
  // to 64 B); 8-B pairs when rows are only 8-B aligned (the 934-column first layer)
  const bool vec = (job.off % 4 == 0) && (job.cols % 4 == 0);
  const bool vec2 = !vec && (job.off % 2 == 0) && (job.cols % 2 == 0);
  const bool dst_vec = job.dst && ((job.dst_ld * esz) % (4 * esz) == 0) &&
                       ((reinterpret_cast<uintptr_t>(job.dst) & (4 * esz - 1)) == 0);
#pragma unroll
  for (int i = 0; i < kPackTile / 16; ++i) {
    const int rr = rq + 16 * i;
    const int64_t r = r0 + rr, c = c0 + cq;
    float nv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool row_in = r < job.rows;
    const bool full = row_in && c + 3 < job.cols;
    const int64_t e = job.off + r * job.cols + c;
    if (full && vec) {
      float4 pv = *reinterpret_cast<float4 *>(p + e);
      const float4 gv = *reinterpret_cast<const float4 *>(g + e);
      float4 mv = *reinterpret_cast<float4 *>(m + e);
      float4 vv = *reinterpret_cast<float4 *>(v + e);
      float *pp = &pv.x, *mm = &mv.x, *vq = &vv.x;
      const float *gg = &gv.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        adam_one(pp[k], gg[k], mm[k], vq[k], gm, ss, bc2s, b1, b2, eps);
        nv[k] = pp[k];
      }
      *reinterpret_cast<float4 *>(p + e) = pv;
      *reinterpret_cast<float4 *>(m + e) = mv;
      *reinterpret_cast<float4 *>(v + e) = vv;
    } else if (full && vec2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float2 pv = *reinterpret_cast<float2 *>(p + e + 2 * h);
        const float2 gv = *reinterpret_cast<const float2 *>(g + e + 2 * h);
        float2 mv = *reinterpret_cast<float2 *>(m + e + 2 * h);
        float2 vv = *reinterpret_cast<float2 *>(v + e + 2 * h);
        adam_one(pv.x, gv.x, mv.x, vv.x, gm, ss, bc2s, b1, b2, eps);
        adam_one(pv.y, gv.y, mv.y, vv.y, gm, ss, bc2s, b1, b2, eps);
        nv[2 * h] = pv.x;
        nv[2 * h + 1] = pv.y;
        *reinterpret_cast<float2 *>(p + e + 2 * h) = pv;
        *reinterpret_cast<float2 *>(m + e + 2 * h) = mv;
        *reinterpret_cast<float2 *>(v + e + 2 * h) = vv;
      }
    } else if (row_in) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < job.cols) {
          float pe = p[e + k], me = m[e + k], ve = v[e + k];
          adam_one(pe, g[e + k], me, ve, gm, ss, bc2s, b1, b2, eps);
          p[e + k] = pe; m[e + k] = me; v[e + k] = ve;
          nv[k] = pe;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rr][cq + k] = nv[k];
    if (job.dst && row_in) {
      if (full) {
        pack_store4(job.dst, r * job.dst_ld + c, job.dtype, nv, dst_vec);
      } else {
        for (int k = 0; k < 4; ++k)
          if (c + k < job.cols) pack_store(job.dst, r * job.dst_ld + c + k, job.dtype, nv[k]);
      }
    }
  }
  if (!job.dst_t) return;
  __syncthreads();
  const bool t_vec = ((job.dst_t_ld * esz) % (4 * esz) == 0) &&
                     ((reinterpret_cast<uintptr_t>(job.dst_t) & (4 * esz - 1)) == 0);
#pragma unroll
  for (int i = 0; i < kPackTile / 16; ++i) {  // dst_t row c0 + cc, columns r0 + rq4 .. +3
    const int cc = (threadIdx.x >> 4) + 16 * i, rq4 = (threadIdx.x & 15) * 4;
    const int64_t c = c0 + cc, r = r0 + rq4;
    if (c >= job.cols) continue;
    const float w4[4] = {tile[rq4][cc], tile[rq4 + 1][cc], tile[rq4 + 2][cc], tile[rq4 + 3][cc]};
    if (r + 3 < job.rows) {
      pack_store4(job.dst_t, c * job.dst_t_ld + r, job.dtype, w4, t_vec);
    } else {
      for (int k = 0; k < 4; ++k)
        if (r + k < job.rows) pack_store(job.dst_t, c * job.dst_t_ld + r + k, job.dtype, w4[k]);
    }
  }
}

}  // namespace phc

using namespace phc;

extern "C" int phc_pack_weights(const phc_pack_job *jobs, int32_t num_jobs, void *stream) {
  PHC_REQUIRE(jobs && num_jobs >= 0 && num_jobs <= PHC_MAX_PACK_JOBS, "pack_weights: 0..%d jobs", PHC_MAX_PACK_JOBS);
  PackJobs js{};
  int64_t blocks = 0;
  int n = 0;
  for (int q = 0; q < num_jobs; ++q) {
    const phc_pack_job &j = jobs[q];
    PHC_REQUIRE(j.rows >= 0 && j.cols >= 0 && j.src_ld >= j.cols, "pack_weights: job %d bad shape", q);
    PHC_REQUIRE(j.dtype == PHC_DT_F32 || j.dtype == PHC_DT_F16 || j.dtype == PHC_DT_BF16,
                "pack_weights: job %d bad dtype", q);
    if (j.rows * j.cols == 0 || (!j.dst && !j.dst_t)) continue;
    PHC_REQUIRE(j.src, "pack_weights: job %d null source", q);
    PHC_REQUIRE(!j.dst || j.dst_ld >= j.cols, "pack_weights: job %d dst_ld < cols", q);
    PHC_REQUIRE(!j.dst_t || j.dst_t_ld >= j.rows, "pack_weights: job %d dst_t_ld < rows", q);
    js.j[n] = j;
    js.first_block[n] = blocks;
    js.tiles_c[n] = (j.cols + kPackTile - 1) / kPackTile;
    blocks += ((j.rows + kPackTile - 1) / kPackTile) * js.tiles_c[n];
    ++n;
  }
  if (n == 0) return PHC_OK;
  js.first_block[n] = blocks;
  js.n = n;
  PHC_REQUIRE(blocks < (1ll << 31), "pack_weights: too large");
  hipLaunchKernelGGL(k_pack_weights, dim3((unsigned)blocks), dim3(kPackThreads), 0, as_stream(stream), js);
  return check_launch("pack_weights");
}

extern "C" int phc_reduce_into(const phc_reduce_job *jobs, int32_t num_jobs, void *stream) {
  PHC_REQUIRE(jobs && num_jobs >= 0 && num_jobs <= PHC_MAX_REDUCE_JOBS, "reduce_into: 0..%d jobs",
              PHC_MAX_REDUCE_JOBS);
  ReduceJobs js{};
  int64_t blocks = 0;
  int n = 0;
  for (int q = 0; q < num_jobs; ++q) {
    const phc_reduce_job &j = jobs[q];
    PHC_REQUIRE(j.rows >= 0 && j.cols >= 0 && j.parts >= 1 && j.src_ld >= j.cols, "reduce_into: job %d bad shape", q);
    if (j.rows * j.cols == 0) continue;
    PHC_REQUIRE(j.src && j.dst, "reduce_into: job %d null pointer", q);
    js.j[n] = j;
    js.first_block[n] = blocks;
    blocks += (j.rows * j.cols + red_elems_per_block(j) - 1) / red_elems_per_block(j);
    ++n;
  }
  if (n == 0) return PHC_OK;
  js.first_block[n] = blocks;
  js.n = n;
  PHC_REQUIRE(blocks < (1ll << 31), "reduce_into: too large");
  hipLaunchKernelGGL(k_reduce_into, dim3((unsigned)blocks), dim3(kRedThreads), 0, as_stream(stream), js);
  return check_launch("reduce_into");
}

extern "C" int64_t phc_opt_block_elems(void) { return 16384; }

extern "C" int phc_opt_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                            const int64_t *blk_range, int32_t nblk, const int32_t *seg_blk, int32_t nseg,
                            const phc_adam_params *hp, phc_opt_state *state, float *norm_out,
                            const float *param_init, void *workspace, double *norm_acc, void *stream) {
  PHC_REQUIRE(param && grad && exp_avg && exp_avg_sq && blk_range && seg_blk && hp && state && workspace,
              "opt_step: null argument");
  PHC_REQUIRE(!norm_acc || norm_out, "opt_step: norm_acc needs norm_out");
  PHC_REQUIRE(n > 0 && nblk > 0 && nseg > 0, "opt_step: empty parameter set");
  PHC_REQUIRE(((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0,
              "opt_step: flat buffers must be 16-byte aligned");
  PHC_REQUIRE(!hp->use_loss_scale || hp->growth_interval > 0, "opt_step: bad loss-scale growth interval");
  hipStream_t st = as_stream(stream);
  double *part_sq = static_cast<double *>(workspace);
  double *part_l2 = param_init ? part_sq + nblk : nullptr;
  int *part_bad = reinterpret_cast<int *>(part_sq + 2 * (int64_t)nblk);
  hipLaunchKernelGGL(k_grad_partials, dim3((unsigned)nblk), dim3(kOptBlock), 0, st, grad, blk_range, part_sq,
                     part_bad, param, param_init, part_l2);
  hipLaunchKernelGGL(k_opt_finish, dim3(1), dim3(kFinThreads), 0, st, part_sq, part_bad, part_l2, blk_range, seg_blk,
                     (int)nseg, *hp, state, norm_out, norm_acc);
  const int64_t quads = (n + 3) / 4;
  const int64_t blocks = std::min<int64_t>((quads + kOptBlock - 1) / kOptBlock, 4096);
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(kOptBlock), 0, st, param, grad, exp_avg, exp_avg_sq, n,
                     *hp, state);
  return check_launch("opt_step");
}

extern "C" int64_t phc_adam_job_blocks(int32_t kind, int64_t rows, int64_t cols) {
  if (rows <= 0) return 0;
  if (kind == PHC_ADAM_FLAT) return (rows + kAdamFlatElems - 1) / kAdamFlatElems;
  if (cols <= 0) return 0;
  return ((rows + kPackTile - 1) / kPackTile) * ((cols + kPackTile - 1) / kPackTile);
}

extern "C" int phc_opt_step_operands(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                                     const int64_t *blk_range, int32_t nblk, const int32_t *seg_blk, int32_t nseg,
                                     const phc_adam_params *hp, phc_opt_state *state, float *norm_out,
                                     const float *param_init, void *workspace, double *norm_acc,
                                     const phc_adam_job *jobs, int32_t njobs, int64_t nblocks, void *stream) {
  PHC_REQUIRE(param && grad && exp_avg && exp_avg_sq && blk_range && seg_blk && hp && state && workspace && jobs,
              "opt_step_operands: null argument");
  PHC_REQUIRE(n > 0 && nblk > 0 && nseg > 0, "opt_step_operands: empty parameter set");
  PHC_REQUIRE(njobs >= 1 && njobs <= PHC_MAX_ADAM_JOBS && nblocks >= 1 && nblocks < (1ll << 31),
              "opt_step_operands: 1..%d jobs, 1..2^31 workgroups", PHC_MAX_ADAM_JOBS);
  PHC_REQUIRE(!hp->use_loss_scale || hp->growth_interval > 0, "opt_step_operands: bad loss-scale growth interval");
  hipStream_t st = as_stream(stream);
  double *part_sq = static_cast<double *>(workspace);
  double *part_l2 = param_init ? part_sq + nblk : nullptr;
  int *part_bad = reinterpret_cast<int *>(part_sq + 2 * (int64_t)nblk);
  hipLaunchKernelGGL(k_grad_partials, dim3((unsigned)nblk), dim3(kOptBlock), 0, st, grad, blk_range, part_sq,
                     part_bad, param, param_init, part_l2);
  hipLaunchKernelGGL(k_opt_finish, dim3(1), dim3(kFinThreads), 0, st, part_sq, part_bad, part_l2, blk_range, seg_blk,
                     (int)nseg, *hp, state, norm_out, norm_acc);
  hipLaunchKernelGGL(k_adam_ops, dim3((unsigned)nblocks), dim3(kPackThreads), 0, st, param, grad, exp_avg, exp_avg_sq,
                     jobs, (int)njobs, *hp, state);
  return check_launch("opt_step_operands");
}

extern "C" size_t phc_opt_workspace_bytes(int32_t nblk) {
  return nblk <= 0 ? 0 : (size_t)nblk * (2 * sizeof(double) + sizeof(int)) + 16;
}
