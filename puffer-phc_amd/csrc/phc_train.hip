// phc_train.hip — trainer-side kernels: GAE as a parallel affine scan (R20) and the
// RunningNorm batch statistics / normalisation (R17).  All HBM-bound.
#include "phc_common.h"

namespace phc {

// ------------------------------------------------------------------- GAE --
// c_gae.pyx:11-32 runs, for t = n-2 .. 0 (nnt = 1 - done[t+1]):
//   last = (r[t+1] + g*v[t+1]*nnt - v[t]) + ((g*l)*nnt)*last;   adv[t] = last;   adv[n-1] = 0
// i.e. adv[t] = D_t + C_t * adv[t+1], an affine map per element.  Maps compose as
// (C1,D1)∘(C2,D2) = (C1*C2, D1 + C1*D2).  Each thread owns kSeg consecutive elements and runs
// the exact sequential recurrence over them; only the carry entering each segment comes from
// the composed maps (block scan of segment maps + a serial fold over block maps).
constexpr int kSeg = 16;
constexpr int kGaeBlock = 256;
constexpr int64_t kGaeChunk = (int64_t)kSeg * kGaeBlock;

struct Aff {
  float c, d;
};

__device__ __forceinline__ void gae_elem(const float *__restrict__ dn, const float *__restrict__ v,
                                         const float *__restrict__ r, int64_t t, float g, float gl, float &c,
                                         float &d) {
  const float nnt = 1.0f - dn[t + 1];
  d = r[t + 1] + g * v[t + 1] * nnt - v[t];
  c = gl * nnt;
}

// segment map of elements [lo, hi) (hi <= n-1): applied right-to-left
__device__ __forceinline__ Aff seg_map(const float *dn, const float *v, const float *r, int64_t lo, int64_t hi,
                                       float g, float gl) {
  Aff a = {1.0f, 0.0f};
  for (int64_t t = hi - 1; t >= lo; --t) {
    float c, d;
    gae_elem(dn, v, r, t, g, gl, c, d);
    a = {c * a.c, d + c * a.d};
  }
  return a;
}

// block-wide exclusive "suffix" scan: out[i] = map_{i+1} ∘ ... ∘ map_{last} (identity for last)
__device__ Aff block_suffix_scan(Aff mine, Aff *sh) {
  const int tid = threadIdx.x;
  sh[tid] = mine;
  __syncthreads();
  // Hillis-Steele over reversed index: acc_i = map_i ∘ map_{i+1} ∘ ... (inclusive)
  for (int off = 1; off < kGaeBlock; off <<= 1) {
    Aff cur = sh[tid];
    Aff nxt = (tid + off < kGaeBlock) ? sh[tid + off] : Aff{1.0f, 0.0f};
    __syncthreads();
    sh[tid] = {cur.c * nxt.c, cur.d + cur.c * nxt.d};
    __syncthreads();
  }
  Aff excl = (tid + 1 < kGaeBlock) ? sh[tid + 1] : Aff{1.0f, 0.0f};
  __syncthreads();
  return excl;
}

__global__ __launch_bounds__(kGaeBlock) void k_gae_blocks(const float *dn, const float *v, const float *r, int64_t n,
                                                          float g, float gl, Aff *blk, Aff *seg) {
  __shared__ Aff sh[kGaeBlock];
  const int64_t m = n - 1;  // number of recurrence elements
  const int64_t lo = (int64_t)blockIdx.x * kGaeChunk + (int64_t)threadIdx.x * kSeg;
  const int64_t hi = lo + kSeg < m ? lo + kSeg : m;
  const Aff mine = lo < m ? seg_map(dn, v, r, lo, hi, g, gl) : Aff{1.0f, 0.0f};
  seg[(int64_t)blockIdx.x * kGaeBlock + threadIdx.x] = mine;
  const Aff excl = block_suffix_scan(mine, sh);
  if (threadIdx.x == 0) blk[blockIdx.x] = {mine.c * excl.c, mine.d + mine.c * excl.d};
}

__global__ __launch_bounds__(kGaeBlock) void k_gae_apply(const float *dn, const float *v, const float *r, int64_t n,
                                                         float g, float gl, const Aff *blk, const Aff *seg,
                                                         int64_t nblk, float *adv) {
  __shared__ Aff sh[kGaeBlock];
  __shared__ float carry_in;
  const int64_t m = n - 1;
  if (threadIdx.x == 0) {
    float x = 0.0f;  // adv[n-1] = 0
    for (int64_t k = nblk - 1; k > (int64_t)blockIdx.x; --k) x = blk[k].d + blk[k].c * x;
    carry_in = x;
  }
  const Aff mine = seg[(int64_t)blockIdx.x * kGaeBlock + threadIdx.x];
  const Aff excl = block_suffix_scan(mine, sh);
  const float carry = excl.d + excl.c * carry_in;  // adv value just after this segment
  const int64_t lo = (int64_t)blockIdx.x * kGaeChunk + (int64_t)threadIdx.x * kSeg;
  const int64_t hi = lo + kSeg < m ? lo + kSeg : m;
  float last = carry;
  for (int64_t t = hi - 1; t >= lo; --t) {
    const float nnt = 1.0f - dn[t + 1];
    const float delta = r[t + 1] + g * v[t + 1] * nnt - v[t];
    last = delta + gl * nnt * last;  // ((gamma*lam)*nnt)*last as in c_gae.pyx:30
    adv[t] = last;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) adv[m] = 0.0f;
}

// ------------------------------------------------------------------- RMS --
// RunningNorm.update: batch mean / biased var per column, then
//   mean = mean*(1-w) + bm*w; var = var*(1-w) + bv*w; w = 1/count; count += 1.
// Pass 1: each workgroup sums a row chunk of 256 columns in float64 (sum, sum of squares).
// Pass 2: per column, merge chunk partials (Chan) and apply the running update.
constexpr int kRmsCols = 256;
constexpr int64_t kRmsRows = 512;

// (mean, M2) of one column chunk from its float64 sums
__device__ __forceinline__ void rms_store_part(double *__restrict__ part, int64_t cols, int64_t col, double s, double s2,
                                               int64_t nrc) {
  const double mean = s / (double)nrc;
  double m2 = s2 - s * mean;
  if (m2 < 0.0) m2 = 0.0;
  double *p = part + ((int64_t)blockIdx.y * cols + col) * 2;
  p[0] = mean;
  p[1] = m2;
}

// Each thread sums TWO adjacent columns (one 8-B load per row when the row starts allow it) over
// the chunk's rows in row order — the same float64 sums as one column per thread — with the next
// kPf rows' loads in flight ahead of the adds (the serial chain otherwise waits a memory round
// trip per row).  32 rows in flight (round 4; 8 before: 278 us for the 490 MB rollout batch, one
// memory round trip per 8 rows with only 2 workgroups per CU)
constexpr int kRmsPf = 32;
__global__ __launch_bounds__(kRmsCols) void k_rms_partial(const float *__restrict__ x, int64_t rows, int64_t cols,
                                                          double *__restrict__ part) {
  const int64_t col = ((int64_t)blockIdx.x * kRmsCols + threadIdx.x) * 2;
  const int64_t r0 = (int64_t)blockIdx.y * kRmsRows;
  const int64_t r1 = r0 + kRmsRows < rows ? r0 + kRmsRows : rows;
  if (col >= cols) return;
  const bool two = col + 1 < cols;
  const bool vec = two && (cols % 2 == 0) && ((reinterpret_cast<uintptr_t>(x) & 7) == 0);
  double s0 = 0.0, q0 = 0.0, s1 = 0.0, q1 = 0.0;
  float2 buf[kRmsPf];
  auto load = [&](int64_t r) -> float2 {
    const float *p = x + r * cols + col;
    if (vec) return *reinterpret_cast<const float2 *>(p);
    return float2{p[0], two ? p[1] : 0.0f};
  };
  int64_t r = r0;
  // the unrolled loads must not sit behind a per-load select: hipcc then branches around each
  // load and waits vmcnt(0) per row (measured: 280 us for the 490 MB rollout batch, 1.75 TB/s)
  if (vec) {
    for (; r + kRmsPf <= r1; r += kRmsPf) {
      const float *p = x + r * cols + col;
#pragma unroll
      for (int u = 0; u < kRmsPf; ++u) buf[u] = *reinterpret_cast<const float2 *>(p + u * cols);
#pragma unroll
      for (int u = 0; u < kRmsPf; ++u) {
        const double a = (double)buf[u].x, b = (double)buf[u].y;
        s0 += a;
        q0 += a * a;
        s1 += b;
        q1 += b * b;
      }
    }
  }
  for (; r < r1; ++r) {
    const float2 v = load(r);
    const double a = (double)v.x, b = (double)v.y;
    s0 += a;
    q0 += a * a;
    s1 += b;
    q1 += b * b;
  }
  rms_store_part(part, cols, col, s0, q0, r1 - r0);
  if (two) rms_store_part(part, cols, col + 1, s1, q1, r1 - r0);
}

// Chan merge of a column's row-chunk partials (mean, M2) in chunk order
__device__ __forceinline__ void rms_chunk_merge(const double *__restrict__ part, int64_t rows, int64_t cols,
                                                int64_t nchunks, int64_t col, double &n, double &mean, double &m2) {
  n = 0.0;
  mean = 0.0;
  m2 = 0.0;
  // the chunk partials of the next 8 chunks are loaded before they are merged (same order)
  constexpr int PF = 8;
  for (int64_t k0 = 0; k0 < nchunks; k0 += PF) {
    double2 pb[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (k0 + u < nchunks) pb[u] = *reinterpret_cast<const double2 *>(part + ((k0 + u) * cols + col) * 2);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int64_t k = k0 + u;
      if (k >= nchunks) break;
      const double nb = (double)((k + 1) * kRmsRows < rows ? kRmsRows : rows - k * kRmsRows);
      const double mb = pb[u].x;
      const double m2b = pb[u].y;
      const double tot = n + nb;
      const double delta = mb - mean;
      mean += delta * (nb / tot);
      m2 += m2b + delta * delta * (n * nb / tot);
      n = tot;
    }
  }
}

__device__ __forceinline__ void rms_running_update(float *__restrict__ rmean, float *__restrict__ rvar,
                                                   const float *__restrict__ count, int64_t col, double mean,
                                                   double m2, double n) {
  const float bm = (float)mean;
  const float bv = (float)(m2 / n);
  const float w = 1.0f / count[0];
  rmean[col] = rmean[col] * (1.0f - w) + bm * w;
  rvar[col] = rvar[col] * (1.0f - w) + bv * w;
}

__global__ __launch_bounds__(kRmsCols) void k_rms_merge(const double *__restrict__ part, int64_t rows, int64_t cols,
                                                        int64_t nchunks, float *__restrict__ rmean,
                                                        float *__restrict__ rvar, const float *__restrict__ count) {
  const int64_t col = (int64_t)blockIdx.x * kRmsCols + threadIdx.x;
  if (col >= cols) return;
  double n, mean, m2;
  rms_chunk_merge(part, rows, cols, nchunks, col, n, mean, m2);
  rms_running_update(rmean, rvar, count, col, mean, m2, n);
}

// data parallel: this rank's batch moments (mean, M2) per column, exchanged by the caller
__global__ __launch_bounds__(kRmsCols) void k_rms_moments(const double *__restrict__ part, int64_t rows, int64_t cols,
                                                          int64_t nchunks, double *__restrict__ mom) {
  const int64_t col = (int64_t)blockIdx.x * kRmsCols + threadIdx.x;
  if (col >= cols) return;
  double n, mean, m2;
  rms_chunk_merge(part, rows, cols, nchunks, col, n, mean, m2);
  mom[col * 2] = mean;
  mom[col * 2 + 1] = m2;
}

// every rank's moments merged in rank order (the same result on every rank), then the running
// update; with one part this is exactly k_rms_merge's result
__global__ __launch_bounds__(kRmsCols) void k_rms_apply(const double *__restrict__ mom, const double *__restrict__ prows,
                                                        int32_t parts, int64_t cols, float *__restrict__ rmean,
                                                        float *__restrict__ rvar, const float *__restrict__ count) {
  const int64_t col = (int64_t)blockIdx.x * kRmsCols + threadIdx.x;
  if (col >= cols) return;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int32_t k = 0; k < parts; ++k) {
    const double nb = prows[k];
    if (nb <= 0.0) continue;
    const double mb = mom[((int64_t)k * cols + col) * 2];
    const double m2b = mom[((int64_t)k * cols + col) * 2 + 1];
    const double tot = n + nb;
    const double delta = mb - mean;
    mean += delta * (nb / tot);
    m2 += m2b + delta * delta * (n * nb / tot);
    n = tot;
  }
  rms_running_update(rmean, rvar, count, col, mean, m2, n);
}

__global__ void k_count_inc(float *count) { count[0] = count[0] + 1.0f; }

__global__ __launch_bounds__(256) void k_rms_normalize(const float *__restrict__ x, float *__restrict__ y, int64_t total,
                                                       int64_t cols, const float *__restrict__ mean,
                                                       const float *__restrict__ var, float eps, float clip) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t c = i % cols;
    float v = (x[i] - mean[c]) / sqrtf(var[c] + eps);
    v = v < -clip ? -clip : (v > clip ? clip : v);
    y[i] = v;
  }
}

}  // namespace phc

using namespace phc;

extern "C" size_t phc_gae_workspace_bytes(int64_t n) {
  const int64_t nblk = n > 1 ? (n - 1 + kGaeChunk - 1) / kGaeChunk : 1;
  return (size_t)(nblk * (kGaeBlock + 1)) * sizeof(Aff) + 256;
}

extern "C" int phc_gae(const float *dones, const float *values, const float *rewards, int64_t n, float gamma,
                       float lam, float *adv, void *workspace, void *stream) {
  PHC_REQUIRE(dones && values && rewards && adv && workspace, "gae: null argument");
  if (n <= 0) return PHC_OK;
  hipStream_t s = as_stream(stream);
  if (n == 1) {
    if (hipMemsetAsync(adv, 0, sizeof(float), s) != hipSuccess) return check_launch("gae memset");
    return PHC_OK;
  }
  const int64_t nblk = (n - 1 + kGaeChunk - 1) / kGaeChunk;
  Aff *blk = reinterpret_cast<Aff *>(workspace);
  Aff *seg = blk + nblk;
  const float gl = gamma * lam;
  hipLaunchKernelGGL(k_gae_blocks, dim3((unsigned)nblk), dim3(kGaeBlock), 0, s, dones, values, rewards, n, gamma, gl,
                     blk, seg);
  if (int rc = check_launch("gae_blocks")) return rc;
  hipLaunchKernelGGL(k_gae_apply, dim3((unsigned)nblk), dim3(kGaeBlock), 0, s, dones, values, rewards, n, gamma, gl,
                     blk, seg, nblk, adv);
  return check_launch("gae_apply");
}

extern "C" size_t phc_rms_workspace_bytes(int64_t rows, int64_t cols) {
  const int64_t nchunks = (rows + kRmsRows - 1) / kRmsRows;
  return (size_t)(nchunks * cols * 2) * sizeof(double);
}

extern "C" int phc_rms_update(const float *x, int64_t rows, int64_t cols, float *mean, float *var, float *count,
                              void *workspace, void *stream) {
  PHC_REQUIRE(x && mean && var && count && workspace, "rms_update: null argument");
  PHC_REQUIRE(rows > 0 && cols > 0, "rms_update: empty batch");
  hipStream_t s = as_stream(stream);
  const int64_t nchunks = (rows + kRmsRows - 1) / kRmsRows;
  double *part = reinterpret_cast<double *>(workspace);
  const unsigned gx = (unsigned)((cols + kRmsCols - 1) / kRmsCols);
  const unsigned gp = (unsigned)((cols + 2 * kRmsCols - 1) / (2 * kRmsCols));  // two columns per thread
  hipLaunchKernelGGL(k_rms_partial, dim3(gp, (unsigned)nchunks), dim3(kRmsCols), 0, s, x, rows, cols, part);
  if (int rc = check_launch("rms_partial")) return rc;
  hipLaunchKernelGGL(k_rms_merge, dim3(gx), dim3(kRmsCols), 0, s, part, rows, cols, nchunks, mean, var, count);
  if (int rc = check_launch("rms_merge")) return rc;
  hipLaunchKernelGGL(k_count_inc, dim3(1), dim3(1), 0, s, count);
  return check_launch("rms_count");
}

extern "C" int phc_rms_moments(const float *x, int64_t rows, int64_t cols, double *moments, void *workspace,
                               void *stream) {
  PHC_REQUIRE(x && moments && workspace, "rms_moments: null argument");
  PHC_REQUIRE(rows > 0 && cols > 0, "rms_moments: empty batch");
  hipStream_t s = as_stream(stream);
  const int64_t nchunks = (rows + kRmsRows - 1) / kRmsRows;
  double *part = reinterpret_cast<double *>(workspace);
  const unsigned gx = (unsigned)((cols + kRmsCols - 1) / kRmsCols);
  const unsigned gp = (unsigned)((cols + 2 * kRmsCols - 1) / (2 * kRmsCols));  // two columns per thread
  hipLaunchKernelGGL(k_rms_partial, dim3(gp, (unsigned)nchunks), dim3(kRmsCols), 0, s, x, rows, cols, part);
  if (int rc = check_launch("rms_partial")) return rc;
  hipLaunchKernelGGL(k_rms_moments, dim3(gx), dim3(kRmsCols), 0, s, part, rows, cols, nchunks, moments);
  return check_launch("rms_moments");
}

extern "C" int phc_rms_apply(const double *moments, const double *part_rows, int32_t parts, int64_t cols, float *mean,
                             float *var, float *count, void *stream) {
  PHC_REQUIRE(moments && part_rows && mean && var && count, "rms_apply: null argument");
  PHC_REQUIRE(parts > 0 && cols > 0, "rms_apply: empty");
  hipStream_t s = as_stream(stream);
  const unsigned gx = (unsigned)((cols + kRmsCols - 1) / kRmsCols);
  hipLaunchKernelGGL(k_rms_apply, dim3(gx), dim3(kRmsCols), 0, s, moments, part_rows, parts, cols, mean, var, count);
  if (int rc = check_launch("rms_apply")) return rc;
  hipLaunchKernelGGL(k_count_inc, dim3(1), dim3(1), 0, s, count);
  return check_launch("rms_count");
}

extern "C" int phc_rms_normalize(const float *x, float *y, int64_t rows, int64_t cols, const float *mean,
                                 const float *var, float eps, float clip, void *stream) {
  PHC_REQUIRE(x && y && mean && var, "rms_normalize: null argument");
  const int64_t total = rows * cols;
  if (total <= 0) return PHC_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_rms_normalize, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), x, y, total, cols,
                     mean, var, eps, clip);
  return check_launch("rms_normalize");
}
