// phc_fk.hip — load-time forward kinematics + velocities of the motion library (R3-R5).
//
// Stage A (one lane per frame): local rotations from global ones in float64 (stored float32,
//   poselib_skeleton.py:574-593), root-replaced local translations (:605-619) and the float32
//   FK chain of transform_mul (:518-539, torch_utils.py:322-330).  The per-frame chain state
//   (24 rotations + positions) lives in LDS, [joint][component][lane], conflict-free.
// Stage B (one lane per frame x joint): np.gradient of positions / dt (float32), the float64
//   angular velocity of consecutive global rotations (:1240-1251) and dof velocities of local
//   rotations (motion_lib.py:119-140).
// Stage C (one lane per frame x joint x axis): the 17-tap gaussian (sigma 2, mode 'nearest')
//   along time inside each clip, accumulated in float64 in scipy's symmetric order.
#include "phc_common.h"

namespace phc {

constexpr int kFkLanes = 64;

struct FkArgs {
  const double *qg;      // [F,24,4]
  const double *rt;      // [F,3]
  const int64_t *starts;
  const int64_t *counts;
  const float *fps;
  int64_t nmot, F;
  const int64_t *parents;
  const float *lt;       // [24,3]
  const double *gw;      // gaussian weights [2r+1]
  int gr;                // radius
  float *frames;         // [F,24,13]
  float *lrs;            // [F,24,4]
  float *dvs;            // [F,23,3]
  float *raw_v;          // [F,24,3] workspace
  double *raw_av;        // [F,24,3] workspace
};

__device__ __forceinline__ int64_t motion_of(const int64_t *starts, int64_t nmot, int64_t f) {
  int64_t lo = 0, hi = nmot - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (starts[mid] <= f) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ Q4<double> ldq(const double *p) { return {p[0], p[1], p[2], p[3]}; }

__global__ __launch_bounds__(kFkLanes) void k_fk_chain(FkArgs a) {
  __shared__ float s_rot[kBodies][4][kFkLanes];
  __shared__ float s_pos[kBodies][3][kFkLanes];
  const int lane = threadIdx.x;
  const int64_t f = (int64_t)blockIdx.x * kFkLanes + lane;
  if (f >= a.F) return;
  const double *q = a.qg + f * kBodies * 4;
  for (int j = 0; j < kBodies; ++j) {
    const int p = (int)a.parents[j];
    const Q4<double> gj = ldq(q + 4 * j);
    q4 lr;
    if (p < 0) {
      lr = {(float)gj.x, (float)gj.y, (float)gj.z, (float)gj.w};
    } else {
      const Q4<double> l = quat_mul_norm(quat_conj(ldq(q + 4 * p)), gj);
      lr = {(float)l.x, (float)l.y, (float)l.z, (float)l.w};
    }
    float *o = a.lrs + (f * kBodies + j) * 4;
    o[0] = lr.x; o[1] = lr.y; o[2] = lr.z; o[3] = lr.w;
    v3 lt = {a.lt[3 * j], a.lt[3 * j + 1], a.lt[3 * j + 2]};
    q4 gr;
    v3 gp;
    if (p < 0) {
      lt = {(float)a.rt[3 * f], (float)a.rt[3 * f + 1], (float)a.rt[3 * f + 2]};
      gr = lr;
      gp = lt;
    } else {
      const q4 pr = {s_rot[p][0][lane], s_rot[p][1][lane], s_rot[p][2][lane], s_rot[p][3][lane]};
      const v3 pp = {s_pos[p][0][lane], s_pos[p][1][lane], s_pos[p][2][lane]};
      gr = quat_mul_norm(pr, lr);
      gp = vadd(quat_rotate(pr, lt), pp);
    }
    s_rot[j][0][lane] = gr.x; s_rot[j][1][lane] = gr.y; s_rot[j][2][lane] = gr.z; s_rot[j][3][lane] = gr.w;
    s_pos[j][0][lane] = gp.x; s_pos[j][1][lane] = gp.y; s_pos[j][2][lane] = gp.z;
    float *fr = a.frames + (f * kBodies + j) * kRec;
    fr[0] = gp.x; fr[1] = gp.y; fr[2] = gp.z;
    fr[3] = (float)gj.x; fr[4] = (float)gj.y; fr[5] = (float)gj.z; fr[6] = (float)gj.w;
  }
}

__global__ __launch_bounds__(256) void k_fk_raw_vel(FkArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.F * kBodies) return;
  const int64_t f = i / kBodies;
  const int j = (int)(i % kBodies);
  const int64_t m = motion_of(a.starts, a.nmot, f);
  const int64_t s = a.starts[m], T = a.counts[m], t = f - s;
  const double dt = 1.0 / (double)a.fps[m];
  const float dtf = (float)dt;
  // linear: np.gradient (edge_order 1) along time, / dt, float32
  float *rv = a.raw_v + i * 3;
  if (T < 2) {
    rv[0] = rv[1] = rv[2] = 0.0f;
  } else {
    int64_t fa, fb;
    float den;
    if (t == 0) { fa = f + 1; fb = f; den = 1.0f; }
    else if (t == T - 1) { fa = f; fb = f - 1; den = 1.0f; }
    else { fa = f + 1; fb = f - 1; den = 2.0f; }
    const float *pa = a.frames + (fa * kBodies + j) * kRec;
    const float *pb = a.frames + (fb * kBodies + j) * kRec;
#pragma unroll
    for (int k = 0; k < 3; ++k) rv[k] = ((pa[k] - pb[k]) / den) / dtf;
  }
  // angular: quat_mul_norm(r[t+1], inv r[t]) -> angle-axis / dt in float64 (identity at the end)
  double *ra = a.raw_av + i * 3;
  if (t < T - 1) {
    const Q4<double> d =
        quat_mul_norm(ldq(a.qg + ((f + 1) * kBodies + j) * 4), quat_conj(ldq(a.qg + (f * kBodies + j) * 4)));
    double ang;
    V3<double> ax;
    quat_angle_axis_d(d, &ang, &ax);
    ra[0] = ax.x * ang / dt; ra[1] = ax.y * ang / dt; ra[2] = ax.z * ang / dt;
  } else {
    double ang;
    V3<double> ax;
    quat_angle_axis_d(Q4<double>{0.0, 0.0, 0.0, 1.0}, &ang, &ax);
    ra[0] = ax.x * ang / dt; ra[1] = ax.y * ang / dt; ra[2] = ax.z * ang / dt;
  }
  // dof velocity of joint j >= 1 (float32): conj(lr[t]) * lr[t+1]; last frame repeats t-1
  if (j >= 1) {
    float *dv = a.dvs + (f * (kBodies - 1) + (j - 1)) * 3;
    if (T < 2) {
      dv[0] = dv[1] = dv[2] = 0.0f;
    } else {
      const int64_t f0 = (t < T - 1) ? f : f - 1;
      const float *l0 = a.lrs + (f0 * kBodies + j) * 4;
      const float *l1 = a.lrs + ((f0 + 1) * kBodies + j) * 4;
      const q4 d = quat_mul(quat_conj(q4{l0[0], l0[1], l0[2], l0[3]}), q4{l1[0], l1[1], l1[2], l1[3]});
      float st;
      const float ang = quat_angle_masked(d, &st);
      v3 ax = {0.0f, 0.0f, 1.0f};
      if (fabsf(st) > 1e-5f) ax = {d.x / st, d.y / st, d.z / st};
      dv[0] = ax.x * ang / dtf; dv[1] = ax.y * ang / dtf; dv[2] = ax.z * ang / dtf;
    }
  }
}

__global__ __launch_bounds__(256) void k_fk_smooth(FkArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (frame, joint, axis)
  if (i >= a.F * kBodies * 3) return;
  const int64_t f = i / (kBodies * 3);
  const int rem = (int)(i % (kBodies * 3));
  const int j = rem / 3, k = rem % 3;
  const int64_t m = motion_of(a.starts, a.nmot, f);
  const int64_t s = a.starts[m], T = a.counts[m], t = f - s;
  const int r = a.gr;
  double lin = (double)a.raw_v[(f * kBodies + j) * 3 + k] * a.gw[r];
  double ang = a.raw_av[(f * kBodies + j) * 3 + k] * a.gw[r];
  for (int q = r; q >= 1; --q) {  // scipy's symmetric loop: far pairs first
    int64_t tp = t + q, tm = t - q;
    tp = tp > T - 1 ? T - 1 : tp;
    tm = tm < 0 ? 0 : tm;
    const int64_t ip = ((s + tp) * kBodies + j) * 3 + k, im = ((s + tm) * kBodies + j) * 3 + k;
    lin = lin + ((double)a.raw_v[im] + (double)a.raw_v[ip]) * a.gw[r - q];
    ang = ang + (a.raw_av[im] + a.raw_av[ip]) * a.gw[r - q];
  }
  float *fr = a.frames + (f * kBodies + j) * kRec;
  fr[7 + k] = (float)lin;
  fr[10 + k] = (float)ang;
}

}  // namespace phc

using namespace phc;

extern "C" size_t phc_fk_workspace_bytes(int64_t F) {
  return (size_t)F * kBodies * 3 * (sizeof(float) + sizeof(double)) + 256;
}

extern "C" int phc_fk_motions(const double *quat_global, const double *root_trans, const int64_t *starts,
                              const int64_t *counts, const float *fps, int64_t num_motions, int64_t F,
                              const int64_t *parents, const float *local_translation, const double *gauss_weights,
                              int32_t gauss_radius, float *frames, float *local_rot, float *dof_vel, void *workspace,
                              void *stream) {
  PHC_REQUIRE(quat_global && root_trans && starts && counts && fps && parents && local_translation &&
                  gauss_weights && frames && local_rot && dof_vel && workspace,
              "fk_motions: null argument");
  PHC_REQUIRE(num_motions > 0 && F > 0 && gauss_radius >= 0, "fk_motions: empty input");
  hipStream_t s = as_stream(stream);
  FkArgs a;
  a.qg = quat_global; a.rt = root_trans; a.starts = starts; a.counts = counts; a.fps = fps;
  a.nmot = num_motions; a.F = F; a.parents = parents; a.lt = local_translation; a.gw = gauss_weights;
  a.gr = gauss_radius; a.frames = frames; a.lrs = local_rot; a.dvs = dof_vel;
  a.raw_v = reinterpret_cast<float *>(workspace);
  size_t off = (size_t)F * kBodies * 3 * sizeof(float);
  off = (off + 255) & ~(size_t)255;
  a.raw_av = reinterpret_cast<double *>(reinterpret_cast<char *>(workspace) + off);
  hipLaunchKernelGGL(k_fk_chain, dim3((unsigned)((F + kFkLanes - 1) / kFkLanes)), dim3(kFkLanes), 0, s, a);
  if (int rc = check_launch("fk_chain")) return rc;
  const int64_t nj = F * kBodies;
  hipLaunchKernelGGL(k_fk_raw_vel, dim3((unsigned)((nj + 255) / 256)), dim3(256), 0, s, a);
  if (int rc = check_launch("fk_raw_vel")) return rc;
  hipLaunchKernelGGL(k_fk_smooth, dim3((unsigned)((nj * 3 + 255) / 256)), dim3(256), 0, s, a);
  return check_launch("fk_smooth");
}
