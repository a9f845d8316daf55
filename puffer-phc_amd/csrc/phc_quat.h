// phc_quat.h — device quaternion/transform math for the PHC hot path (gfx950).
//
// Every function follows the reference's TorchScript expression order
// (puffer_phc/torch_utils.py) so that, compiled with -ffp-contract=off, each IEEE
// add/mul/div/sqrt rounds exactly as torch-CPU's separate elementwise kernels do; only
// libm transcendentals (acos/atan2/sin/cos/exp) differ, by ulps.  Quaternions are xyzw.
#pragma once
#include <hip/hip_runtime.h>

namespace phc {

// PHC_FAST_ENV_MATH (default 1): the float divisions and square roots of the per-step env math that no
// index or flag depends on (slerp's weights, heading quaternions, the replay's quat_unit, the reward's
// means and termination distance) on the hardware reciprocal / square root (1-ulp class) instead of the
// correctly rounded IEEE sequences hipcc emits (~10 VALU each): the results stay within the north_star's
// 1e-5 of the reference (tests/test_gpu_env_sizes.py).  Frame indices, blend weights and times
// (frame_blend, the reset time draw) keep the IEEE division: they must match the reference bit for bit.
#ifndef PHC_FAST_ENV_MATH
#define PHC_FAST_ENV_MATH 1
#endif
__device__ __forceinline__ float fdiv_env(float a, float b) {
#if PHC_FAST_ENV_MATH
  return a * __builtin_amdgcn_rcpf(b);
#else
  return a / b;
#endif
}
__device__ __forceinline__ float fsqrt_env(float x) {
#if PHC_FAST_ENV_MATH
  return __builtin_amdgcn_sqrtf(x);
#else
  return sqrtf(x);
#endif
}
__device__ __forceinline__ float fexp_env(float x) {
#if PHC_FAST_ENV_MATH
  return __expf(x);
#else
  return expf(x);
#endif
}

// PHC_FAST_ENV_TRIG (default 1): slerp's acos / sin and the rotation angle's acos as short polynomials
// instead of the libm (OCML) routines with their range reductions: acos by Abramowitz & Stegun 4.4.46
// (sqrt(1 - |x|) times a degree-7 polynomial, |error| <= 2e-8 before float rounding), sin on slerp's
// [0, pi/2] by its Taylor series to x^11 (relative truncation <= 3e-8 there).  Both stay far inside
// the 1e-5 the env's observations and rewards are held to; no flag or index depends on them (the
// termination distance uses positions, which blend linearly).
#ifndef PHC_FAST_ENV_TRIG
#define PHC_FAST_ENV_TRIG 1
#endif
__device__ __forceinline__ float facos_env(float x) {
#if PHC_FAST_ENV_TRIG
  const float a = fabsf(x);
  float p = -0.0012624911f;
  p = fmaf(p, a, 0.0066700901f);
  p = fmaf(p, a, -0.0170881256f);
  p = fmaf(p, a, 0.0308918810f);
  p = fmaf(p, a, -0.0501743046f);
  p = fmaf(p, a, 0.0889789874f);
  p = fmaf(p, a, -0.2145988016f);
  p = fmaf(p, a, 1.5707963050f);
  const float r = __builtin_amdgcn_sqrtf(1.0f - a) * p;
  return x < 0.0f ? 3.14159265358979f - r : r;
#else
  return acosf(x);
#endif
}
// sin(x) for x in [0, pi/2] (slerp's weights)
__device__ __forceinline__ float fsin_half_env(float x) {
#if PHC_FAST_ENV_TRIG
  const float x2 = x * x;
  float p = -2.5052108e-8f;                // -1/11!
  p = fmaf(p, x2, 2.7557319e-6f);          // 1/9!
  p = fmaf(p, x2, -1.9841270e-4f);         // -1/7!
  p = fmaf(p, x2, 8.3333333e-3f);          // 1/5!
  p = fmaf(p, x2, -1.6666667e-1f);         // -1/3!
  return fmaf(x * x2, p, x);
#else
  return sinf(x);
#endif
}

template <typename T> struct Q4 { T x, y, z, w; };
template <typename T> struct V3 { T x, y, z; };

using q4 = Q4<float>;
using v3 = V3<float>;

template <typename T> __device__ __forceinline__ V3<T> vsub(V3<T> a, V3<T> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename T> __device__ __forceinline__ V3<T> vadd(V3<T> a, V3<T> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }

// torch_utils.py:55-75 — the 8-multiply quaternion product.
template <typename T>
__device__ __forceinline__ Q4<T> quat_mul(Q4<T> a, Q4<T> b) {
  const T ww = (a.z + a.x) * (b.x + b.y);
  const T yy = (a.w - a.y) * (b.w + b.z);
  const T zz = (a.w + a.y) * (b.w - b.z);
  const T xx = ww + yy + zz;
  const T qq = T(0.5) * (xx + (a.z - a.x) * (b.x - b.y));
  const T w = qq - ww + (a.z - a.y) * (b.y - b.z);
  const T x = qq - xx + (a.x + a.w) * (b.x + b.w);
  const T y = qq - yy + (a.w - a.x) * (b.y + b.z);
  const T z = qq - zz + (a.z + a.y) * (b.w - b.x);
  return {x, y, z, w};
}

// torch_utils.py:79-82
template <typename T> __device__ __forceinline__ Q4<T> quat_conj(Q4<T> a) { return {-a.x, -a.y, -a.z, a.w}; }

// torch.norm(p=2, dim=-1) over 3 / 4 elements: sequential sum of squares, then sqrt.
template <typename T> __device__ __forceinline__ T norm3(V3<T> v) {
  T s = v.x * v.x;
  s = s + v.y * v.y;
  s = s + v.z * v.z;
  return sqrt(s);
}
template <typename T> __device__ __forceinline__ T norm4(Q4<T> q) {
  T s = q.x * q.x;
  s = s + q.y * q.y;
  s = s + q.z * q.z;
  s = s + q.w * q.w;
  return sqrt(s);
}

// torch_utils.py:174-179 quat_unit
template <typename T> __device__ __forceinline__ Q4<T> quat_unit(Q4<T> q) {
  T n = norm4(q);
  n = n < T(1e-9) ? T(1e-9) : n;
  return {q.x / n, q.y / n, q.z / n, q.w / n};
}

// quat_unit (above) of a float quaternion on the hardware square root / reciprocal (PHC_FAST_ENV_MATH)
__device__ __forceinline__ q4 quat_unit_env(q4 q) {
#if PHC_FAST_ENV_MATH
  float n = fsqrt_env(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  n = n < 1e-9f ? 1e-9f : n;
  const float in = __builtin_amdgcn_rcpf(n);
  return {q.x * in, q.y * in, q.z * in, q.w * in};
#else
  return quat_unit(q);
#endif
}

// torch_utils.py:154-161 quat_pos (a sign flip by an exact +-1 factor) then quat_unit.
template <typename T> __device__ __forceinline__ Q4<T> quat_normalize(Q4<T> q) {
  if (q.w < T(0)) q = {-q.x, -q.y, -q.z, -q.w};
  return quat_unit(q);
}

template <typename T> __device__ __forceinline__ Q4<T> quat_mul_norm(Q4<T> a, Q4<T> b) {
  return quat_normalize(quat_mul(a, b));
}

// torch_utils.py:273-279 — rotation through the full quaternion product.
template <typename T> __device__ __forceinline__ V3<T> quat_rotate(Q4<T> r, V3<T> v) {
  const Q4<T> o = {v.x, v.y, v.z, T(0)};
  const Q4<T> t = quat_mul(quat_mul(r, o), quat_conj(r));
  return {t.x, t.y, t.z};
}

// torch_utils.py:283-291 my_quat_rotate: a + b + c.
__device__ __forceinline__ v3 my_quat_rotate(q4 q, v3 v) {
  const float s = 2.0f * (q.w * q.w) - 1.0f;
  const v3 a = {v.x * s, v.y * s, v.z * s};
  const float cx = q.y * v.z - q.z * v.y;
  const float cy = q.z * v.x - q.x * v.z;
  const float cz = q.x * v.y - q.y * v.x;
  const v3 b = {cx * q.w * 2.0f, cy * q.w * 2.0f, cz * q.w * 2.0f};
  const float dot = q.x * v.x + q.y * v.y + q.z * v.z;
  const v3 c = {q.x * dot * 2.0f, q.y * dot * 2.0f, q.z * dot * 2.0f};
  return {a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z};
}

// torch_utils.py:294-307 quat_to_tan_norm: rotate x-axis and z-axis.
__device__ __forceinline__ void quat_to_tan_norm(q4 q, float out[6]) {
  const v3 t = my_quat_rotate(q, v3{1.0f, 0.0f, 0.0f});
  const v3 n = my_quat_rotate(q, v3{0.0f, 0.0f, 1.0f});
  out[0] = t.x; out[1] = t.y; out[2] = t.z;
  out[3] = n.x; out[4] = n.y; out[5] = n.z;
}

// ---- exact specialisations -------------------------------------------------------------
// The reference evaluates its generic formulas on operands with structural zeros (unit axes,
// heading quaternions (0,0,z,w)).  Every product with such a zero is +-0 and every sum with it
// is exact, so dropping those terms (keeping the association of the surviving ones) gives the
// same float32 result bit for bit (up to the sign of an exact zero) at a third of the VALU cost.

// quat_to_tan_norm(q) = [my_quat_rotate(q, x-axis), my_quat_rotate(q, z-axis)]
__device__ __forceinline__ void tan_norm_fast(q4 q, float out[6]) {
  const float s = 2.0f * (q.w * q.w) - 1.0f;
  out[0] = s + (q.x * q.x) * 2.0f;
  out[1] = (q.z * q.w) * 2.0f + (q.y * q.x) * 2.0f;
  out[2] = (-q.y * q.w) * 2.0f + (q.z * q.x) * 2.0f;
  out[3] = (q.y * q.w) * 2.0f + (q.x * q.z) * 2.0f;
  out[4] = (-q.x * q.w) * 2.0f + (q.y * q.z) * 2.0f;
  out[5] = s + (q.z * q.z) * 2.0f;
}

// Heading quaternion h = (0, 0, z, w) with its my_quat_rotate coefficient precomputed.
struct Heading {
  float z, w, s;  // s = 2 w^2 - 1
};

__device__ __forceinline__ Heading make_heading(float z, float w) { return {z, w, 2.0f * (w * w) - 1.0f}; }

// my_quat_rotate(h, v) for h = (0,0,z,w): a + b + c with cross = (-(z vy), z vx, 0), dot = z vz
__device__ __forceinline__ v3 rot_heading(const Heading &h, v3 v) {
  return {v.x * h.s + ((-(h.z * v.y)) * h.w) * 2.0f,
          v.y * h.s + ((h.z * v.x) * h.w) * 2.0f,
          v.z * h.s + (h.z * (h.z * v.z)) * 2.0f};
}

// quat_mul(h, b) for h = (0,0,z,w) (8-multiply form with a.x = a.y = 0)
__device__ __forceinline__ q4 qmul_heading_left(const Heading &h, q4 b) {
  const float ww = h.z * (b.x + b.y);
  const float yy = h.w * (b.w + b.z);
  const float zz = h.w * (b.w - b.z);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + h.z * (b.x - b.y));
  return {qq - xx + h.w * (b.x + b.w), qq - yy + h.w * (b.y + b.z), qq - zz + h.z * (b.w - b.x),
          qq - ww + h.z * (b.y - b.z)};
}

// quat_mul(a, h) for h = (0,0,z,w) (8-multiply form with b.x = b.y = 0)
__device__ __forceinline__ q4 qmul_heading_right(q4 a, const Heading &h) {
  const float yy = (a.w - a.y) * (h.w + h.z);
  const float zz = (a.w + a.y) * (h.w - h.z);
  const float xx = yy + zz;
  const float qq = 0.5f * xx;
  return {qq - xx + (a.x + a.w) * h.w, qq - yy + (a.w - a.x) * h.z, qq - zz + (a.z + a.y) * h.w,
          qq + (a.z - a.y) * (-h.z)};
}

// torch_utils.py:50-51
__device__ __forceinline__ float normalize_angle(float x) { return atan2f(sinf(x), cosf(x)); }

// normalize_angle(a) for a in [0, 2pi] (a = 2*acos(w)): atan2(sin a, cos a) is a itself up
// to libm rounding below pi and a - 2pi above it, so fold the range instead of evaluating
// three transcendentals.
__device__ __forceinline__ float fold_angle_0_2pi(float a) { return a > 3.14159265f ? a - 6.28318531f : a; }

// torch_utils.py:86-106 quat_to_angle_axis: NaN lanes masked exactly like torch.where.
__device__ __forceinline__ float quat_angle_masked(q4 q, float *sin_theta_out) {
  const float sin_theta = fsqrt_env(1.0f - q.w * q.w);
  *sin_theta_out = sin_theta;
  if (!(fabsf(sin_theta) > 1e-5f)) return 0.0f;
  return fold_angle_0_2pi(2.0f * facos_env(q.w));
}

__device__ __forceinline__ v3 quat_to_exp_map(q4 q) {
  float s;
  const float angle = quat_angle_masked(q, &s);
  if (!(fabsf(s) > 1e-5f)) return {0.0f, 0.0f, 0.0f};  // angle 0 times default axis (0,0,1)
  const v3 axis = {q.x / s, q.y / s, q.z / s};
  return {angle * axis.x, angle * axis.y, angle * axis.z};
}

// torch_utils.py:110-131 slerp (branch order reproduces the two torch.where overrides).
__device__ __forceinline__ q4 slerp(q4 q0, q4 q1, float t) {
  float c = q0.x * q1.x + q0.y * q1.y + q0.z * q1.z + q0.w * q1.w;
  if (c < 0.0f) q1 = {-q1.x, -q1.y, -q1.z, -q1.w};
  c = fabsf(c);
  if (fabsf(c) >= 1.0f) return q0;
  const float sin_half = fsqrt_env(1.0f - c * c);
  if (fabsf(sin_half) < 0.001f)
    return {0.5f * q0.x + 0.5f * q1.x, 0.5f * q0.y + 0.5f * q1.y, 0.5f * q0.z + 0.5f * q1.z,
            0.5f * q0.w + 0.5f * q1.w};
  const float half = facos_env(c);
#if PHC_FAST_ENV_MATH
  const float inv = fdiv_env(1.0f, sin_half);
  const float ra = fsin_half_env((1.0f - t) * half) * inv;
  const float rb = fsin_half_env(t * half) * inv;
#else
  const float ra = sinf((1.0f - t) * half) / sin_half;
  const float rb = sinf(t * half) / sin_half;
#endif
  return {ra * q0.x + rb * q1.x, ra * q0.y + rb * q1.y, ra * q0.z + rb * q1.z, ra * q0.w + rb * q1.w};
}

// torch_utils.py:354-358 quat_from_angle_axis with axis = +z (normalize(z) == z exactly).
__device__ __forceinline__ q4 quat_from_angle_z(float angle) {
  const float theta = angle / 2.0f;
  const float s = sinf(theta);
  const q4 q = {0.0f * s, 0.0f * s, 1.0f * s, cosf(theta)};
  return quat_unit(q);
}

// torch_utils.py:334-365 exp_map_to_quat
__device__ __forceinline__ q4 exp_map_to_quat(v3 e) {
  float angle = norm3(e);
  v3 axis = {e.x / angle, e.y / angle, e.z / angle};
  angle = normalize_angle(angle);
  if (!(fabsf(angle) > 1e-5f)) {
    angle = 0.0f;
    axis = {0.0f, 0.0f, 1.0f};
  }
  const float theta = angle / 2.0f;
  float n = norm3(axis);
  n = n < 1e-9f ? 1e-9f : n;
  const float s = sinf(theta);
  const q4 q = {axis.x / n * s, axis.y / n * s, axis.z / n * s, cosf(theta)};
  return quat_unit(q);
}

// torch_utils.py:369-408 heading from the rotated x-axis; returns heading angle.
__device__ __forceinline__ float calc_heading(q4 q) {
  const v3 d = my_quat_rotate(q, v3{1.0f, 0.0f, 0.0f});
  return atan2f(d.y, d.x);
}

// calc_heading_quat / calc_heading_quat_inv (torch_utils.py:384-408) without atan2/sin/cos:
// with (c, s) = (cos h, sin h) of the heading h = atan2(y, x), the half-angle identities give
// cos(h/2) = sqrt((1+c)/2), sin(h/2) = s / (2 cos(h/2)) for c >= 0 and sin(h/2) =
// sign(s) sqrt((1-c)/2), cos(h/2) = s / (2 sin(h/2)) for c < 0 (both well conditioned), then
// quat_unit as the reference.  Agrees with the transcendental path to a few ulps.
__device__ __forceinline__ void heading_quats(q4 root_rot, Heading *hrot, Heading *hinv) {
  float tn[6];
  tan_norm_fast(root_rot, tn);  // tn[0..2] = my_quat_rotate(root_rot, x-axis)
  const v3 d = {tn[0], tn[1], tn[2]};
  const float r = fsqrt_env(d.x * d.x + d.y * d.y);
  float ch = 1.0f, sh = 0.0f;
  if (r > 0.0f) {
    const float ir = fdiv_env(1.0f, r);
    ch = PHC_FAST_ENV_MATH ? d.x * ir : d.x / r;
    sh = PHC_FAST_ENV_MATH ? d.y * ir : d.y / r;
  }
  float C, S;
  if (ch >= 0.0f) {
    C = fsqrt_env((1.0f + ch) * 0.5f);
    S = fdiv_env(sh, 2.0f * C);
  } else {
    S = copysignf(fsqrt_env((1.0f - ch) * 0.5f), sh);
    C = fdiv_env(sh, 2.0f * S);
  }
  // quat_unit of (0,0,+-S,C): the norm sqrt(S^2 + C^2) is shared and -S/n == -(S/n) exactly
  float n = fsqrt_env(S * S + C * C);
  n = n < 1e-9f ? 1e-9f : n;
  const float in = fdiv_env(1.0f, n);
  const float z = PHC_FAST_ENV_MATH ? S * in : S / n, w = PHC_FAST_ENV_MATH ? C * in : C / n;
  *hrot = make_heading(z, w);
  *hinv = make_heading(-z, w);
}

// torch_utils.py:219-228 quat_angle_axis (float64 use at load time): angle in [0, pi].
__device__ __forceinline__ void quat_angle_axis_d(Q4<double> x, double *angle, V3<double> *axis) {
  double s = 2.0 * (x.w * x.w) - 1.0;
  s = s < -1.0 ? -1.0 : (s > 1.0 ? 1.0 : s);
  *angle = acos(s);
  double n = norm3(V3<double>{x.x, x.y, x.z});
  n = n < 1e-9 ? 1e-9 : n;
  *axis = {x.x / n, x.y / n, x.z / n};
}

// Counter-based RNG (splitmix64 finaliser): uniform float in [0, 1) with 24 random bits.
// splitmix64's finaliser without its increment (mix64(z) == mix64_fin(z + 0x9E3779B97F4A7C15))
__device__ __forceinline__ unsigned long long mix64_fin(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long counter,
                                           unsigned long long idx) {
  const unsigned long long h = mix64(seed ^ mix64(counter * 0xD1B54A32D192ED03ull ^ mix64(idx)));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float normal01(unsigned long long seed, unsigned long long counter,
                                          unsigned long long idx) {
  const float u1 = uniform01(seed, counter, 2 * idx) + (1.0f / 33554432.0f);
  const float u2 = uniform01(seed, counter, 2 * idx + 1);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530718f * u2);
}

}  // namespace phc
