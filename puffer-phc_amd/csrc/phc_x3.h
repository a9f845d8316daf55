// phc_x3.h — fp32-class products on the bf16 MFMA (shared by phc_head.hip and phc_policy.hip).
//
// Every fp32 operand x is split exactly as x = hi + mid + lo with hi = bf16(x), mid = bf16(x - hi),
// lo = bf16(x - hi - mid) (8 + 8 + 8 significand bits: the fp32 significand), and each 16x16x32
// step accumulates the six products whose magnitude reaches 2^-16 of hi·hi (smallest first):
//   hi·lo + lo·hi + mid·mid + hi·mid + mid·hi + hi·hi
// The dropped terms (mid·lo, lo·mid, lo·lo) are below 2^-23 of |x||w|, so each product carries
// fp32-class error (the fp32 head's ulp, not the reference's TF32 2^-11) and the sums stay fp32.
// bf16 keeps fp32's exponent range, so no scaling is needed for tiny gradients.
#pragma once

#include <hip/hip_runtime.h>

namespace phc {

using x3f4 = __attribute__((ext_vector_type(4))) float;
using x3b8 = __attribute__((ext_vector_type(8))) __bf16;

struct X3 {
  x3b8 h, m, l;
};

__device__ __forceinline__ void split3(const float4 &x0, const float4 &x1, X3 &s) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = (__bf16)v[j];
    float r = v[j] - (float)a;
    const __bf16 m = (__bf16)r;
    r -= (float)m;
    s.h[j] = a;
    s.m[j] = m;
    s.l[j] = (__bf16)r;
  }
}

// the six terms for n independent accumulators, term-major: consecutive MFMAs write different
// accumulators, so no MFMA waits for the previous one's result
template <int n>
__device__ __forceinline__ void mma_x3_n(const X3 *a, const X3 *b, x3f4 *c, bool a_shared) {
#define PHC_X3_TERM(P, Q)                                                                        \
  _Pragma("unroll") for (int i = 0; i < n; ++i) c[i] =                                           \
      __builtin_amdgcn_mfma_f32_16x16x32_bf16((a_shared ? a[0] : a[i]).P, (a_shared ? b[i] : b[0]).Q, c[i], 0, 0, 0);
  PHC_X3_TERM(h, l)
  PHC_X3_TERM(l, h)
  PHC_X3_TERM(m, m)
  PHC_X3_TERM(h, m)
  PHC_X3_TERM(m, h)
  PHC_X3_TERM(h, h)
#undef PHC_X3_TERM
}

__device__ __forceinline__ x3f4 mma_x3(const X3 &a, const X3 &b, x3f4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, c, 0, 0, 0);
}

}  // namespace phc
