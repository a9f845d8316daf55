// phc_measure.h — measurement-only instrumentation of the env and GEMM kernels (never part of a product
// build).
// Env kernels.  A product build (Makefile default) defines nothing here: ENV_PHASE / ENV_PHASE_USE expand to nothing
// and phc_env_phase_copy is absent from the library.  tools/build_variants.sh builds the measurement
// library with -DPHC_MEASURE_ENV_PHASES=1: lane 0 of every wave of k_env_replay stamps the constant clock
// at its phase boundaries into g_env_phase[wave][8] (tools/env_phase_probe.py reads them):
// 0 start, 1 scalars used, 2 frame rows in LDS, 3 replay + reward done, 4 observation row written,
// 5 rows copied out, 6 stats flushed.
#pragma once

#ifndef PHC_MEASURE_GEMM_ONLY  // the GEMM translation unit takes only the GEMM section below
#if defined(PHC_MEASURE_ENV_PHASES) && PHC_MEASURE_ENV_PHASES
namespace phc {
constexpr int kPhaseWaves = 1 << 15;
__device__ unsigned long long g_env_phase[kPhaseWaves * 8];
}  // namespace phc
#define ENV_PHASE(k)                                                                                  \
  do {                                                                                                \
    const int gw_ = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);                              \
    if ((threadIdx.x & 63) == 0 && gw_ < kPhaseWaves) g_env_phase[gw_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// a use of a value before a stamp, so the stamp cannot move above the work that produces it
#define ENV_PHASE_USE(x)                 \
  do {                                   \
    if ((x) == -12345) e.rew[0] = 0.0f;  \
  } while (0)
#define PHC_ENV_PHASE_COPY                                                                                         \
  extern "C" int phc_env_phase_copy(unsigned long long *dst, int64_t waves) {                                       \
    const int64_t n = (waves < kPhaseWaves ? waves : kPhaseWaves) * 8;                                              \
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_env_phase), n * sizeof(unsigned long long), 0,                    \
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;                                       \
  }
#else
#define ENV_PHASE(k) \
  do {               \
  } while (0)
#define ENV_PHASE_USE(x) \
  do {                   \
  } while (0)
#define PHC_ENV_PHASE_COPY
#endif
#endif  // PHC_MEASURE_GEMM_ONLY

// GEMM kernels.  A product build defines neither PHC_MEASURE_GEMM nor PHC_GEMM_PROBE: the probes compile to
// nothing and phc_gemm_discard() is the constant 0.  tools/build_variants.sh builds the measurement library
// with -DPHC_MEASURE_GEMM=1 (and optionally -DPHC_GEMM_PROBE=n):
//   PHC_GEMM_PROBE 1 = every tile stages the operand panels of tile (0, 0) (L2-hot operands, same
//     instruction stream); 2 = only the first K-tile is staged (LDS fragment reads + MFMA, no operand
//     traffic); 3 = B staged once and its fragments kept;
//   PHC_GEMM_DISCARD=1 in the environment (read at library load) = main loop only, =2 = the whole
//     epilogue but no global stores.
#if defined(PHC_MEASURE_GEMM) && PHC_MEASURE_GEMM
#ifndef PHC_GEMM_PROBE
#define PHC_GEMM_PROBE 0
#endif
#include <cstdlib>
static inline int phc_gemm_discard() {
  static const int mode = [] {
    const char *e = getenv("PHC_GEMM_DISCARD");
    return e ? (atoi(e) == 2 ? 2 : 1) : 0;
  }();
  return mode;
}
#else
#if defined(PHC_GEMM_PROBE) && PHC_GEMM_PROBE
#error "PHC_GEMM_PROBE is a measurement build: add -DPHC_MEASURE_GEMM=1 (tools/build_variants.sh)"
#endif
#undef PHC_GEMM_PROBE
#define PHC_GEMM_PROBE 0
static inline int phc_gemm_discard() { return 0; }
#endif
