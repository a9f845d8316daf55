// phc_measure.h — measurement-only instrumentation of the env kernels (never part of a product build).
// A product build (Makefile default) defines nothing here: ENV_PHASE / ENV_PHASE_USE expand to nothing
// and phc_env_phase_copy is absent from the library.  tools/build_variants.sh builds the measurement
// library with -DPHC_MEASURE_ENV_PHASES=1: lane 0 of every wave of k_env_replay stamps the constant clock
// at its phase boundaries into g_env_phase[wave][8] (tools/env_phase_probe.py reads them):
// 0 start, 1 scalars used, 2 frame rows in LDS, 3 replay + reward done, 4 observation row written,
// 5 rows copied out, 6 stats flushed.
#pragma once

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
