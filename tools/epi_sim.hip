// GEMM epilogue simulator: B blocks of 512 threads (one per CU: 128 KB LDS each) that each spin for
// `spin_us` (a stand-in for a 256 x 256 tile's main loop) and then store a tile's epilogue: two
// passes of 8 rows x 16 B per thread into `out` and `aux` (256 KB per tile, rows 8 KB apart), as
// k_twin_gemm's BIAS_SILU epilogue does.  Prints the launch time against tiles_per_cu x spin: the
// difference is the epilogue's exposed cost per tile.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/epi_sim tools/epi_sim.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned u4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_tile(uint4 *out, uint4 *aux, int64_t ld16, uint32_t spin_ticks, int mode,
                                              uint32_t stagger_ticks, int first_wave) {
  extern __shared__ char lds[];
  if (spin_ticks == 0xffffffffu) lds[threadIdx.x] = 0;
  // stagger (argv[3] > 0): every other workgroup of the first dispatch wave spins that much longer
  uint32_t ticks = spin_ticks;
  if (stagger_ticks && blockIdx.x < first_wave && (blockIdx.x & 1)) ticks += stagger_ticks;
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
  if (mode == 3) return;  // spin only
  const int tid = threadIdx.x, col = tid % 32, rg = tid / 32;
  const int64_t row0 = (int64_t)blockIdx.x * 256;
  const uint4 v = make_uint4(tid, blockIdx.x, 1, 2);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int64_t r = row0 + pass * 128 + rg + 16 * it;
      if (mode == 1) {
        __builtin_nontemporal_store(__builtin_bit_cast(u4v, v), reinterpret_cast<u4v *>(aux + r * ld16 + col));
        __builtin_nontemporal_store(__builtin_bit_cast(u4v, v), reinterpret_cast<u4v *>(out + r * ld16 + col));
      } else if (mode == 2) {  // out only
        out[r * ld16 + col] = v;
      } else {
        aux[r * ld16 + col] = v;
        out[r * ld16 + col] = v;
      }
    }
    __syncthreads();
  }
}

int main(int argc, char **argv) {
  const float spin_us = argc > 1 ? atof(argv[1]) : 58.0f;
  const int tiles_per_cu = argc > 2 ? atoi(argv[2]) : 6;
  const float stagger_us = argc > 3 ? atof(argv[3]) : 0.0f;
  int cus = 0, khz = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const double ticks_per_us = khz / 1000.0;
  const int blocks = cus * tiles_per_cu;
  const int64_t ld16 = 8192 / 16;  // 8-KB rows
  const size_t bytes = (size_t)blocks * 256 * 8192;
  uint4 *out = nullptr, *aux = nullptr;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&aux, bytes) != hipSuccess) return 1;
  const int lds = 128 * 1024;
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_tile), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs %d, wall clock %.1f MHz, %d blocks (%d per CU), spin %.1f us, stagger %.1f us\n", cus, ticks_per_us, blocks,
         tiles_per_cu, spin_us, stagger_us);
  const char *names[] = {"plain out+aux", "nt out+aux", "plain out only", "spin only"};
  for (int mode : {3, 0, 1, 2}) {
    const uint32_t ticks = (uint32_t)(spin_us * ticks_per_us), st = (uint32_t)(stagger_us * ticks_per_us);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_tile, dim3(blocks), dim3(512), lds, 0, out, aux, ld16, ticks, mode, st, cus);
    hipEventRecord(e0);
    const int reps = 5;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k_tile, dim3(blocks), dim3(512), lds, 0, out, aux, ld16, ticks, mode, st, cus);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-16s %8.1f us  (%.2f us per tile over the spin)\n", names[mode], us, (us - tiles_per_cu * spin_us) / tiles_per_cu);
  }
  return 0;
}
