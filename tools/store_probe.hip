// Store-throughput probe for the GEMM epilogue question: how long do B blocks of 512 threads take
// to write S KB each (16 B per lane per store, rows of 512 B as the 256 x 256 f16 epilogue writes
// them), with plain or non-temporal stores, as a function of B (one block per CU up to 256)?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned u4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_store(uint4 *out, int64_t row_stride_16, int rows_per_block, int nt,
                                               int lds_bytes_dummy) {
  extern __shared__ char lds[];  // sized by the launch: one block per CU when 128 KB
  if (lds_bytes_dummy < 0) lds[threadIdx.x] = 0;
  const int tid = threadIdx.x;
  const uint4 v = make_uint4(tid, blockIdx.x, 1, 2);
  if (nt >= 2) {  // contiguous: the block's bytes as one span, 8 KB per block-wide store
    uint4 *base = out + (int64_t)blockIdx.x * rows_per_block * 32;
    for (int i = tid; i < rows_per_block * 32; i += 512) {
      if (nt == 3) __builtin_nontemporal_store(__builtin_bit_cast(u4v, v), reinterpret_cast<u4v *>(base + i));
      else base[i] = v;
    }
    return;
  }
  if (nt >= 4) {  // the register-direct epilogue's pattern over 256 x 256 f16 tile images (8 waves of 128 x 64)
    const int lane = tid & 63, w = tid >> 6, wm = w / 4, wn = w % 4;
    for (int img = 0; img < rows_per_block / 256; ++img) {
      const int64_t r0 = (int64_t)blockIdx.x * rows_per_block + img * 256 + wm * 128;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          int r, c16;  // row in the wave's 128, 16-B column chunk in the 512-B row
          if (nt == 4) {  // MFMA-native: lane = row (lane & 15), 4 lanes per row spread over the wave's rows
            const int g = lane >> 4;
            r = i * 16 + (lane & 15);
            c16 = wn * 8 + jp * 4 + ((g & 1) << 1) + (g >> 1);
          } else {  // 4 consecutive lanes per row: 64 B coalesced per lane quad
            r = i * 16 + (lane >> 2);
            c16 = wn * 8 + jp * 4 + (lane & 3);
          }
          uint4 *p = out + (r0 + r) * row_stride_16 + c16;
          __builtin_nontemporal_store(__builtin_bit_cast(u4v, v), reinterpret_cast<u4v *>(p));
        }
    }
    return;
  }
  const int col = tid % 32, rg = tid / 32;  // 32 threads x 16 B = one 512-B row segment, 16 rows per pass
  const int64_t block_row0 = (int64_t)blockIdx.x * rows_per_block;
  for (int r = rg; r < rows_per_block; r += 16) {
    uint4 *p = out + (block_row0 + r) * row_stride_16 + col;
    if (nt) __builtin_nontemporal_store(__builtin_bit_cast(u4v, v), reinterpret_cast<u4v *>(p));
    else *p = v;
  }
}

int main(int argc, char **argv) {
  const int kb = argc > 1 ? atoi(argv[1]) : 256;  // KB written per block
  const int rows = kb * 1024 / 512;
  const int64_t stride16 = 4096 * 2 / 16;  // rows 8 KB apart (a 4096-column f16 tensor)
  const int max_blocks = 2048;
  uint4 *out = nullptr;
  if (hipMalloc(&out, (size_t)max_blocks * rows * stride16 * 16) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int lds = 128 * 1024;
  hipFuncSetAttribute(reinterpret_cast<const void *>(k_store), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  for (int nt = 0; nt < 6; ++nt)
    for (int blocks : {32, 128, 256, 1024}) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_store, dim3(blocks), dim3(512), lds, 0, out, stride16, rows, nt, 0);
      hipEventRecord(e0);
      const int reps = 20;
      for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k_store, dim3(blocks), dim3(512), lds, 0, out, stride16, rows, nt, 0);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      const double bytes = (double)blocks * kb * 1024;
      printf("nt=%d blocks=%5d KB/block=%d  %8.2f us  %7.2f TB/s  %6.1f GB/s per block\n", nt, blocks, kb, us,
             bytes / us / 1e6, bytes / blocks / us / 1e3);
    }
  hipFree(out);
  return 0;
}
