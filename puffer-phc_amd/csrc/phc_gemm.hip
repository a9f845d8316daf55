// phc_gemm.hip — half-precision MFMA GEMM with the twin-trunk epilogues fused (R19/R21).
//
// C[b] = A[b] · B[b]^T for b < batch, A [m, k] and B [n, k] row-major f16 / bf16 (both operands
// k-contiguous: the forward's X · W^T, and the input-gradient G · W with W pre-transposed),
// fp32 accumulation on v_mfma_f32_16x16x32_{f16,bf16}.  What the reference does between its GEMMs
// (nn.Linear bias + nn.SiLU forward, their backward and the bias gradient; policies/phc_policy.py:
// 10-61 under torch autograd) runs on the accumulator tile before it leaves the CU:
//   PHC_EPI_STORE     : out = acc
//   PHC_EPI_BIAS      : out = acc + bias
//   PHC_EPI_BIAS_SILU : pre = acc + bias (aux, fp32 or the operand type, nullable), out = silu(pre)
//   PHC_EPI_SILU_GRAD : out = acc * silu'(aux + bias) (bias nullable: aux is then the whole
//                       pre-activation, as BIAS_SILU writes it); bias_grad = column sums of out
//   PHC_EPI_BIAS_RELU : out = relu(acc + bias)   (the AMP discriminator's Linear + ReLU,
//                       policies/discriminator_policy.py:43-53)
//   PHC_EPI_BIAS_SILU_D : BIAS_SILU with aux = silu'(pre) = s (1 + pre (1 - s)), s = sigmoid(pre)
//                       (the only thing the backward needs of the pre-activation, in the same bytes)
//   PHC_EPI_DSILU_GRAD: out = acc * aux (aux = BIAS_SILU_D's silu'(pre), bias null); bias_grad as below:
//                       the input gradient's epilogue without the sigmoid (it was VALU-bound on it)
//   PHC_EPI_RELU_GRAD : out = acc * [aux + bias > 0] (aux = the forward's ReLU output, bias null:
//                       relu' from the output as torch's threshold_backward); bias_grad as above
// so no fp32 GEMM output makes an HBM round trip through a separate elementwise kernel.
//
// Tiling: 128 x 128 output tile per 256-thread block (4 waves as 2 x 2, 64 x 64 per wave =
// 4 x 4 MFMA blocks), K in steps of 64.  Operand tiles move global -> LDS by global_load_lds
// (16 B per lane, no VGPR staging) into two LDS buffers: tile t+1 streams in while the waves
// compute on tile t, one barrier per K-step.  The LDS image of a tile is [row][8 chunks of 16 B]
// with chunk c of row r stored at slot c ^ (r & 7) (the source address is pre-swizzled, the
// DMA's LDS side stays lane-linear), so the 16 rows one ds_read_b128 touches hit 8 distinct
// 16-B bank slots.  Blocks are renumbered XCD-major (bijective remap) so the blocks sharing an
// XCD's L2 walk the column tiles of the same A row panel.  m and n may be ragged (loads clamp
// to the last row, stores are masked); k must be a multiple of 64.
#include "phc_common.h"
#define PHC_MEASURE_GEMM_ONLY
#include "phc_measure.h"  // PHC_GEMM_PROBE / phc_gemm_discard(): measurement builds only

#include <hip/hip_ext.h>

#include <cstdlib>
#include <type_traits>

namespace phc {

constexpr int kGBK = 64;
// experiment knobs (compile-time): MFMA priority (off), the B operand's DMA issued PHC_GEMM_SPLIT_DMA
// eighths of a K-step after the A operand's (0 = together)
#ifndef PHC_GEMM_PRIO
#define PHC_GEMM_PRIO 0
#endif
#ifndef PHC_WGRAD_SPLIT
#define PHC_WGRAD_SPLIT 2
#endif
#ifndef PHC_GEMM_EPI_VW
#define PHC_GEMM_EPI_VW 8  // output columns per thread in the epilogue for f16 / bf16 outputs (4 or 8)
#endif
#ifndef PHC_GEMM_GRAD_U8
#define PHC_GEMM_GRAD_U8 2
#endif
#ifndef PHC_GEMM_SPLIT_A
#define PHC_GEMM_SPLIT_A 0
#endif
#ifndef PHC_GEMM_SPLIT_DMA
#define PHC_GEMM_SPLIT_DMA 2
#endif
// 256 x 256 tiles: the second wave of every SIMD (waves 4-7) issues its share of the next K-tile's
// DMA at MFMA groups PHC_GEMM_STG_A / _B instead of with waves 0-3, so one wave of each SIMD keeps
// the matrix pipe fed while the other issues its LDS-DMA (0 = off)
#ifndef PHC_GEMM_STG
#define PHC_GEMM_STG 0
#endif
#ifndef PHC_GEMM_STG_A
#define PHC_GEMM_STG_A 1
#endif
#ifndef PHC_GEMM_STG_B
#define PHC_GEMM_STG_B 3
#endif
using f4 = __attribute__((ext_vector_type(4))) float;
using h8 = __attribute__((ext_vector_type(8))) _Float16;
using b8 = __attribute__((ext_vector_type(8))) __bf16;
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const char *a, *b;
  int64_t a_bs, b_bs, lda, ldb;  // element strides
  int64_t m;
  int n, k, batch;
  const float *bias;
  void *aux;
  int aux_layout;
  void *out;
  int out_layout;
  int tg, tc;  // twin geometry of out / aux: logical column b * n + j -> group / column
  float *partial;
  int tiles_m, tiles_n;
  int discard;
  int aux_half;  // aux in the operand type T instead of fp32
  int nt;        // non-temporal epilogue traffic: 1 = out stores, 2 = aux stores, 4 = aux loads
  unsigned long long *clk;  // the launch's timer slot (phc_timer_take), null when untimed
};

// 4 consecutive aux values (fp32, or the operand type T when g.aux_half) at element offset off
template <typename T> __device__ __forceinline__ float4 aux_load4(const GemmArgs &g, int64_t off) {
  if (g.aux_half) {
    const uint2 raw = *reinterpret_cast<const uint2 *>(static_cast<const T *>(g.aux) + off);
    T h[4];
    __builtin_memcpy(h, &raw, sizeof(raw));
    return float4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
  return *reinterpret_cast<const float4 *>(static_cast<const float *>(g.aux) + off);
}
template <typename T> __device__ __forceinline__ float aux_load1(const GemmArgs &g, int64_t off) {
  return g.aux_half ? (float)static_cast<const T *>(g.aux)[off] : static_cast<const float *>(g.aux)[off];
}
template <typename T> __device__ __forceinline__ void aux_store4(const GemmArgs &g, int64_t off, const float v[4]) {
  if (g.aux_half) {
    const T h[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
    uint2 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    if (g.nt & 2)
      __builtin_nontemporal_store(__builtin_bit_cast(u2v, raw), reinterpret_cast<u2v *>(static_cast<T *>(g.aux) + off));
    else
      *reinterpret_cast<uint2 *>(static_cast<T *>(g.aux) + off) = raw;
  } else {
    *reinterpret_cast<float4 *>(static_cast<float *>(g.aux) + off) = float4{v[0], v[1], v[2], v[3]};
  }
}
template <typename T> __device__ __forceinline__ void aux_store1(const GemmArgs &g, int64_t off, float v) {
  if (g.aux_half) static_cast<T *>(g.aux)[off] = (T)v;
  else static_cast<float *>(g.aux)[off] = v;
}

// element offset of (row, logical column c) in a twin tensor of tg groups x tc columns
__device__ __forceinline__ int64_t gemm_twin_off(const GemmArgs &g, int layout, int64_t row, int c) {
  const int grp = c / g.tc, j = c - grp * g.tc;
  if (layout == PHC_LAYOUT_SPLIT) return row * (int64_t)(g.tg * g.tc) + c;
  return ((int64_t)grp * g.m + row) * g.tc + j;
}

// sigmoid from the hardware exp2 / reciprocal (1-ulp class, the values land in f16 / bf16 operands)
__device__ __forceinline__ float gemm_sigmoid(float a) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-a * 1.44269504088896341f));
}
__device__ __forceinline__ float gemm_silu(float a) { return a * gemm_sigmoid(a); }
// y = silu(z) (gemm_silu's arithmetic) and d = silu'(z) = s (1 + z (1 - s)) = s + y - y s from one
// sigmoid: one add and one fma on top of y (the store waves' epilogue is VALU-bound)
__device__ __forceinline__ void gemm_silu_d(float z, float &y, float &d) {
  const float s = gemm_sigmoid(z);
  y = z * s;
  d = __builtin_fmaf(-y, s, s + y);
}

// workgroup barrier for the epilogue's LDS hand-offs: waits for this wave's LDS operations only
// (lgkmcnt), not for its global stores (vmcnt), so the stores of one
// image pass drain while the next pass runs, and past the end of the block while the CU's next
// tile starts its main loop
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// workgroup barrier after which every wave's LDS-DMA (global_load_lds) writes have landed: each
// wave drains its own DMA (vmcnt), then the barrier.  __syncthreads() is NOT enough: its fence
// does not count LDS-DMA, and the compiler's own vmcnt for the DMA may land after the barrier
// (seen in the persistent tile loop: waves read operand tiles other waves' DMA had not written).
#ifndef PHC_GEMM_WAIT_BUILTIN
#define PHC_GEMM_WAIT_BUILTIN 1
#endif
__device__ __forceinline__ void dma_barrier() {
  if constexpr (PHC_GEMM_WAIT_BUILTIN) {
    // the wait as the compiler's own instruction (s_waitcnt with every counter 0): its wait-insertion
    // pass then knows every earlier fragment read has completed and does not drain the reads issued
    // after the barrier before the first MFMA that needs none of them (inline asm is opaque to it)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// Wave-specialised persistent tiles (PHC_GEMM_WS): waves 0-3 issue every operand DMA, waves 4-7 every
// epilogue store, so no wave's vmcnt holds both.  A DMA wave waits for its DMA (vmcnt 0) before the
// K-step barrier; a store wave waits only for its LDS reads (lgkmcnt 0): the previous tile's
// epilogue stores keep draining while the next tile's main loop runs (with one counter for loads and
// stores, a wave that had issued both would have to wait for its stores at the first K-step).
// `dma_wave` must be wave-uniform in an SGPR (readfirstlane): s_waitcnt ignores the exec mask.
#ifndef PHC_GEMM_WS
#define PHC_GEMM_WS 1
#endif
__device__ __forceinline__ void ws_barrier(bool dma_wave) {
  asm volatile("" ::: "memory");
  if (dma_wave) __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
  else __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0) only (vmcnt 63, expcnt 7)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename OutT> __device__ __forceinline__ void gemm_store(void *p, int64_t off, float v) {
  static_cast<OutT *>(p)[off] = (OutT)v;
}

template <typename OutT> __device__ __forceinline__ void gemm_store4(void *p, int64_t off, const float v[4], bool nt) {
  if constexpr (sizeof(OutT) == 4) {
    *reinterpret_cast<float4 *>(static_cast<float *>(p) + off) = float4{v[0], v[1], v[2], v[3]};
  } else {
    OutT h[4] = {(OutT)v[0], (OutT)v[1], (OutT)v[2], (OutT)v[3]};
    uint2 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    if (nt)
      __builtin_nontemporal_store(__builtin_bit_cast(u2v, raw), reinterpret_cast<u2v *>(static_cast<OutT *>(p) + off));
    else
      *reinterpret_cast<uint2 *>(static_cast<OutT *>(p) + off) = raw;
  }
}

// VW consecutive values at element offset off: fp32 as float4s, f16 / bf16 packed (16 B for VW 8)
template <typename OutT, int VW>
__device__ __forceinline__ void gemm_store_v(void *p, int64_t off, const float v[VW], bool nt) {
  if constexpr (sizeof(OutT) == 4 || VW == 4) {
#pragma unroll
    for (int h = 0; h < VW / 4; ++h) gemm_store4<OutT>(p, off + 4 * h, v + 4 * h, nt);
  } else {
    OutT h[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = (OutT)v[q];
    uint4 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    if (nt)
      __builtin_nontemporal_store(__builtin_bit_cast(u4v, raw), reinterpret_cast<u4v *>(static_cast<OutT *>(p) + off));
    else
      *reinterpret_cast<uint4 *>(static_cast<OutT *>(p) + off) = raw;
  }
}

template <typename T, int VW> __device__ __forceinline__ void aux_store_v(const GemmArgs &g, int64_t off, const float v[VW]) {
  if (VW == 8 && g.aux_half) {
    T h[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = (T)v[q];
    uint4 raw;
    __builtin_memcpy(&raw, h, sizeof(raw));
    if (g.nt & 2)
      __builtin_nontemporal_store(__builtin_bit_cast(u4v, raw), reinterpret_cast<u4v *>(static_cast<T *>(g.aux) + off));
    else
      *reinterpret_cast<uint4 *>(static_cast<T *>(g.aux) + off) = raw;
  } else {
#pragma unroll
    for (int h = 0; h < VW / 4; ++h) aux_store4<T>(g, off + 4 * h, v + 4 * h);
  }
}


// issue the global_load_lds of one R-row x BK-column operand tile (R * BK / 512 wave-instructions
// over the block's W waves).  BK = 64: LDS row r holds tile row r, its 16-B chunk c at slot
// c ^ (r & 7).  BK = 32: LDS row R holds tile rows 2R (chunks 0-3) and 2R + 1 (chunks 4-7), slot
// p ^ (R & 7); either way the 16 rows one ds_read_b128 fragment read touches hit 16 distinct
// 16-B bank slots in each of its lane groups (checked exhaustively for both layouts).
template <int R, int W, int BK>
__device__ __forceinline__ void stage_tile(const char *base, int64_t ld, int64_t row0, int64_t rows, int k0,
                                           char *lds_tile, int wave, int lane) {
  static_assert(BK == 64 || BK == 32, "BK 32 or 64");
  constexpr int kInstr = R * BK / 512;
  static_assert(kInstr % W == 0, "tile rows must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < kInstr / W; ++i) {
    const int q0 = (i * W + wave) * 64;  // first 16-B LDS slot this wave-instruction fills
    const int q = q0 + lane;
    const int lr = q >> 3, sl = (q & 7) ^ (lr & 7);
    const int r = BK == 64 ? lr : 2 * lr + (sl >> 2);
    const int c = BK == 64 ? sl : (sl & 3);
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const char *src = base + (gr * ld + k0 + (c << 3)) * 2;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (lds_void *)(lds_tile + q0 * 16), 16, 0, 0);
  }
}

// stage_tile for the wave-specialised tiles: the 4 DMA waves issue a whole R x 64 operand tile
// (R / 32 wave-instructions each).  Lane l of DMA wave w fills LDS rows w * 8 + (l >> 3) + 32 i; its
// chunk (l & 7) ^ (row & 7) does not depend on i, so one per-lane byte pointer per operand and tile
// (`lane_src`) plus wave-uniform offsets (k0, 32 i rows: SGPRs) address every instruction, and the
// LDS destination (M0) is scalar: the generic form's per-instruction row / pointer registers spilled
// once the DMA waves carried twice the instructions.  Rows are not clamped: whole tiles only.
struct WsSrc {
  const char *p;     // this lane's source byte pointer at k0 = 0, instruction 0
  int64_t row_step;  // bytes between the rows of instruction i and i + 1 (32 rows)
};
__device__ __forceinline__ WsSrc ws_src(const char *base, int64_t ld, int64_t row0, int wsg, int lane) {
  const int rl = wsg * 8 + (lane >> 3);
  const int c = (lane & 7) ^ ((lane >> 3) & 7);
  return {base + ((row0 + rl) * ld + (c << 3)) * 2, 32 * ld * 2};
}
template <int R>
__device__ __forceinline__ void stage_tile_ws(const WsSrc &src, int k0, char *lds_tile, int wsg) {
  constexpr int kInstr = R * 64 / 512 / 4;  // per DMA wave
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    const char *a = src.p + (int64_t)k0 * 2 + (int64_t)i * src.row_step;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)a,
                                     (lds_void *)(lds_tile + (i * 4 + wsg) * 64 * 16), 16, 0, 0);
  }
}

template <int BK, typename T>
__device__ __forceinline__ void read_frag(const char *lds_tile, int row, int chunk, T &f) {
  if constexpr (BK == 64) {
    f = *reinterpret_cast<const T *>(lds_tile + row * 128 + ((chunk ^ (row & 7)) << 4));
  } else {
    const int lr = row >> 1;
    f = *reinterpret_cast<const T *>(lds_tile + lr * 128 + ((((row & 1) << 2) + chunk) ^ (lr & 7)) * 16);
  }
}

// Tile geometry: BM x BN block tile, WGM x WGN waves, each owning a TM x TN = (BM / WGM) x
// (BN / WGN) sub-tile of (TM / 16) x (TN / 16) MFMA blocks; STAGES operand buffers in LDS.
template <int BM_, int BN_, int WGM_, int WGN_, int STAGES_, int BK_ = 64, int WPE_ = 1> struct Tile {
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, STAGES = STAGES_, BK = BK_;
  static constexpr int kWavesPerEU = WPE_;  // occupancy floor handed to the register allocator
  static constexpr int kWaves = WGM * WGN, kThreads = kWaves * 64;
  static constexpr int TM = BM / WGM, TN = BN / WGN, MI = TM / 16, NI = TN / 16;
  static constexpr int kStageBytes = (BM + BN) * BK * 2;
  static constexpr int kLoadsPerTile = (BM + BN) * BK / 512 / kWaves;  // glds per thread per K-step
  static constexpr int kOpBytes = STAGES * kStageBytes;
  // epilogue: the fp32 LDS image (reusing the operand buffers) holds the whole tile, or passes of
  // every wave's next TM / kEpPasses rows (so half the accumulators die after the first pass)
  static constexpr int kEpPasses = (BM * BN * 4 + kOpBytes - 1) / kOpBytes;
  static constexpr int kEpRows = BM / kEpPasses, kEpWaveRows = TM / kEpPasses, kEpMI = MI / kEpPasses;
  static constexpr int kLdsBytes = kOpBytes;
  static_assert(MI % kEpPasses == 0 && kEpRows * BN * 4 <= kOpBytes, "epilogue image must fit the operand buffers");
  static_assert(MI >= 1 && NI >= 1 && TM % 16 == 0 && TN % 16 == 0, "bad wave tile");
};

// first tile of XCD x when `total` tiles are split XCD-major over the 8 XCDs (bijective for any
// count), and how many it gets
__device__ __forceinline__ int xcd_first(int total, int x) {
  const int q8 = total / 8, r8 = total % 8;
  return x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
}
__device__ __forceinline__ int xcd_count(int total, int x) { return total / 8 + (x < total % 8 ? 1 : 0); }

// s_waitcnt vmcnt(n * L) for a run-time n <= NMAX (the immediate must be a constant)
template <int L, int NMAX> __device__ __forceinline__ void wait_vmcnt_tiles(int n) {
  static_assert(NMAX * L <= 63, "vmcnt range");
  if (NMAX >= 3 && n >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * L) : "memory");
  else if (NMAX >= 2 && n == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
  else if (NMAX >= 1 && n == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One K-step: issue the DMA of operand tile `next` into `wr` (when `issue`) and run the MFMAs of
// the current one from `rd`.  The two LDS buffers are restrict parameters, so after inlining the
// fragment reads and the LDS-DMA writes carry disjoint alias scopes and the compiler's wait
// insertion does not drain the in-flight DMA before the first fragment read.  A K-step is BK / 32
// MFMA sub-steps of 32; within it the (MI / 2) pairs of A fragments are walked as groups of
// 2 x NI MFMAs, the fragments of group q + 1 read from LDS while the MFMAs of group q run (two
// fragment register sets; B fragments re-read per sub-step).
template <typename T, typename TL, typename Stage>
__device__ __forceinline__ void gemm_step(const char *__restrict__ rd, char *__restrict__ wr, bool issue,
                                          const Stage &stage, int next, int wave, int lane,
                                          f4 (&acc)[TL::MI][TL::NI]) {
  constexpr int MI = TL::MI, NI = TL::NI, BK = TL::BK;
  using V8 = typename std::conditional<std::is_same<T, _Float16>::value, h8, b8>::type;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;
  constexpr int GP = MI / 2, NS = BK / 32, NG = NS * GP;
  // the B operand's DMA a quarter K-step after A's on 256 x 256 tiles (measured: -4 % on the
  // minibatch GEMMs); on the short K-steps of 128 x 128 tiles the late B tile is exposed (+25 %)
  constexpr int SPLIT = TL::BM >= 256 ? PHC_GEMM_SPLIT_DMA : 0;
  constexpr bool kStg = PHC_GEMM_STG && SPLIT && !PHC_GEMM_SPLIT_A && TL::kWaves == 8;
  const bool late = kStg && __builtin_amdgcn_readfirstlane(wave) >= 4;
  if (!SPLIT && issue) stage(next, wr, 3);
  if (SPLIT && !PHC_GEMM_SPLIT_A && issue && !late) stage(next, wr, 1);
  if (SPLIT && PHC_GEMM_SPLIT_A && issue) stage(next, wr, 4);
  const char *ta = rd;
  const char *tb = rd + TL::BM * BK * 2;
  static_assert(MI % 2 == 0, "A fragments are walked in pairs");
  V8 fa[2][2], fb[2][NI];
  auto load_b = [&](V8 *f, int s) {
#pragma unroll
    for (int j = 0; j < NI; ++j) read_frag<BK>(tb, wn * TL::TN + j * 16 + (lane & 15), s * 4 + (lane >> 4), f[j]);
  };
  auto load_a = [&](V8 *f, int s, int p) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
      read_frag<BK>(ta, wm * TL::TM + (2 * p + ii) * 16 + (lane & 15), s * 4 + (lane >> 4), f[ii]);
  };
  load_b(fb[0], 0);
  load_a(fa[0], 0, 0);
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int s = q / GP, p = q % GP;
    if (q + 1 < NG) {
      const int s1 = (q + 1) / GP, p1 = (q + 1) % GP;
      if (s1 != s) load_b(fb[s1 & 1], s1);
      load_a(fa[(q + 1) & 1], s1, p1);
    }
    if (SPLIT && PHC_GEMM_SPLIT_A && issue && q == PHC_GEMM_SPLIT_A * NG / 8) stage(next, wr, 8);
    if (kStg) {
      if (issue && late && q == PHC_GEMM_STG_A) stage(next, wr, 1);
      if (issue && q == (late ? PHC_GEMM_STG_B : SPLIT * NG / 8)) stage(next, wr, 2);
    } else if (SPLIT && issue && q == (SPLIT * NG / 8 < NG ? SPLIT * NG / 8 : NG - 1)) {
      stage(next, wr, 2);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this group's MFMAs
    if (PHC_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        f4 &c = acc[2 * p + ii][j];
        if constexpr (std::is_same<T, _Float16>::value)
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[q & 1][ii], fb[s & 1][j], c, 0, 0, 0);
        else
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q & 1][ii], fb[s & 1][j], c, 0, 0, 0);
      }
    if (PHC_GEMM_PRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
}

// ---- K-steps with the last MFMA group deferred across the barrier (PHC_GEMM_DEFER) -----------
// gemm_step runs a K-step's MFMA groups 0 .. NG-1 after the workgroup barrier that publishes its
// operand tile, so each K-step starts with every wave waiting for its first fragment reads (the
// barrier lines the waves up: both waves of a SIMD stall together).  Here the last group's MFMAs of
// K-step kt (fragments already in registers: fa[1], fb[1]) run after the barrier of K-step kt + 1,
// behind that step's first fragment reads (fa[0], fb[0]: other registers), so the LDS latency after
// the barrier hides behind 2 x NI MFMAs.  The operand buffer the deferred group came from may be
// overwritten by the next DMA as soon as the barrier passes: its fragments were read (lgkmcnt 0)
// before it.  gemm_flush runs the last deferred group after the final K-step.
#ifndef PHC_GEMM_DEFER
#define PHC_GEMM_DEFER 1
#endif
template <typename V8, int NI> struct GemmFrags {
  V8 fa[2][2], fb[2][NI];
};

template <typename T, typename V8, int NI>
__device__ __forceinline__ void mfma_group(const V8 (&a)[2], const V8 (&b)[NI], f4 *acc0, f4 *acc1) {
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    if constexpr (std::is_same<T, _Float16>::value) {
      acc0[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[j], acc0[j], 0, 0, 0);
      acc1[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[j], acc1[j], 0, 0, 0);
    } else {
      acc0[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j], acc0[j], 0, 0, 0);
      acc1[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j], acc1[j], 0, 0, 0);
    }
  }
}

template <typename T, typename TL, typename Stage, typename V8>
__device__ __forceinline__ void gemm_step_defer(const char *__restrict__ rd, char *__restrict__ wr, bool issue,
                                                bool carry, const Stage &stage, int next, int wave, int lane,
                                                f4 (&acc)[TL::MI][TL::NI], GemmFrags<V8, TL::NI> &f) {
  constexpr int MI = TL::MI, NI = TL::NI, BK = TL::BK;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;
  constexpr int GP = MI / 2, NS = BK / 32, NG = NS * GP;
  static_assert(NG % 2 == 0, "the deferred group must use the second fragment set");
  constexpr int SPLIT = TL::BM >= 256 ? PHC_GEMM_SPLIT_DMA : 0;
  if (!SPLIT && issue) stage(next, wr, 3);
  if (SPLIT && issue) stage(next, wr, 1);
  const char *ta = rd;
  const char *tb = rd + TL::BM * BK * 2;
  auto load_b = [&](V8 *fb, int s) {
#pragma unroll
    for (int j = 0; j < NI; ++j) read_frag<BK>(tb, wn * TL::TN + j * 16 + (lane & 15), s * 4 + (lane >> 4), fb[j]);
  };
  auto load_a = [&](V8 *fa, int s, int p) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      read_frag<BK>(ta, wm * TL::TM + (2 * p + ii) * 16 + (lane & 15), s * 4 + (lane >> 4), fa[ii]);
    }
  };
  // PHC_GEMM_PROBE 3 (measurement): B fragments read from LDS at the first K-step only — the main loop's cost
  // without B's LDS traffic (the bound of a B operand loaded straight into registers)
  const bool read_b = !(PHC_GEMM_PROBE == 3 && carry);
  if (read_b) load_b(f.fb[0], 0);
  load_a(f.fa[0], 0, 0);
  if (carry) {  // the previous K-step's last group, behind this step's first reads
    __builtin_amdgcn_sched_barrier(0);
    mfma_group<T, V8, NI>(f.fa[1], f.fb[1], acc[MI - 2], acc[MI - 1]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int q = 0; q + 1 < NG; ++q) {  // group NG - 1 is left in f.fa[1] / f.fb[1] for the next call
    const int s = q / GP, p = q % GP;
    const int s1 = (q + 1) / GP, p1 = (q + 1) % GP;
    if (s1 != s && read_b) load_b(f.fb[s1 & 1], s1);
    load_a(f.fa[(q + 1) & 1], s1, p1);
    if (SPLIT && issue && q == (SPLIT * NG / 8 < NG - 1 ? SPLIT * NG / 8 : NG - 2)) stage(next, wr, 2);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this group's MFMAs
    mfma_group<T, V8, NI>(f.fa[q & 1], f.fb[s & 1], acc[2 * p], acc[2 * p + 1]);
  }
}

template <typename T, typename TL, typename V8>
__device__ __forceinline__ void gemm_flush(f4 (&acc)[TL::MI][TL::NI], GemmFrags<V8, TL::NI> &f) {
  mfma_group<T, V8, TL::NI>(f.fa[1], f.fb[1], acc[TL::MI - 2], acc[TL::MI - 1]);
}

// ---- 256 x 256 main loop as a ping-pong of two wave groups (PHC_GEMM_8PH) -------------------
// The 8 waves form two groups (wave rows wm = 0 / 1, one wave of each on every SIMD) that run one
// workgroup barrier apart: while one group issues its LDS fragment reads and its share of the next
// K-tile's LDS-DMA, the other runs 16 MFMAs, then they swap — the SIMD's matrix pipe always has a
// wave with MFMA work.  A K-tile is four phases, one per quadrant of a wave's 128 x 64 output
// (64 rows x 32 columns x K 64 = 16 MFMAs): (A lo, B lo), (A lo, B hi), (A hi, B hi), (A hi, B lo),
// so a phase reads 12, 4, 8 or 0 fragments.  The operand tile moves in four half-tiles named by
// the phase that first reads them — B lo (the first 32 of every wave's 64 B rows), A lo (the first
// 64 of every wave's 128 A rows), B hi, A hi — each phase issuing one half-tile (2 glds per
// thread) of the NEXT K-tile, three phases before it is read; a counted vmcnt before the first
// barrier of the phase ahead of the read retires it, so two half-tiles stay in flight across
// every barrier and no wait drains the DMA.  Restaging a slot is >= 2 phases after its last read.
#ifndef PHC_GEMM_8PH
#define PHC_GEMM_8PH 0
#endif
#ifndef PHC_8PH_RELOAD_B  // 1: phase 4 re-reads the B lo fragments (one B register set instead of two)
#define PHC_8PH_RELOAD_B 0
#endif

// local row lr (0..127) of half-tile `hi` -> tile row: groups of SPAN rows, every other group
template <int SPAN> __device__ __forceinline__ int half_row(int lr, int hi) {
  return (lr / SPAN) * 2 * SPAN + hi * SPAN + lr % SPAN;
}

// glds of one half-tile: 128 rows x 64 k (16 KB), 2 wave-instructions per wave of 8; LDS rows keep
// the tile's [row][8 chunks] image (chunk c of row r at slot c ^ (r & 7))
template <int SPAN>
__device__ __forceinline__ void stage_half(const char *base, int64_t ld, int64_t row0, int64_t rows, int k0,
                                           char *lds_tile, int hi, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = i * 8 + wave;  // local rows 8j .. 8j + 7
    const int r0 = half_row<SPAN>(8 * j, hi);
    const int r = r0 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const char *src = base + (gr * ld + k0 + (c << 3)) * 2;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (lds_void *)(lds_tile + r0 * 128), 16, 0, 0);
  }
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// one phase's MFMAs: quadrant (QM, QN) of the wave's accumulators over the K-tile's two 32-deep steps
template <typename T, int QM, int QN, typename V8, int MI, int NI>
__device__ __forceinline__ void phase_mfma(f4 (&acc)[MI][NI], const V8 (&fa)[4][2], const V8 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        f4 &c = acc[4 * QM + ii][2 * QN + jj];
        if constexpr (std::is_same<T, _Float16>::value)
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][s], fb[jj][s], c, 0, 0, 0);
        else
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ii][s], fb[jj][s], c, 0, 0, 0);
      }
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void phase_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// One K-tile (four phases) from `rd`, issuing the next K-tile's half-tiles into `wr` (issue), or on
// the last K-tile `aux` (the grad epilogue's LDS-DMA of its first three aux passes, 12 glds per
// wave, issued in phase 1; then the counted waits leave them in flight).  rd / wr restrict: the
// compiler's own wait insertion does not drain the DMA before the fragment reads.
template <typename T, typename TL, typename AuxFn>
__device__ __forceinline__ void ktile_8ph(const char *__restrict__ rd, char *__restrict__ wr, bool issue, bool aux,
                                          const AuxFn &aux_fn, const char *A, int64_t lda, int64_t m0, int64_t m,
                                          const char *B, int64_t ldb, int64_t n0, int64_t n, int k0n, int wave,
                                          int lane, f4 (&acc)[TL::MI][TL::NI]) {
  using V8 = typename std::conditional<std::is_same<T, _Float16>::value, h8, b8>::type;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;
  const char *ta = rd;
  const char *tb = rd + TL::BM * 128;
  char *wa = wr;
  char *wb = wr + TL::BM * 128;
#if PHC_8PH_RELOAD_B
  V8 fa[4][2], fb0[2][2];
  V8(&fb1)[2][2] = fb0;
#else
  V8 fa[4][2], fb0[2][2], fb1[2][2];
#endif
  auto load_a = [&](int qm) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
        read_frag<64>(ta, wm * TL::TM + (4 * qm + ii) * 16 + (lane & 15), s * 4 + (lane >> 4), fa[ii][s]);
  };
  auto load_b = [&](V8(&f)[2][2], int qn) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        read_frag<64>(tb, wn * TL::TN + (2 * qn + jj) * 16 + (lane & 15), s * 4 + (lane >> 4), f[jj][s]);
  };
  // phase 1: issue B lo of the next K-tile (or the aux rows), read A lo + B lo, retire B hi
  if (issue) stage_half<32>(B, ldb, n0, n, k0n, wb, 0, wave, lane);
  if (aux) aux_fn();
  load_b(fb0, 0);
  load_a(0);
  if (issue) wait_vm<4>();
  else if (aux) wait_vm<14>();
  else wait_vm<2>();
  phase_barrier();
  phase_mfma<T, 0, 0>(acc, fa, fb0);
  phase_barrier();
  // phase 2: issue A lo, read B hi, retire A hi
  if (issue) stage_half<64>(A, lda, m0, m, k0n, wa, 0, wave, lane);
  load_b(fb1, 1);
  if (issue) wait_vm<4>();
  else if (aux) wait_vm<12>();
  else wait_vm<0>();
  phase_barrier();
  phase_mfma<T, 0, 1>(acc, fa, fb1);
  phase_barrier();
  // phase 3: issue B hi, read A hi
  if (issue) stage_half<32>(B, ldb, n0, n, k0n, wb, 1, wave, lane);
  load_a(1);
  phase_barrier();
  phase_mfma<T, 1, 1>(acc, fa, fb1);
  phase_barrier();
  // phase 4: issue A hi, (re-read B lo,) retire the next K-tile's A lo + B lo
  if (issue) stage_half<64>(A, lda, m0, m, k0n, wa, 1, wave, lane);
  if (PHC_8PH_RELOAD_B) load_b(fb0, 0);
  if (issue) wait_vm<4>();
  phase_barrier();
  phase_mfma<T, 1, 0>(acc, fa, fb0);
  phase_barrier();
}

// Grad epilogues (SiLU' / ReLU' with a half-precision aux) of 256 x 256 tiles stage the aux
// (pre-activation) rows through LDS: the rows of epilogue passes 0-2 move by LDS-DMA during the
// last K-step (into the operand buffer that step does not read and the 32 KB above the operand
// buffers), those of pass 3 during pass 1; the image then takes four 64-KB passes.  The epilogue
// reads aux from LDS instead of waiting on HBM round trips per row batch.
// the persistent tile loop's forward (store-only) epilogues on 256 x 256 tiles run wave-specialised;
// the tile's bias row is staged by the DMA waves into LDS past the operand buffers (kWsBiasBytes), so
// the store waves issue no global load at all (a load's wait would also wait for their stores)
// the silu'-aux pair instantiates its own kernels (a run-time switch in the shared body spilled the
// wave-specialised forward): the body sees the base epilogue plus kDeriv
constexpr int epi_base(int e) {
  return e == PHC_EPI_BIAS_SILU_D ? PHC_EPI_BIAS_SILU : (e == PHC_EPI_DSILU_GRAD ? PHC_EPI_SILU_GRAD : e);
}

template <int EPI, typename TL>
constexpr bool kWsTile = PHC_GEMM_WS && TL::BM == 256 && TL::BN == 256 && TL::kWaves == 8 && TL::STAGES == 2 &&
                         PHC_GEMM_DEFER && !PHC_GEMM_8PH &&
                         !(epi_base(EPI) == PHC_EPI_SILU_GRAD || EPI == PHC_EPI_RELU_GRAD);

constexpr int kWsBiasBytes = 1024;  // 256 fp32 bias values

template <int EPI, typename TL, typename OutT> struct EpStage {
  static constexpr bool kOn = (epi_base(EPI) == PHC_EPI_SILU_GRAD || EPI == PHC_EPI_RELU_GRAD) && TL::BM == 256 && TL::BN == 256 &&
                              TL::STAGES == 2 && TL::BK == 64 && TL::kWaves == 8 && sizeof(OutT) == 2;
  static constexpr int kPasses = kOn ? 4 : TL::kEpPasses;
  static constexpr int kSlotBytes = 64 * 256 * 2;  // one pass's aux rows: 64 x 256 half-precision values
  static constexpr int kLdsBytes = kOn ? TL::kOpBytes + kSlotBytes : TL::kLdsBytes + (kWsTile<EPI, TL> ? kWsBiasBytes : 0);
  static_assert(!kOn || TL::kOpBytes + kSlotBytes <= 163840, "LDS");
};

// One output tile: main loop + fused epilogue.  `wg` is the tile's linear index (n fastest within
// an A panel, then m, then batch); smem holds the operand stages and, after the main loop, the
// epilogue image.
// ROLE (wave-specialised persistent tiles, kWsTile): 0 = every wave does everything; 1 = the DMA
// waves' copy (operand DMA, main loop, image writes); 2 = the store waves' copy (main loop, image
// writes, image reads + global stores).  Separate instantiations, so the compiler's wait insertion
// for each role sees only its own memory operations (in one shared body it put vmcnt(0) waits meant
// for the DMA into the store waves' path as well).
template <typename T, typename OutT, int EPIX, typename TL, int ROLE = 0>
__device__ __forceinline__ void twin_gemm_tile(const GemmArgs &g, char *smem, int wg) {
  constexpr int EPI = epi_base(EPIX);
  constexpr bool kDeriv = EPIX != EPI;  // BIAS_SILU_D / DSILU_GRAD: the aux is silu'(pre)
  constexpr bool WS = ROLE != 0;
  constexpr int BM = TL::BM, BN = TL::BN, MI = TL::MI, NI = TL::NI;
  constexpr bool kGrad = EPI == PHC_EPI_SILU_GRAD || EPI == PHC_EPI_RELU_GRAD;  // aux read + column sums
  constexpr bool kBiasFwd = EPI == PHC_EPI_BIAS || EPI == PHC_EPI_BIAS_SILU || EPI == PHC_EPI_BIAS_RELU;
  int tid_ = threadIdx.x;
  // the persistent loop calls this once per tile: an opaque thread index keeps the compiler from
  // hoisting the per-thread epilogue addressing out of that loop (long-lived registers that spilled)
  asm volatile("" : "+v"(tid_));
  const int tid = tid_, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;
  static_assert(!WS || (TL::kWaves == 8 && TL::STAGES == 2 && PHC_GEMM_DEFER && !PHC_GEMM_8PH &&
                        !(EPI == PHC_EPI_SILU_GRAD || EPI == PHC_EPI_RELU_GRAD)),
                "wave specialisation: 8-wave, 2-stage deferred main loop, store-only epilogues");
  const int wsg = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform (SGPR)
  constexpr bool dma_wave = ROLE != 2;
  constexpr int kDW = WS ? TL::kWaves / 2 : TL::kWaves;  // waves issuing the operand DMA
  const int tn = wg % g.tiles_n;
  const int tm = (wg / g.tiles_n) % g.tiles_m;
  const int bt = wg / (g.tiles_n * g.tiles_m);
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const char *A = g.a + bt * g.a_bs * 2;
  const char *B = g.b + bt * g.b_bs * 2;
  using ES = EpStage<EPI, TL, OutT>;
  constexpr int EP = ES::kPasses, WR = TL::TM / EP;
  const int kt_last = (g.k / TL::BK - 1) & 1;  // the operand buffer the last K-step reads
  const bool stage_aux = ES::kOn && g.aux_half && g.tc % BN == 0 && g.n % BN == 0 && m0 + BM <= g.m;
  // aux slot s: the halves of the buffer the last K-step does not read, then the spare 32 KB
  auto aux_slot = [&](int sl) -> char * {
    return sl < 2 ? smem + (kt_last ^ 1) * TL::kStageBytes + sl * ES::kSlotBytes : smem + TL::kOpBytes;
  };
  // LDS-DMA of pass p's 64 aux rows (512 B each, image-row order) into a slot: wave-instruction i
  // moves rows 2i, 2i + 1; 4 per wave
  auto stage_aux_pass = [&](int p, char *slot) {
    if constexpr (ES::kOn) {
      const int64_t lc0 = (int64_t)bt * g.n + n0;
      const bool split = g.aux_layout == PHC_LAYOUT_SPLIT;
      const int64_t base0 = split ? lc0 : (lc0 / g.tc) * g.m * g.tc + lc0 % g.tc;
      const int64_t stride = split ? (int64_t)g.tg * g.tc : g.tc;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = wave * 4 + u;
        const int rr = 2 * i + (lane >> 5);
        const int64_t tr = m0 + (rr / WR) * TL::TM + p * WR + rr % WR;
        const T *src = static_cast<const T *>(g.aux) + base0 + tr * stride + (lane & 31) * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (lds_void *)(slot + i * 1024), 16, 0, 0);
      }
    }
  };

  f4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};

  {
  const int kt_n = g.k / TL::BK;
  const int64_t m0_ = m0;
  const int n0_ = n0;
  // WS: whole tiles stage through per-lane pointers (stage_tile_ws); ragged ones (never in the PPO
  // minibatch) through the clamped generic path
  const bool ws_full = WS && m0 + BM <= g.m && n0 + BN <= g.n;
  const WsSrc ws_a = ws_src(A, g.lda, m0, wsg, lane), ws_b = ws_src(B, g.ldb, n0, wsg, lane);
  if constexpr (ROLE == 1) {
    if (g.bias && (EPI == PHC_EPI_BIAS || EPI == PHC_EPI_BIAS_SILU || EPI == PHC_EPI_BIAS_RELU)) {
      // the tile's 256 bias values (4-B granules: a bias view may be 4-byte aligned only), wave w
      // values 64 w .. 64 w + 63; landed by the first K-step's vmcnt(0) + barrier
      int c = n0 + wsg * 64 + lane;
      c = c < g.n ? c : g.n - 1;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(g.bias + bt * g.n + c),
                                       (lds_void *)(smem + TL::kOpBytes + wsg * 256), 4, 0, 0);
    }
  }
  auto stage = [&](int kt, char *st, int parts = 3) {  // parts: 1 = A tile, 2 = B tile, 4 / 8 = A halves
    if (PHC_GEMM_PROBE == 2 && kt > 0) return;
    if (PHC_GEMM_PROBE == 3 && kt > 0) parts &= ~2;  // measurement: B staged once, its fragments kept
    if (WS && !dma_wave) return;                     // the store waves issue no DMA
    if constexpr (WS && PHC_GEMM_PROBE == 0) {
      if (ws_full) {
        if (parts & 1) stage_tile_ws<BM>(ws_a, kt * TL::BK, st, wsg);
        if (parts & 2) stage_tile_ws<BN>(ws_b, kt * TL::BK, st + BM * TL::BK * 2, wsg);
        return;
      }
    }
    const int64_t m0 = PHC_GEMM_PROBE == 1 ? 0 : m0_;
    const int n0 = PHC_GEMM_PROBE == 1 ? 0 : n0_;
    if (parts & 1) stage_tile<BM, kDW, TL::BK>(A, g.lda, m0, g.m, kt * TL::BK, st, wave, lane);
    if (parts & 4) stage_tile<BM / 2, kDW, TL::BK>(A, g.lda, m0, g.m, kt * TL::BK, st, wave, lane);
    if (parts & 8)
      stage_tile<BM / 2, kDW, TL::BK>(A, g.lda, m0 + BM / 2, g.m, kt * TL::BK, st + BM / 2 * TL::BK * 2, wave, lane);
    if (parts & 2) stage_tile<BN, kDW, TL::BK>(B, g.ldb, n0, g.n, kt * TL::BK, st + BM * TL::BK * 2, wave, lane);
  };
  if constexpr (PHC_GEMM_8PH && BM == 256 && BN == 256 && TL::kWaves == 8 && TL::STAGES == 2 && TL::BK == 64 &&
                TL::WGM == 2 && TL::WGN == 4) {
    // the ping-pong main loop: K-tile 0's half-tiles in read order, A lo + B lo retired, then the
    // second wave group (waves 4-7) falls one barrier behind the first and catches up at the end
    const bool second = (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) >= 4;
    char *b0 = smem + BM * 128;
    stage_half<32>(B, g.ldb, n0, g.n, 0, b0, 0, wave, lane);
    stage_half<64>(A, g.lda, m0, g.m, 0, smem, 0, wave, lane);
    stage_half<32>(B, g.ldb, n0, g.n, 0, b0, 1, wave, lane);
    stage_half<64>(A, g.lda, m0, g.m, 0, smem, 1, wave, lane);
    wait_vm<4>();
    phase_barrier();
    if (second) phase_barrier();
    auto aux3 = [&]() {
      stage_aux_pass(0, aux_slot(0));
      stage_aux_pass(1, aux_slot(1));
      stage_aux_pass(2, aux_slot(2));
    };
    for (int kt = 0; kt < kt_n; ++kt) {
      const bool last = kt + 1 == kt_n;
      ktile_8ph<T, TL>(smem + (kt & 1) * TL::kStageBytes, smem + ((kt + 1) & 1) * TL::kStageBytes, !last,
                       last && stage_aux, aux3, A, g.lda, m0, g.m, B, g.ldb, n0, g.n, (kt + 1) * TL::BK, wave, lane,
                       acc);
    }
    if (!second) phase_barrier();
  } else if constexpr (TL::STAGES == 2 && PHC_GEMM_DEFER) {
    using V8 = typename std::conditional<std::is_same<T, _Float16>::value, h8, b8>::type;
    GemmFrags<V8, NI> fr;
    stage(0, smem);
    for (int kt = 0; kt < kt_n; ++kt) {
      if constexpr (WS) ws_barrier(dma_wave);  // tile kt landed (every DMA wave drained its own)
      else dma_barrier();  // tile kt landed; buffer (kt+1)&1 is no longer read
      if (stage_aux && kt == kt_n - 1) {  // nothing else to stage: the epilogue's aux rows
        stage_aux_pass(0, aux_slot(0));
        stage_aux_pass(1, aux_slot(1));
        stage_aux_pass(2, aux_slot(2));
      }
      gemm_step_defer<T, TL>(smem + (kt & 1) * TL::kStageBytes, smem + ((kt + 1) & 1) * TL::kStageBytes, kt + 1 < kt_n,
                             kt > 0, stage, kt + 1, wave, lane, acc, fr);
    }
    gemm_flush<T, TL>(acc, fr);
  } else if constexpr (TL::STAGES == 2) {
    stage(0, smem);
    for (int kt = 0; kt < kt_n; ++kt) {
      dma_barrier();  // tile kt landed; buffer (kt+1)&1 is no longer read
      if (stage_aux && kt == kt_n - 1) {  // nothing else to stage: the epilogue's aux rows
        stage_aux_pass(0, aux_slot(0));
        stage_aux_pass(1, aux_slot(1));
        stage_aux_pass(2, aux_slot(2));
      }
      gemm_step<T, TL>(smem + (kt & 1) * TL::kStageBytes, smem + ((kt + 1) & 1) * TL::kStageBytes, kt + 1 < kt_n,
                       stage, kt + 1, wave, lane, acc);
    }
  } else {
    constexpr int S = TL::STAGES;
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
      if (i < kt_n) stage(i, smem + i * TL::kStageBytes);
    int rd = 0;
    for (int kt = 0; kt < kt_n; ++kt) {
      // this thread's part of tile kt has landed (the younger tiles may stay in flight); after the
      // barrier every thread's part has, and every wave is done with tile kt - 1's buffer, which
      // the DMA of tile kt + S - 1 refills
      const int younger = kt_n - 1 - kt < S - 2 ? kt_n - 1 - kt : S - 2;
      wait_vmcnt_tiles<TL::kLoadsPerTile, S - 2>(younger);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int wr = rd == 0 ? S - 1 : rd - 1;
      gemm_step<T, TL>(smem + rd * TL::kStageBytes, smem + wr * TL::kStageBytes, kt + S - 1 < kt_n, stage,
                       kt + S - 1, wave, lane, acc);
      rd = rd == S - 1 ? 0 : rd + 1;
    }
  }
  }

  if (g.discard == 1) {  // measurement aid: main loop only (keeps the accumulators alive)
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) static_cast<float *>(g.out)[0] = t;
    return;
  }
  // ---- epilogue.  The accumulators (lane: column lane & 15, rows 4 * (lane >> 4) + e of each
  // 16 x 16 block) go through LDS as an fp32 [rows][BN] image, 16-column groups XOR-swizzled by
  // (row >> 2) & 3 so both the scattered writes and the row reads are conflict-free; pass p holds
  // rows [p * kEpWaveRows, (p + 1) * kEpWaveRows) of every wave row.  Then each thread owns VW
  // consecutive columns of every kRowGroups-th image row — 8 for a half-precision output, so every
  // global store (and the input gradient's pre-activation load) moves 16 B per lane: the store
  // tail of a tile is issue-bound, and halving its instruction count is what shortens it — and
  // BN * sizeof(OutT) contiguous bytes per row.
  constexpr int VW = sizeof(OutT) == 2 ? PHC_GEMM_EPI_VW : 4;
  static_assert(VW == 4 || VW == 8, "4 or 8 columns per thread");
  // WS: only the store waves (the upper half of the workgroup) read the image and store
  constexpr int kStThreads = WS ? TL::kThreads / 2 : TL::kThreads;
  constexpr int kColThreads = BN / VW, kRowGroups = kStThreads / kColThreads;
  constexpr int kEpRows = BM / EP, kEpMI = MI / EP, IT = kEpRows / kRowGroups;
  static_assert(MI % EP == 0 && kEpRows * BN * 4 <= TL::kOpBytes, "epilogue passes");
  static_assert(!ES::kOn || kEpRows * BN * 4 <= TL::kStageBytes, "a staged-aux image pass fits one operand buffer");
  float *ep = reinterpret_cast<float *>(smem + (stage_aux ? kt_last * TL::kStageBytes : 0));
  const int st_tid = WS ? tid - (TL::kThreads - kStThreads) : tid;  // store role index (WS: waves 4-7)
  const int cv = (st_tid % kColThreads) * VW, rg = st_tid / kColThreads;
  const int gcol = n0 + cv;
  const bool vec = gcol + VW - 1 < g.n && g.tc % VW == 0;
  const bool full = vec && m0 + BM <= g.m;
  float biasv[VW], csum[VW];
#pragma unroll
  for (int q = 0; q < VW; ++q) {
    biasv[q] = 0.0f;
    csum[q] = 0.0f;
  }
  if constexpr (ROLE == 2) {
    if (EPI != PHC_EPI_STORE && g.bias) {
      const float *bl = reinterpret_cast<const float *>(smem + TL::kOpBytes);
#pragma unroll
      for (int q = 0; q < VW; ++q) biasv[q] = bl[cv + q];  // columns past n: clamped copies, masked
    }
  } else if (ROLE == 0 && EPI != PHC_EPI_STORE && g.bias) {
#pragma unroll
    for (int q = 0; q < VW; ++q)
      if (gcol + q < g.n) biasv[q] = g.bias[bt * g.n + gcol + q];
  }
  // element offsets of this thread's VW columns: base + row * stride in either layout
  const int lc = bt * g.n + gcol;
  const int grp = lc / g.tc, jc = lc - grp * g.tc;
  auto lin = [&](int layout, int64_t &base, int64_t &stride) {
    if (layout == PHC_LAYOUT_SPLIT) { base = lc; stride = (int64_t)g.tg * g.tc; }
    else { base = (int64_t)grp * g.m * g.tc + jc; stride = g.tc; }
  };
  int64_t ob, os, ab = 0, as = 0;
  lin(g.out_layout, ob, os);
  lin(g.aux_layout, ab, as);
  // tile row of this thread's it-th image row in pass p
  auto trow = [&](int p, int it) {
    const int r = rg + kRowGroups * it;
    return (r / WR) * TL::TM + p * WR + r % WR;
  };
  // the VW image values of image row r at this thread's columns
  auto read_image = [&](int r, float v[VW]) {
#pragma unroll
    for (int h = 0; h < VW / 4; ++h) {
      const float4 t = *reinterpret_cast<const float4 *>(&ep[r * BN + ((cv + 4 * h) ^ (((r >> 2) & 3) << 4))]);
      v[4 * h] = t.x; v[4 * h + 1] = t.y; v[4 * h + 2] = t.z; v[4 * h + 3] = t.w;
    }
  };
  using RawV = typename std::conditional<VW == 8, uint4, uint2>::type;  // VW half-precision values
  using RawN = typename std::conditional<VW == 8, u4v, u2v>::type;
  // the grad epilogues' aux (pre-activation) rows of a pass: the first batch is issued before the
  // pass's image write so its HBM latency overlaps the LDS round trip
  constexpr int U = (kGrad && VW == 8) ? PHC_GEMM_GRAD_U8 : 4;  // 16-B aux rows in flight per batch
  static_assert(IT % U == 0, "row batches");
  const bool pipe = kGrad && g.aux_half;
  RawV raw[2][kGrad ? U : 1];
  auto load_raw = [&](int pass, int b) {
    if constexpr (kGrad) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = m0 + trow(pass, b * U + u);
        const T *src = static_cast<const T *>(g.aux) + ab + row * as;
        raw[b & 1][u] = (g.nt & 4) ? __builtin_bit_cast(RawV, __builtin_nontemporal_load(reinterpret_cast<const RawN *>(src)))
                                   : *reinterpret_cast<const RawV *>(src);
      }
    }
  };
#pragma unroll
  for (int pass = 0; pass < EP; ++pass) {
    if (full && pipe && !stage_aux) load_raw(pass, 0);
    lds_barrier();  // operand tiles / the previous pass's image (and aux slot) are no longer read
    if (stage_aux && pass == 1) stage_aux_pass(3, aux_slot(0));  // pass 0's slot is free
#pragma unroll
    for (int i = pass * kEpMI; i < (pass + 1) * kEpMI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = wm * WR + (i - pass * kEpMI) * 16 + 4 * (lane >> 4) + e;
          const int c = wn * TL::TN + j * 16 + (lane & 15);
          ep[r * BN + (c ^ (((r >> 2) & 3) << 4))] = acc[i][j][e];
        }
    if (stage_aux) {
      // this wave's aux DMA for the pass has landed (all waves' after the barrier): passes 0-2 were
      // issued in the last K-step; pass 3's in pass 1, before the 2 x IT stores of passes 1 and 2
      if (pass == 0 || g.discard) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (pass == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * IT) : "memory");
    }
    lds_barrier();
    if (WS && dma_wave) continue;  // the DMA waves only write the image
    const char *aux_lds = stage_aux ? aux_slot(pass == 3 ? 0 : pass) : nullptr;
    if (full) {
      // whole tile in range, VW whole columns per thread: offsets are base + row * stride, rows
      // in batches of U; a half-precision aux is software-pipelined (batch b + 1's loads in
      // flight while batch b is processed), an fp32 one loaded per batch
#pragma unroll
      for (int i0 = 0; i0 < IT; i0 += U) {
        float av[U][VW];
        if constexpr (kGrad) {
          if (stage_aux) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int r = rg + kRowGroups * (i0 + u);
              T h[VW];
              const uint4 q4 = *reinterpret_cast<const uint4 *>(aux_lds + r * (BN * 2) + cv * 2);
              __builtin_memcpy(h, &q4, sizeof(h));
#pragma unroll
              for (int q = 0; q < VW; ++q) av[u][q] = (float)h[q];
            }
          } else if (pipe) {
            if (i0 + U < IT) load_raw(pass, i0 / U + 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              T h[VW];
              __builtin_memcpy(h, &raw[(i0 / U) & 1][u], sizeof(h));
#pragma unroll
              for (int q = 0; q < VW; ++q) av[u][q] = (float)h[q];
            }
          } else {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
              for (int h = 0; h < VW / 4; ++h) {
                const float4 a4 = aux_load4<T>(g, ab + (m0 + trow(pass, i0 + u)) * as + 4 * h);
                av[u][4 * h] = a4.x; av[u][4 * h + 1] = a4.y; av[u][4 * h + 2] = a4.z; av[u][4 * h + 3] = a4.w;
              }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = rg + kRowGroups * (i0 + u);
          const int64_t row = m0 + trow(pass, i0 + u);
          float v[VW];
          read_image(r, v);
          if constexpr (EPI == PHC_EPI_SILU_GRAD) {
            if constexpr (kDeriv) {  // aux = silu'(pre): one multiply
#pragma unroll
              for (int q = 0; q < VW; ++q) {
                v[q] = v[q] * av[u][q];
                csum[q] += v[q];
              }
            } else {
#pragma unroll
              for (int q = 0; q < VW; ++q) {
                const float x = av[u][q] + biasv[q];
                const float sg = gemm_sigmoid(x);
                v[q] = v[q] * sg * (1.0f + x * (1.0f - sg));
                csum[q] += v[q];
              }
            }
          } else if constexpr (EPI == PHC_EPI_RELU_GRAD) {
#pragma unroll
            for (int q = 0; q < VW; ++q) {
              v[q] = av[u][q] + biasv[q] > 0.0f ? v[q] : 0.0f;
              csum[q] += v[q];
            }
          } else if constexpr (kBiasFwd) {
#pragma unroll
            for (int q = 0; q < VW; ++q) v[q] += biasv[q];
            if constexpr (EPI == PHC_EPI_BIAS_SILU) {
              if constexpr (kDeriv) {
                float d[VW];
#pragma unroll
                for (int q = 0; q < VW; ++q) gemm_silu_d(v[q], v[q], d[q]);
                if (g.aux && g.discard != 2) aux_store_v<T, VW>(g, ab + row * as, d);
              } else {
                if (g.aux && g.discard != 2) aux_store_v<T, VW>(g, ab + row * as, v);
#pragma unroll
                for (int q = 0; q < VW; ++q) v[q] = gemm_silu(v[q]);
              }
            } else if constexpr (EPI == PHC_EPI_BIAS_RELU) {
#pragma unroll
              for (int q = 0; q < VW; ++q) v[q] = v[q] > 0.0f ? v[q] : 0.0f;
            }
          }
          if (g.discard != 2) gemm_store_v<OutT, VW>(g.out, ob + row * os, v, g.nt & 1);
        }
      }
      continue;
    }
    for (int it = 0; it < IT; ++it) {
      const int r = rg + kRowGroups * it;
      const int64_t row = m0 + trow(pass, it);
      if (row >= g.m) continue;
      float v[VW], a[VW];
      read_image(r, v);
#pragma unroll
      for (int q = 0; q < VW; ++q) a[q] = 0.0f;
      if constexpr (kGrad) {
        if (vec) {
#pragma unroll
          for (int h = 0; h < VW / 4; ++h) {
            const float4 a4 = aux_load4<T>(g, gemm_twin_off(g, g.aux_layout, row, lc) + 4 * h);
            a[4 * h] = a4.x; a[4 * h + 1] = a4.y; a[4 * h + 2] = a4.z; a[4 * h + 3] = a4.w;
          }
        } else {
          for (int q = 0; q < VW; ++q)
            if (gcol + q < g.n) a[q] = aux_load1<T>(g, gemm_twin_off(g, g.aux_layout, row, lc + q));
        }
      }
#pragma unroll
      for (int q = 0; q < VW; ++q) {
        if constexpr (kBiasFwd) {
          v[q] += biasv[q];
          a[q] = v[q];
          if constexpr (EPI == PHC_EPI_BIAS_SILU) {
            if constexpr (kDeriv) gemm_silu_d(a[q], v[q], a[q]);
            else v[q] = gemm_silu(v[q]);
          }
          if constexpr (EPI == PHC_EPI_BIAS_RELU) v[q] = v[q] > 0.0f ? v[q] : 0.0f;
        } else if constexpr (EPI == PHC_EPI_SILU_GRAD) {
          if constexpr (kDeriv) {
            v[q] = v[q] * a[q];
          } else {
            const float x = a[q] + biasv[q];
            const float sg = gemm_sigmoid(x);
            v[q] = v[q] * sg * (1.0f + x * (1.0f - sg));
          }
          csum[q] += gcol + q < g.n ? v[q] : 0.0f;
        } else if constexpr (EPI == PHC_EPI_RELU_GRAD) {
          v[q] = a[q] + biasv[q] > 0.0f ? v[q] : 0.0f;
          csum[q] += gcol + q < g.n ? v[q] : 0.0f;
        }
      }
      if (vec) {
        if constexpr (EPI == PHC_EPI_BIAS_SILU) {
          if (g.aux) aux_store_v<T, VW>(g, gemm_twin_off(g, g.aux_layout, row, lc), a);
        }
        gemm_store_v<OutT, VW>(g.out, gemm_twin_off(g, g.out_layout, row, lc), v, g.nt & 1);
      } else {
        for (int q = 0; q < VW; ++q) {
          if (gcol + q >= g.n) break;
          if constexpr (EPI == PHC_EPI_BIAS_SILU) {
            if (g.aux) aux_store1<T>(g, gemm_twin_off(g, g.aux_layout, row, lc + q), a[q]);
          }
          gemm_store<OutT>(g.out, gemm_twin_off(g, g.out_layout, row, lc + q), v[q]);
        }
      }
    }
  }
  if constexpr (kGrad) {
    if (!g.partial) return;
    // column sums over the tile's rows: row groups inside a wave by shuffle, the waves by LDS
    if constexpr (kColThreads < 64) {
#pragma unroll
      for (int o = kColThreads; o < 64; o <<= 1)
#pragma unroll
        for (int q = 0; q < VW; ++q) csum[q] += __shfl_xor(csum[q], o, 64);
    }
    lds_barrier();  // the epilogue image is no longer read
    constexpr int kSlots = kColThreads >= 64 ? kRowGroups : TL::kWaves;
    if (kColThreads >= 64 || lane < kColThreads) {
      const int wc = (kColThreads >= 64 ? (tid % kColThreads) : lane) * VW;
      const int slot = kColThreads >= 64 ? (tid / kColThreads) : wave;
#pragma unroll
      for (int h = 0; h < VW / 4; ++h)
        *reinterpret_cast<float4 *>(&ep[slot * BN + wc + 4 * h]) =
            float4{csum[4 * h], csum[4 * h + 1], csum[4 * h + 2], csum[4 * h + 3]};
    }
    lds_barrier();
    if (tid < kColThreads) {
      float o[VW];
#pragma unroll
      for (int q = 0; q < VW; ++q) o[q] = 0.0f;
      for (int w = 0; w < kSlots; ++w)
#pragma unroll
        for (int q = 0; q < VW; ++q) o[q] += ep[w * BN + cv + q];
      float *pr = g.partial + (int64_t)tm * (g.batch * g.n) + bt * g.n;
      for (int q = 0; q < VW; ++q)
        if (gcol + q < g.n) pr[gcol + q] = o[q];
    }
  }
}

// One tile per workgroup, XCD-major renumbering (bijective for any grid size); or (PERSIST, with
// fewer workgroups than tiles: phc_gemm_desc.max_workgroups) a persistent loop: step s hands tiles
// [s * nwg, (s + 1) * nwg) out XCD-major, so the workgroups sharing an XCD's L2 walk neighbouring
// tiles of the same A panels at every step.  Separate instantiations: inlined into one kernel the
// persistent copy's hoisted epilogue addresses spilled registers of the one-tile copy as well.
template <typename T, typename OutT, int EPI, typename TL, bool PERSIST>
__global__ __launch_bounds__(TL::kThreads) __attribute__((amdgpu_waves_per_eu(TL::kWavesPerEU, 8))) void k_twin_gemm(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [stage][A BM rows | B BN rows]
  const int nwg = gridDim.x, orig = blockIdx.x;
  launch_clock_begin(g.clk);
  if constexpr (!PERSIST) {
    twin_gemm_tile<T, OutT, EPI, TL>(g, smem, xcd_first(nwg, orig % 8) + orig / 8);
  } else if constexpr (kWsTile<EPI, TL>) {
    // the same tile sequence in both role copies: their barriers pair up one for one
    const int total = g.tiles_m * g.tiles_n * g.batch;
    const int x = orig % 8, l = orig / 8;
    auto walk = [&](auto role) {
      for (int base = 0; base < total; base += nwg) {
        const int cnt = total - base < nwg ? total - base : nwg;
        if (l < xcd_count(cnt, x)) twin_gemm_tile<T, OutT, EPI, TL, decltype(role)::value>(g, smem, base + xcd_first(cnt, x) + l);
        lds_barrier();  // the epilogue image is read out before the next tile's operands land
      }
    };
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < TL::kWaves / 2) walk(std::integral_constant<int, 1>{});
    else walk(std::integral_constant<int, 2>{});
  } else {
    const int total = g.tiles_m * g.tiles_n * g.batch;
    const int x = orig % 8, l = orig / 8;
    for (int base = 0; base < total; base += nwg) {
      const int cnt = total - base < nwg ? total - base : nwg;
      if (l < xcd_count(cnt, x)) twin_gemm_tile<T, OutT, EPI, TL>(g, smem, base + xcd_first(cnt, x) + l);
      lds_barrier();  // the epilogue image is read out before the next tile's operands land
    }
  }
  launch_clock_end(g.clk);
}

// ------------------------------------------------------------------ weight gradients (R21) --
// dW[b] = G[b]^T · Z[b] summed over the rows of G [rows, m] (the layer's output gradient) and
// Z [rows, n] (its input), both as the forward / input-gradient GEMMs wrote them: row-major, the
// feature dimension contiguous, the reduction over rows.  Operand tiles are therefore staged as
// [64 rows][BM or BN columns] (16-B chunks of the global rows, chunk c of LDS row r holding source
// chunk c ^ wg_swz(r)), and the MFMA fragments, which want 8 consecutive reduction rows per lane,
// are gathered column-wise by ds_read_b64_tr_b16: lane 4q + p of a 16-lane group names row q,
// columns 4p..4p+3 of a 4 x 16 block and lane i receives column i of the 4 rows.  The XOR moves
// 32-B column pairs, so the 8 rows a 32-lane half touches (k rows 8G + 4h + q of two groups) land
// on 8 distinct pairs of the 256-B bank window: conflict-free.  Split-K over the rows (S chunks,
// the split index slowest so every tile of a split streams the same rows at the same time and
// the XCD's L2 serves the re-reads); the fp32 partials go to out[s][b][m][n].
struct WgradArgs {
  const char *g, *z;
  int64_t g_bs, z_bs, ldg, ldz;  // element strides
  int64_t rows_per_split;
  int m, n, batch, splits;
  int tiles_m, tiles_n;
  float *out;
  int discard;
  unsigned long long *clk;  // the launch's timer slot, null when untimed
};

__device__ __forceinline__ int wg_swz(int r) { return ((r & 3) | ((r >> 1) & 4)) << 1; }

// global_load_lds of one 64-row x C-column operand tile (C / 8 wave-instructions over W waves)
template <int C, int W>
__device__ __forceinline__ void stage_tile_k(const char *base, int64_t ld, int64_t row0, int col0, int cols,
                                             char *lds_tile, int wave, int lane) {
  constexpr int CPR = C / 8;  // 16-B chunks per tile row
  static_assert(CPR >= 16, "the swizzle moves chunks within aligned groups of 16");
  static_assert((C / 8) % W == 0, "tile chunks must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < C / 8 / W; ++i) {
    const int q0 = (i * W + wave) * 64;
    const int q = q0 + lane;
    const int r = q / CPR, c = q % CPR;
    int gc = col0 + ((c ^ wg_swz(r)) << 3);
    gc = gc + 8 <= cols ? gc : cols - 8;  // ragged last tile: in-bounds filler, its outputs are masked
    const char *src = base + ((row0 + r) * ld + gc) * 2;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (lds_void *)(lds_tile + q0 * 16), 16, 0, 0);
  }
}

typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

// the 16x16x32 operand fragment of columns cb..cb+15, reduction rows 32 s..32 s+31 of a tile with
// `rowbytes`-byte rows: lane l gets column cb + (l & 15), rows 32 s + 8 (l >> 4) + 0..7
template <typename V8>
__device__ __forceinline__ void read_frag_tr(const char *lds_tile, int rowbytes, int cb, int s, int lane, V8 &f) {
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (cb >> 3) + (p >> 1);
  const int r0 = 32 * s + 8 * grp + q, r1 = r0 + 4;
  const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4v *)(lds_tile + r0 * rowbytes + ((ch ^ wg_swz(r0)) << 4) + 8 * (p & 1)));
  const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4v *)(lds_tile + r1 * rowbytes + ((ch ^ wg_swz(r1)) << 4) + 8 * (p & 1)));
  const s8v both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  f = __builtin_bit_cast(V8, both);
}

// One K-step: issue the DMA of the next operand tile into `wr` (when `issue`) and run the MFMAs
// of the current one from `rd`.  The two LDS buffers are restrict parameters, so after inlining
// the fragment reads and the LDS-DMA writes carry disjoint alias scopes and the compiler's wait
// insertion does not drain the in-flight DMA (vmcnt(0)) before the first fragment read.
template <typename T, typename TL>
__device__ __forceinline__ void wgrad_step(const char *__restrict__ rd, char *__restrict__ wr, bool issue,
                                           const char *A, int64_t lda, int am, const char *B, int64_t ldb, int bn,
                                           int64_t row0, int m0, int n0, int wave, int lane,
                                           f4 (&acc)[TL::MI][TL::NI]) {
  constexpr int BM = TL::BM, BN = TL::BN, MI = TL::MI, NI = TL::NI;
  using V8 = typename std::conditional<std::is_same<T, _Float16>::value, h8, b8>::type;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;
  constexpr int GP = MI / 2, NG = 2 * GP;
  if (issue) stage_tile_k<BM, TL::kWaves>(A, lda, row0, m0, am, wr, wave, lane);
  if (!PHC_WGRAD_SPLIT && issue) stage_tile_k<BN, TL::kWaves>(B, ldb, row0, n0, bn, wr + BM * 128, wave, lane);
  const char *ta = rd;
  const char *tb = rd + BM * 128;
  static_assert(MI % 2 == 0, "A fragments are walked in pairs");
  V8 fa[2][2], fb[2][NI];
  auto load_b = [&](V8 *f, int s) {
#pragma unroll
    for (int j = 0; j < NI; ++j) read_frag_tr(tb, BN * 2, wn * TL::TN + j * 16, s, lane, f[j]);
  };
  auto load_a = [&](V8 *f, int s, int p) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) read_frag_tr(ta, BM * 2, wm * TL::TM + (2 * p + ii) * 16, s, lane, f[ii]);
  };
  load_b(fb[0], 0);
  load_a(fa[0], 0, 0);
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int s = q / GP, p = q % GP;
    if (q + 1 < NG) {
      const int s1 = (q + 1) / GP, p1 = (q + 1) % GP;
      if (s1 != s) load_b(fb[s1 & 1], s1);
      load_a(fa[(q + 1) & 1], s1, p1);
    }
    if (PHC_WGRAD_SPLIT && issue && q == (PHC_WGRAD_SPLIT * NG / 8 < NG ? PHC_WGRAD_SPLIT * NG / 8 : NG - 1))
      stage_tile_k<BN, TL::kWaves>(B, ldb, row0, n0, bn, wr + BM * 128, wave, lane);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        f4 &c = acc[2 * p + ii][j];
        if constexpr (std::is_same<T, _Float16>::value)
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[q & 1][ii], fb[s & 1][j], c, 0, 0, 0);
        else
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[q & 1][ii], fb[s & 1][j], c, 0, 0, 0);
      }
  }
}

template <typename T, typename TL>
__global__ __launch_bounds__(TL::kThreads) void k_wgrad(WgradArgs g) {
  constexpr int BM = TL::BM, BN = TL::BN, MI = TL::MI, NI = TL::NI;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [stage][A 64 x BM | B 64 x BN]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;

  const int nwg = gridDim.x, orig = blockIdx.x;
  launch_clock_begin(g.clk);
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tn = wg % g.tiles_n;
  const int tm = (wg / g.tiles_n) % g.tiles_m;
  const int rest = wg / (g.tiles_n * g.tiles_m);
  const int bt = rest % g.batch, sp = rest / g.batch;
  const int m0 = tm * BM, n0 = tn * BN;
  const int64_t r0 = (int64_t)sp * g.rows_per_split;
  const char *A = g.g + bt * g.g_bs * 2;
  const char *B = g.z + bt * g.z_bs * 2;

  f4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};

  const int kt_n = (int)(g.rows_per_split / kGBK);
  stage_tile_k<BM, TL::kWaves>(A, g.ldg, r0, m0, g.m, smem, wave, lane);
  stage_tile_k<BN, TL::kWaves>(B, g.ldz, r0, n0, g.n, smem + BM * 128, wave, lane);
  for (int kt = 0; kt < kt_n; ++kt) {
    dma_barrier();  // tile kt landed; buffer (kt + 1) & 1 is no longer read
    char *cur = smem + (kt & 1) * TL::kStageBytes;
    char *nxt = smem + ((kt + 1) & 1) * TL::kStageBytes;
    wgrad_step<T, TL>(cur, nxt, kt + 1 < kt_n, A, g.ldg, g.m, B, g.ldz, g.n, r0 + (int64_t)(kt + 1) * kGBK, m0, n0,
                      wave, lane, acc);
  }
  if (g.discard) {
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) g.out[0] = t;
    return;
  }
  // partial tile straight from the accumulators: lane holds column (lane & 15) of rows
  // 4 (lane >> 4) + e of each 16 x 16 block (64-B row segments per store instruction)
  float *o = g.out + ((int64_t)sp * g.batch + bt) * g.m * g.n;
  const int cl = lane & 15, rl = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int col = n0 + wn * TL::TN + j * 16 + cl;
    if (col >= g.n) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = m0 + wm * TL::TM + i * 16 + rl;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (row + e < g.m) o[(int64_t)(row + e) * g.n + col] = acc[i][j][e];
    }
  }
  launch_clock_end(g.clk);
}

// Grouped form: the weight gradients of several layers in ONE launch, no split: every output tile
// of every layer reduces over all rows in one workgroup and adds (or stores) its fp32 result
// straight into the gradient buffers — deterministic, no partials.  With equal rows per tile the
// workgroups of all layers carry equal work, so the grid quantises over the CUs as a whole
// (the default trunk: 64 + 96 + 48 + 32 + 16 = 256 tiles of 256 x 256, one per CU).
constexpr int kWgradGroupMax = 8;
struct WgradProblem {
  const char *g, *z;
  int64_t g_bs, z_bs, ldg, ldz, ldd;
  float *dst[2];
  int m, n, batch, split_row, n_valid, tiles_m, tiles_n, block0;
};
struct WgradGroupArgs {
  WgradProblem p[kWgradGroupMax];
  int count, accumulate, discard;
  int64_t rows;
  unsigned long long *clk;  // the launch's timer slot, null when untimed
};

template <typename T, typename TL>
__global__ __launch_bounds__(TL::kThreads) void k_wgrad_group(WgradGroupArgs ga) {
  constexpr int BM = TL::BM, BN = TL::BN, MI = TL::MI, NI = TL::NI;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / TL::WGN, wn = wave % TL::WGN;

  const int nwg = gridDim.x, orig = blockIdx.x;
  launch_clock_begin(ga.clk);
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int pi = 0;
#pragma unroll
  for (int i = 1; i < kWgradGroupMax; ++i)
    if (i < ga.count && wg >= ga.p[i].block0) pi = i;
  const WgradProblem &P = ga.p[pi];
  const int local = wg - P.block0;
  const int tn = local % P.tiles_n;
  const int tm = (local / P.tiles_n) % P.tiles_m;
  const int bt = local / (P.tiles_n * P.tiles_m);
  const int m0 = tm * BM, n0 = tn * BN;
  const char *A = P.g + bt * P.g_bs * 2;
  const char *B = P.z + bt * P.z_bs * 2;
  const int64_t lda = P.ldg, ldb = P.ldz;
  const int am = P.m, bn = P.n;

  f4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};

  const int kt_n = (int)(ga.rows / kGBK);
  stage_tile_k<BM, TL::kWaves>(A, lda, 0, m0, am, smem, wave, lane);
  stage_tile_k<BN, TL::kWaves>(B, ldb, 0, n0, bn, smem + BM * 128, wave, lane);
  for (int kt = 0; kt < kt_n; ++kt) {
    dma_barrier();
    char *cur = smem + (kt & 1) * TL::kStageBytes;
    char *nxt = smem + ((kt + 1) & 1) * TL::kStageBytes;
    wgrad_step<T, TL>(cur, nxt, kt + 1 < kt_n, A, lda, am, B, ldb, bn, (int64_t)(kt + 1) * kGBK, m0, n0, wave,
                      lane, acc);
  }
  if (ga.discard) {
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) P.dst[0][0] = t;
    return;
  }
  // output row r of batch bt -> dst[bt + (r >= split_row)] row r (- split_row), columns < n_valid
  const int cl = lane & 15, rl = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int col = n0 + wn * TL::TN + j * 16 + cl;
    if (col >= P.n_valid) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = m0 + wm * TL::TM + i * 16 + rl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = row + e;
        if (r >= P.m) continue;
        const bool hi = r >= P.split_row;
        float *d = P.dst[bt + (hi ? 1 : 0)] + (int64_t)(hi ? r - P.split_row : r) * P.ldd + col;
        *d = ga.accumulate ? *d + acc[i][j][e] : acc[i][j][e];
      }
    }
  }
  launch_clock_end(ga.clk);
}

// tile configurations
using Tile128x2 = Tile<128, 128, 2, 2, 2>;
using Tile256sq = Tile<256, 256, 2, 4, 2>;
// the twin GEMM's 256 x 256 tile: 8 waves of 128 x 64 (default), or (measurement build PHC_GEMM_TW4=1)
// 4 waves of 128 x 128, one per SIMD, 512 registers: a third fewer LDS fragment reads per MFMA
#ifndef PHC_GEMM_TW4
#define PHC_GEMM_TW4 0
#endif
#if PHC_GEMM_TW4 && !(defined(PHC_MEASURE_GEMM) && PHC_MEASURE_GEMM)
#error "PHC_GEMM_TW4 is a measurement build: add -DPHC_MEASURE_GEMM=1"
#endif
using Tile256tw = typename std::conditional<PHC_GEMM_TW4 != 0, Tile<256, 256, 2, 2, 2>, Tile256sq>::type;
enum { kCfg128 = 0, kCfg256sq = 2 };

// 256 x 256 tiles when they still give every CU a tile (the rollout's 4096-row first layer), else
// 128 x 128 (the other 4096-row rollout GEMMs: a half- or quarter-filled grid of 256 x 256 tiles is
// slower there; PPO iteration 1.71 vs 1.68 M env-steps/s with the threshold at 64 tiles)
static int gemm_config(int64_t m, int n, int batch) {
  static const int forced = [] {
    const char *e = getenv("PHC_GEMM_CFG");  // tuning aid (tools/twin_gemm_probe.py)
    return e ? atoi(e) : -1;
  }();
  if (forced >= 0) return forced;
  static const int big_min = [] {
    const char *e = getenv("PHC_GEMM_BIG_MIN");  // tuning aid: fewest 256 x 256 tiles that select them
    return e ? atoi(e) : 256;
  }();
  const int64_t big = ((m + 255) / 256) * ((n + 255) / 256) * batch;
  return big >= big_min ? kCfg256sq : kCfg128;
}

static void gemm_tile_dims(int cfg, int *bm, int *bn) {
  *bm = cfg == kCfg256sq ? 256 : 128;
  *bn = cfg == kCfg256sq ? 256 : 128;
}

static phc_kernel_timer *g_gemm_timer = nullptr;  // bench.py measurement aid (phc_gemm_set_timer)
// phc_twin_gemm launches of more rows than this are offered to the timer (the PPO minibatch's trunk
// GEMMs; the rollout's 4,096-row layers are not part of the measured family)
constexpr int64_t kTimedMinRows = 4096;

template <typename T, typename OutT, int EPI, typename TL>
static void launch_one(const GemmArgs &g, int64_t blocks, hipStream_t st) {
  const bool persist = blocks < (int64_t)g.tiles_m * g.tiles_n * g.batch;
  auto kernel = persist ? k_twin_gemm<T, OutT, EPI, TL, true> : k_twin_gemm<T, OutT, EPI, TL, false>;
  constexpr int lds = EpStage<EPI, TL, OutT>::kLdsBytes;
  static bool attr = [&] {
    for (auto k : {k_twin_gemm<T, OutT, EPI, TL, true>, k_twin_gemm<T, OutT, EPI, TL, false>})
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(TL::kThreads), lds, st, g);
}

template <typename T, typename OutT, int EPI>
static void launch_cfg(int cfg, const GemmArgs &g, int64_t blocks, hipStream_t st) {
  if (cfg == kCfg256sq) launch_one<T, OutT, EPI, Tile256tw>(g, blocks, st);
  else launch_one<T, OutT, EPI, Tile128x2>(g, blocks, st);
}

template <typename T, typename OutT>
static void launch_epi(int epi, int cfg, const GemmArgs &g, int64_t blocks, hipStream_t st) {
  switch (epi) {
    case PHC_EPI_STORE: launch_cfg<T, OutT, PHC_EPI_STORE>(cfg, g, blocks, st); break;
    case PHC_EPI_BIAS: launch_cfg<T, OutT, PHC_EPI_BIAS>(cfg, g, blocks, st); break;
    case PHC_EPI_BIAS_SILU: launch_cfg<T, OutT, PHC_EPI_BIAS_SILU>(cfg, g, blocks, st); break;
    case PHC_EPI_SILU_GRAD: launch_cfg<T, OutT, PHC_EPI_SILU_GRAD>(cfg, g, blocks, st); break;
    case PHC_EPI_BIAS_RELU: launch_cfg<T, OutT, PHC_EPI_BIAS_RELU>(cfg, g, blocks, st); break;
    case PHC_EPI_BIAS_SILU_D: launch_cfg<T, OutT, PHC_EPI_BIAS_SILU_D>(cfg, g, blocks, st); break;
    case PHC_EPI_DSILU_GRAD: launch_cfg<T, OutT, PHC_EPI_DSILU_GRAD>(cfg, g, blocks, st); break;
    default: launch_cfg<T, OutT, PHC_EPI_RELU_GRAD>(cfg, g, blocks, st); break;
  }
}

static void launch_gemm(int dtype, int out_dtype, int epi, int cfg, const GemmArgs &g, int64_t blocks,
                        hipStream_t st) {
  if (dtype == PHC_DT_F16) {
    if (out_dtype == PHC_DT_F32) launch_epi<_Float16, float>(epi, cfg, g, blocks, st);
    else launch_epi<_Float16, _Float16>(epi, cfg, g, blocks, st);
  } else {
    if (out_dtype == PHC_DT_F32) launch_epi<__bf16, float>(epi, cfg, g, blocks, st);
    else launch_epi<__bf16, __bf16>(epi, cfg, g, blocks, st);
  }
}

template <typename T>
static void launch_wgrad(const WgradArgs &g, int64_t blocks, hipStream_t st) {
  using TL = Tile256sq;
  auto kernel = k_wgrad<T, TL>;
  static bool attr = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              TL::kLdsBytes);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(TL::kThreads), TL::kLdsBytes, st, g);
}

template <typename T>
static void launch_wgrad_group(const WgradGroupArgs &g, int64_t blocks, hipStream_t st) {
  using TL = Tile256sq;
  auto kernel = k_wgrad_group<T, TL>;
  static bool attr = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              TL::kLdsBytes);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(TL::kThreads), TL::kLdsBytes, st, g);
}

}  // namespace phc

using namespace phc;

extern "C" void phc_gemm_set_timer(phc_kernel_timer *timer) { g_gemm_timer = timer; }

extern "C" size_t phc_twin_gemm_workspace_bytes(int64_t m, int32_t batch, int32_t n) {
  if (m <= 0 || batch <= 0 || n <= 0) return 0;
  return (size_t)((m + 127) / 128) * batch * n * sizeof(float);  // one partial row per m tile (BM >= 128)
}

extern "C" int64_t phc_twin_gemm_m_tiles(int64_t m, int32_t n, int32_t batch) {
  if (m <= 0 || n <= 0 || batch <= 0) return 0;
  int bm, bn;
  gemm_tile_dims(gemm_config(m, n, batch), &bm, &bn);
  return (m + bm - 1) / bm;
}

extern "C" int phc_twin_gemm(const phc_gemm_desc *d, float *bias_grad, void *workspace, void *stream) {
  PHC_REQUIRE(d, "twin_gemm: null descriptor");
  PHC_REQUIRE(d->a && d->b && d->out, "twin_gemm: null operand");
  PHC_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0 && d->batch >= 1, "twin_gemm: bad shape");
  PHC_REQUIRE(d->k % kGBK == 0, "twin_gemm: k (%d) must be a multiple of %d (zero-pad the operands)", d->k, kGBK);
  PHC_REQUIRE(d->lda >= d->k && d->ldb >= d->k && d->lda % 8 == 0 && d->ldb % 8 == 0,
              "twin_gemm: leading dimensions must cover k and be multiples of 8");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(d->a) & 15) == 0 && (reinterpret_cast<uintptr_t>(d->b) & 15) == 0,
              "twin_gemm: operands must be 16-byte aligned");
  PHC_REQUIRE(d->dtype == PHC_DT_F16 || d->dtype == PHC_DT_BF16, "twin_gemm: operands must be f16 or bf16");
  PHC_REQUIRE(d->out_dtype == PHC_DT_F32 || d->out_dtype == d->dtype, "twin_gemm: out must be f32 or the operand type");
  PHC_REQUIRE(d->epilogue >= PHC_EPI_STORE && d->epilogue <= PHC_EPI_DSILU_GRAD, "twin_gemm: bad epilogue");
  const int epi = epi_base(d->epilogue);
  PHC_REQUIRE(!(d->epilogue == PHC_EPI_DSILU_GRAD && d->bias), "twin_gemm: DSILU_GRAD takes no bias (aux is silu'(pre))");
  const bool grad_epi = epi == PHC_EPI_SILU_GRAD || epi == PHC_EPI_RELU_GRAD;
  PHC_REQUIRE(d->twin_groups >= 1 && d->twin_cols >= 1 && d->twin_groups * d->twin_cols == d->batch * d->n,
              "twin_gemm: twin geometry must cover batch * n columns");
  PHC_REQUIRE(!(epi == PHC_EPI_BIAS || epi == PHC_EPI_BIAS_SILU || epi == PHC_EPI_BIAS_RELU) ||
                  d->bias,
              "twin_gemm: epilogue needs the bias");
  PHC_REQUIRE(!grad_epi || d->aux, "twin_gemm: SILU_GRAD / RELU_GRAD need the (pre-)activation (aux)");
  PHC_REQUIRE(d->aux_dtype == PHC_DT_F32 || d->aux_dtype == d->dtype, "twin_gemm: aux must be f32 or the operand type");
  PHC_REQUIRE(!bias_grad || (grad_epi && workspace),
              "twin_gemm: bias_grad needs the SILU_GRAD / RELU_GRAD epilogue and a workspace");
  PHC_REQUIRE(!workspace || grad_epi, "twin_gemm: a workspace receives the grad epilogues' bias-gradient partials");
  hipStream_t st = as_stream(stream);
  const int cfg = gemm_config(d->m, d->n, d->batch);
  int bm, bn;
  gemm_tile_dims(cfg, &bm, &bn);
  const int64_t tiles_m = (d->m + bm - 1) / bm;
  const int64_t tiles_n = (d->n + bn - 1) / bn;
  int64_t blocks = tiles_m * tiles_n * d->batch;
  PHC_REQUIRE(blocks < (1ll << 31), "twin_gemm: grid too large");
  PHC_REQUIRE(d->max_workgroups >= 0, "twin_gemm: max_workgroups must be >= 0");
  if (d->max_workgroups > 0 && d->max_workgroups < blocks) blocks = d->max_workgroups;
  // forward (store-only) epilogues on 256 x 256 tiles with more tiles than CUs: one persistent
  // workgroup per CU, wave-specialised (kWsTile), so each tile's epilogue stores drain under the
  // next tile's main loop.  PHC_GEMM_WS_GRID=0 keeps one tile per workgroup (A/B aid).
  static const bool ws_grid = [] {
    const char *e = getenv("PHC_GEMM_WS_GRID");
    return PHC_GEMM_WS && !(e && atoi(e) == 0);
  }();
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  if (ws_grid && d->max_workgroups == 0 && cfg == kCfg256sq && !grad_epi && blocks > cus) blocks = cus;
  GemmArgs g{};
  g.a = static_cast<const char *>(d->a);
  g.b = static_cast<const char *>(d->b);
  g.a_bs = d->a_batch_stride;
  g.b_bs = d->b_batch_stride;
  g.lda = d->lda;
  g.ldb = d->ldb;
  g.m = d->m;
  g.n = d->n;
  g.k = d->k;
  g.batch = d->batch;
  g.bias = d->bias;
  g.aux = d->aux;
  g.aux_layout = d->aux_layout;
  g.aux_half = d->aux_dtype == d->dtype ? 1 : 0;
  g.out = d->out;
  g.out_layout = d->out_layout;
  g.tg = d->twin_groups;
  g.tc = d->twin_cols;
  g.partial = static_cast<float *>(workspace);  // per-m-tile bias-gradient column sums (grad epilogues)
  g.tiles_m = (int)tiles_m;
  g.tiles_n = (int)tiles_n;
  g.discard = phc_gemm_discard();  // 0 in a product build (phc_measure.h)
  // Non-temporal epilogue traffic: an output of a whole PPO minibatch (tens to hundreds of MB,
  // far past the 4 MB per-XCD L2) streams out without evicting the operand panels the other CUs
  // are still re-reading; the pre-activation (written by the forward, read back once by the backward) always does.  Small
  // outputs (the rollout's 4096-row layers) stay cached for the next layer.  Measured: -8 % on a
  // minibatch's forward + input-gradient GEMMs (profiles/r02_gemm_experiments.txt).
  static const int64_t nt_out_min = [] {
    const char *e = getenv("PHC_GEMM_NT_OUT_MB");  // tuning aid
    return (int64_t)(e ? atof(e) * 1048576.0 : 64.0 * 1048576.0);
  }();
  static const int nt_aux = [] {
    const char *e = getenv("PHC_GEMM_NT_AUX");  // tuning aid: bit 1 = aux stores, bit 2 = aux loads
    return e ? atoi(e) : 3;
  }();
  const int64_t out_bytes = d->m * (int64_t)d->batch * d->n * (d->out_dtype == PHC_DT_F32 ? 4 : 2);
  g.nt = (out_bytes >= nt_out_min ? 1 : 0) | ((nt_aux & 1) ? 2 : 0) | ((nt_aux & 2) ? 4 : 0);
  // the training GEMMs only: the rollout's (inside its captured graph, 4096 rows) stay untimed
  // algorithmic FLOPs: the padded depth's zero columns are not counted (k_valid)
  const int kf = d->k_valid > 0 && d->k_valid < d->k ? d->k_valid : d->k;
  if (d->m > kTimedMinRows) g.clk = phc_timer_take(g_gemm_timer, st, blocks, 2.0 * (double)d->m * d->n * kf * d->batch);
  launch_gemm(d->dtype, d->out_dtype, d->epilogue, cfg, g, blocks, st);
  if (bias_grad) {
    const int c = d->batch * d->n;
    hipLaunchKernelGGL(k_colsum<>, dim3((unsigned)((c + 63) / 64)), dim3(256), 0, st,
                       static_cast<const float *>(workspace), (int)tiles_m, c, bias_grad);
  }
  return check_launch("twin_gemm");
}

extern "C" int phc_weight_grad(const phc_wgrad_desc *d, void *stream) {
  PHC_REQUIRE(d, "weight_grad: null descriptor");
  PHC_REQUIRE(d->g && d->z && d->out, "weight_grad: null operand");
  PHC_REQUIRE(d->m >= 8 && d->n >= 8 && d->m % 8 == 0 && d->n % 8 == 0 && d->batch >= 1,
              "weight_grad: m, n must be multiples of 8 (got %d, %d)", d->m, d->n);
  PHC_REQUIRE(d->splits >= 1 && d->rows > 0 && d->rows % ((int64_t)d->splits * kGBK) == 0,
              "weight_grad: rows (%lld) must be a multiple of 64 * splits (%d)", (long long)d->rows, d->splits);
  PHC_REQUIRE(d->ldg >= d->m && d->ldz >= d->n && d->ldg % 8 == 0 && d->ldz % 8 == 0,
              "weight_grad: leading dimensions must cover the columns and be multiples of 8");
  PHC_REQUIRE(d->g_batch_stride % 8 == 0 && d->z_batch_stride % 8 == 0, "weight_grad: batch strides must be multiples of 8");
  PHC_REQUIRE((reinterpret_cast<uintptr_t>(d->g) & 15) == 0 && (reinterpret_cast<uintptr_t>(d->z) & 15) == 0,
              "weight_grad: operands must be 16-byte aligned");
  PHC_REQUIRE(d->dtype == PHC_DT_F16 || d->dtype == PHC_DT_BF16, "weight_grad: operands must be f16 or bf16");
  const int64_t tiles_m = (d->m + 255) / 256, tiles_n = (d->n + 255) / 256;
  const int64_t blocks = tiles_m * tiles_n * d->batch * d->splits;
  PHC_REQUIRE(blocks < (1ll << 31), "weight_grad: grid too large");
  WgradArgs g{};
  g.g = static_cast<const char *>(d->g);
  g.z = static_cast<const char *>(d->z);
  g.g_bs = d->g_batch_stride;
  g.z_bs = d->z_batch_stride;
  g.ldg = d->ldg;
  g.ldz = d->ldz;
  g.rows_per_split = d->rows / d->splits;
  g.m = d->m;
  g.n = d->n;
  g.batch = d->batch;
  g.splits = d->splits;
  g.tiles_m = (int)tiles_m;
  g.tiles_n = (int)tiles_n;
  g.out = d->out;
  g.discard = phc_gemm_discard() ? 1 : 0;
  hipStream_t st = as_stream(stream);
  g.clk = phc_timer_take(g_gemm_timer, st, blocks, 2.0 * (double)d->m * d->n * d->rows * d->batch);
  if (d->dtype == PHC_DT_F16) launch_wgrad<_Float16>(g, blocks, st);
  else launch_wgrad<__bf16>(g, blocks, st);
  return check_launch("weight_grad");
}

extern "C" int phc_weight_grad_group(const phc_wgrad_problem *probs, int32_t count, int64_t rows, int32_t dtype,
                                     int32_t accumulate, void *stream) {
  PHC_REQUIRE(probs && count >= 1 && count <= kWgradGroupMax, "weight_grad_group: 1..%d problems", kWgradGroupMax);
  PHC_REQUIRE(rows > 0 && rows % kGBK == 0, "weight_grad_group: rows (%lld) must be a multiple of %d",
              (long long)rows, kGBK);
  PHC_REQUIRE(dtype == PHC_DT_F16 || dtype == PHC_DT_BF16, "weight_grad_group: operands must be f16 or bf16");
  WgradGroupArgs ga{};
  int64_t blocks = 0;
  double flops = 0.0;
  for (int i = 0; i < count; ++i) {
    const phc_wgrad_problem &d = probs[i];
    PHC_REQUIRE(d.g && d.z && d.dst[0], "weight_grad_group: problem %d: null operand", i);
    PHC_REQUIRE(d.m >= 8 && d.n >= 8 && d.m % 8 == 0 && d.n % 8 == 0 && (d.batch == 1 || d.batch == 2),
                "weight_grad_group: problem %d: m, n multiples of 8, batch 1 or 2", i);
    PHC_REQUIRE(d.ldg >= d.m && d.ldz >= d.n && d.ldg % 8 == 0 && d.ldz % 8 == 0 && d.g_batch_stride % 8 == 0 &&
                    d.z_batch_stride % 8 == 0,
                "weight_grad_group: problem %d: leading dimensions / batch strides", i);
    PHC_REQUIRE((reinterpret_cast<uintptr_t>(d.g) & 15) == 0 && (reinterpret_cast<uintptr_t>(d.z) & 15) == 0,
                "weight_grad_group: problem %d: operands must be 16-byte aligned", i);
    PHC_REQUIRE(d.n_valid >= 1 && d.n_valid <= d.n && d.ldd >= d.n_valid && d.split_row >= 1,
                "weight_grad_group: problem %d: destination geometry", i);
    const int ndst = d.batch + (d.split_row < d.m ? 1 : 0);
    PHC_REQUIRE(ndst <= 2 && (ndst < 2 || d.dst[1]), "weight_grad_group: problem %d: needs dst[1]", i);
    WgradProblem &p = ga.p[i];
    p.g = static_cast<const char *>(d.g);
    p.z = static_cast<const char *>(d.z);
    p.g_bs = d.g_batch_stride;
    p.z_bs = d.z_batch_stride;
    p.ldg = d.ldg;
    p.ldz = d.ldz;
    p.ldd = d.ldd;
    p.dst[0] = d.dst[0];
    p.dst[1] = d.dst[1];
    p.m = d.m;
    p.n = d.n;
    p.batch = d.batch;
    p.split_row = d.split_row;
    p.n_valid = d.n_valid;
    p.tiles_m = (d.m + 255) / 256;
    p.tiles_n = (d.n + 255) / 256;
    p.block0 = (int)blocks;
    blocks += (int64_t)p.tiles_m * p.tiles_n * d.batch;
    flops += 2.0 * (double)d.m * d.n_valid * rows * d.batch;  // algorithmic: the padded columns not counted
  }
  PHC_REQUIRE(blocks < (1ll << 31), "weight_grad_group: grid too large");
  ga.count = count;
  ga.accumulate = accumulate ? 1 : 0;
  ga.rows = rows;
  ga.discard = phc_gemm_discard() ? 1 : 0;
  hipStream_t st = as_stream(stream);
  ga.clk = phc_timer_take(g_gemm_timer, st, blocks, flops);
  if (dtype == PHC_DT_F16) launch_wgrad_group<_Float16>(ga, blocks, st);
  else launch_wgrad_group<__bf16>(ga, blocks, st);
  return check_launch("weight_grad_group");
}
