// phc_store.hip — Experience.store on the device (R18, clean_pufferl/structs.py:113-131).
//
// The reference appends the mask-true rows of one rollout step to the flat training buffer
// (`idx = nonzero(mask)`, CPU copies, a host-side ptr).  Here one scan block ranks the mask,
// clamps to the remaining capacity and advances a DEVICE cursor; a copy kernel moves every
// field of every taken row.  No host value enters the launch, so the whole rollout step can be
// replayed from a hipGraph; running sums of {n_valid, taken} let the host read back once per rollout.
#include "phc_common.h"

namespace phc {

constexpr int kScanThreads = 1024;
#ifndef PHC_COPY_FLAT
#define PHC_COPY_FLAT 1
#endif

struct RowFields {
  phc_row_field f[PHC_MAX_ROW_FIELDS];
  int n;
};

// workspace: [0] = start row (int64), then rank[n] (int32)
__global__ __launch_bounds__(kScanThreads) void k_rank_mask(const uint8_t *__restrict__ mask, int64_t n,
                                                            int64_t *__restrict__ cursor, int64_t capacity,
                                                            int64_t *__restrict__ counts, int64_t *__restrict__ ws) {
  __shared__ int64_t warp_tot[kScanThreads / 64];
  __shared__ int64_t carry;
  int32_t *rank = reinterpret_cast<int32_t *>(ws + 1);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  // 4 consecutive rows per thread: one pass covers 4096 rows (a whole rollout step at 4096 envs)
  for (int64_t base = 0; base < n; base += 4 * kScanThreads) {
    const int64_t i0 = base + 4 * t;
    int f[4];
    if (mask && i0 + 3 < n) {  // the 4 flags by one unconditional 4-byte-granule read (no per-flag waits)
      uint8_t m4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) m4[q] = mask[i0 + q];
#pragma unroll
      for (int q = 0; q < 4; ++q) f[q] = m4[q] ? 1 : 0;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) f[q] = (i0 + q < n && (!mask || mask[i0 + q])) ? 1 : 0;
    }
    const int v = (f[0] + f[1]) + (f[2] + f[3]);
    // inclusive wave scan of the per-thread counts
    int s = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(s, o, 64);
      if (lane >= o) s += u;
    }
    if (lane == 63) warp_tot[wv] = s;
    __syncthreads();
    int64_t off = carry;
    for (int w = 0; w < wv; ++w) off += warp_tot[w];
    int64_t r = off + s - v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (i0 + q < n) rank[i0 + q] = (int32_t)r;
      r += f[q];
    }
    __syncthreads();
    if (t == kScanThreads - 1) carry = off + s;
    __syncthreads();
  }
  if (t == 0) {
    const int64_t total = carry;
    const int64_t start = *cursor;
    int64_t room = capacity - start;
    room = room < 0 ? 0 : room;
    const int64_t take = total < room ? total : room;
    counts[0] = total;
    counts[1] = take;
    counts[2] += total;  // running sums since the caller last zeroed them: the rollout loop
    counts[3] += take;   // reads these once per evaluate() instead of {n_valid, taken} per step
    ws[0] = start;
    *cursor = start + take;
  }
}

__global__ __launch_bounds__(256) void k_copy_rows(RowFields fs, const uint8_t *__restrict__ mask, int64_t n,
                                                   const int64_t *__restrict__ counts,
                                                   const int64_t *__restrict__ ws) {
  const int64_t row = blockIdx.x;
  if (row >= n || (mask && !mask[row])) return;
  const int32_t *rank = reinterpret_cast<const int32_t *>(ws + 1);
  const int64_t r = rank[row];
  if (r >= counts[1]) return;
  const int64_t dst_row = ws[0] + r;
  for (int k = 0; k < fs.n; ++k) {
    const phc_row_field &f = fs.f[k];
    const int64_t e = f.row_elems;
    if (f.kind == PHC_ROW_COPY32) {
      const uint32_t *s = static_cast<const uint32_t *>(f.src) + row * e;
      uint32_t *d = static_cast<uint32_t *>(f.dst) + dst_row * e;
      if (e % 2 == 0 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 7) == 0) {
        // 8-B granules (the 934-float obs rows start 8-B aligned): half the instructions
        const uint2 *s2 = reinterpret_cast<const uint2 *>(s);
        uint2 *d2 = reinterpret_cast<uint2 *>(d);
        for (int64_t j = threadIdx.x; j < e / 2; j += 256) d2[j] = s2[j];
      } else {
        for (int64_t j = threadIdx.x; j < e; j += 256) d[j] = s[j];
      }
    } else if (f.kind == PHC_ROW_COPY64) {
      const uint64_t *s = static_cast<const uint64_t *>(f.src) + row * e;
      uint64_t *d = static_cast<uint64_t *>(f.dst) + dst_row * e;
      for (int64_t j = threadIdx.x; j < e; j += 256) d[j] = s[j];
    } else {  // PHC_ROW_U8_TO_F32: bool flags stored as float (structs.py:124-125)
      const uint8_t *s = static_cast<const uint8_t *>(f.src) + row * e;
      float *d = static_cast<float *>(f.dst) + dst_row * e;
      for (int64_t j = threadIdx.x; j < e; j += 256) d[j] = s[j] ? 1.0f : 0.0f;
    }
  }
}

// The row's fields as one flat run of 4-byte words (each field's words = its 4-byte elements, two per
// 8-byte element, one per flag byte): thread t moves words t + 256 u.  Every load of the row — the
// control words (mask flag, rank, take, start) and IT data words per thread — is issued in one
// memory round at clamped addresses before the first store: a per-field copy loop put one
// load -> store round trip per field (and per 256-word chunk) on the block's critical path.
// Flag bytes are read through their aligned word, only for fields whose caller vouches that those
// words lie inside the allocation (PHC_ROW_SRC_WORDS); other flag fields take k_copy_rows.
typedef const __attribute__((address_space(1))) uint8_t cu8;
typedef const __attribute__((address_space(1))) uint32_t cu32;
__device__ const uint32_t kOneWord = 1u;  // stands in for a null mask (every row valid)

struct FlatFields {
  const char *src[PHC_MAX_ROW_FIELDS];
  char *dst[PHC_MAX_ROW_FIELDS];
  int64_t srb[PHC_MAX_ROW_FIELDS], drb[PHC_MAX_ROW_FIELDS];  // source / destination bytes per row
  int32_t woff[PHC_MAX_ROW_FIELDS + 1];                      // first flat word of each field; woff[n] = W
  uint32_t u8_mask;                                          // bit k: field k is flag bytes -> float
  int32_t n;
};

// RPB rows per workgroup (PHC_COPY_RPB): every row's loads are issued before the first store, so a
// workgroup's rows share one memory round (one row per workgroup left 4,096 single-round workgroups
// queued two deep per CU)
#ifndef PHC_COPY_RPB
#define PHC_COPY_RPB 4
#endif
template <int IT, int RPB>
__global__ __launch_bounds__(256) void k_copy_rows_flat(FlatFields fs, const uint8_t *__restrict__ mask, int64_t n,
                                                        const int64_t *__restrict__ counts,
                                                        const int64_t *__restrict__ ws) {
  const int64_t row0 = (int64_t)blockIdx.x * RPB;  // grid = ceil(n / RPB)
  const int t = threadIdx.x;
  const int W = fs.woff[fs.n];
  uint32_t mk[RPB];
  int64_t rk[RPB];
#pragma unroll
  for (int j = 0; j < RPB; ++j) {
    const int64_t row = row0 + j < n ? row0 + j : n - 1;  // clamped: the tail rows are skipped below
    mk[j] = *(mask ? (cu8 *)(mask + row) : (cu8 *)&kOneWord);  // pointer select: one load
    rk[j] = reinterpret_cast<const int32_t *>(ws + 1)[row];
  }
  const int64_t take = counts[1], start = ws[0];
  uint32_t v[RPB][IT];
  int k_of[IT], w_of[IT], b_of[IT];  // field, word in the field, byte offset in the source row
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    int vw = t + 256 * u;
    vw = vw < W ? vw : W - 1;
    int k = 0;
#pragma unroll
    for (int q = 1; q < PHC_MAX_ROW_FIELDS; ++q) k = (q < fs.n && vw >= fs.woff[q]) ? q : k;
    const int w = vw - fs.woff[k];
    k_of[u] = k;
    w_of[u] = w;
    b_of[u] = ((fs.u8_mask >> k) & 1u) ? w : 4 * w;
  }
#pragma unroll
  for (int j = 0; j < RPB; ++j) {
    const int64_t row = row0 + j < n ? row0 + j : n - 1;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const char *a = fs.src[k_of[u]] + row * fs.srb[k_of[u]] + b_of[u];
      v[j][u] = *(cu32 *)((uintptr_t)a & ~(uintptr_t)3);
    }
  }
#pragma unroll
  for (int j = 0; j < RPB; ++j) {
    const int64_t row = row0 + j;
    if (row >= n || !mk[j] || rk[j] >= take) continue;
    const int64_t dst_row = start + rk[j];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      if (t + 256 * u >= W) break;
      const int k = k_of[u];
      uint32_t x = v[j][u];
      if ((fs.u8_mask >> k) & 1u) {
        const uintptr_t src = (uintptr_t)(fs.src[k] + row * fs.srb[k] + b_of[u]);
        x = ((x >> (8 * (src & 3))) & 0xFFu) ? 0x3F800000u : 0u;
      }
      *reinterpret_cast<uint32_t *>(fs.dst[k] + dst_row * fs.drb[k] + 4 * w_of[u]) = x;
    }
  }
}

}  // namespace phc

using namespace phc;

extern "C" size_t phc_compact_workspace_bytes(int64_t n) {
  return n <= 0 ? 16 : (size_t)(8 + 4 * n + 15) / 16 * 16;
}

extern "C" int phc_compact_rows(const phc_row_field *fields, int32_t num_fields, const uint8_t *mask, int64_t n,
                                int64_t *cursor, int64_t capacity, int64_t *counts, void *workspace, void *stream) {
  PHC_REQUIRE(fields && num_fields >= 1 && num_fields <= PHC_MAX_ROW_FIELDS, "compact_rows: 1..%d fields",
              PHC_MAX_ROW_FIELDS);
  PHC_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "compact_rows: bad n");
  PHC_REQUIRE(cursor && counts && workspace, "compact_rows: null cursor/counts/workspace");
  PHC_REQUIRE(capacity >= 0, "compact_rows: bad capacity");
  RowFields fs;
  fs.n = num_fields;
  for (int k = 0; k < num_fields; ++k) {
    const phc_row_field &f = fields[k];
    PHC_REQUIRE(f.src && f.dst && f.row_elems > 0, "compact_rows: field %d null or empty", k);
    PHC_REQUIRE(f.kind == PHC_ROW_COPY32 || f.kind == PHC_ROW_COPY64 || f.kind == PHC_ROW_U8_TO_F32,
                "compact_rows: field %d bad kind", k);
    fs.f[k] = f;
  }
  hipStream_t st = as_stream(stream);
  int64_t *ws = static_cast<int64_t *>(workspace);
  hipLaunchKernelGGL(k_rank_mask, dim3(1), dim3(kScanThreads), 0, st, mask, n, cursor, capacity, counts, ws);
  if (n == 0) return check_launch("compact_rows");
  // the flat form when the row's words fit 8 per thread (the rollout's 934-float obs row + the
  // scalar fields: 1,010 words); PHC_COPY_FLAT=0 keeps the per-field loop (A/B)
  FlatFields ff{};
  int64_t words = 0;
  bool flat = PHC_COPY_FLAT != 0;
  for (int k = 0; k < num_fields && flat; ++k) {
    const phc_row_field &f = fields[k];
    const int64_t e = f.row_elems;
    const int64_t w = f.kind == PHC_ROW_COPY64 ? 2 * e : e;
    ff.src[k] = static_cast<const char *>(f.src);
    ff.dst[k] = static_cast<char *>(f.dst);
    ff.srb[k] = f.kind == PHC_ROW_COPY64 ? 8 * e : (f.kind == PHC_ROW_U8_TO_F32 ? e : 4 * e);
    ff.drb[k] = f.kind == PHC_ROW_COPY64 ? 8 * e : 4 * e;
    if (f.kind == PHC_ROW_U8_TO_F32) ff.u8_mask |= 1u << k;
    // word loads: 4-byte aligned sources (flag bytes are read through their aligned word)
    if (f.kind != PHC_ROW_U8_TO_F32 && ((reinterpret_cast<uintptr_t>(f.src) | reinterpret_cast<uintptr_t>(f.dst)) & 3))
      flat = false;
    if (f.kind == PHC_ROW_U8_TO_F32 && ((reinterpret_cast<uintptr_t>(f.dst) & 3) || !(f.flags & PHC_ROW_SRC_WORDS)))
      flat = false;
    ff.woff[k] = (int32_t)words;
    words += w;
  }
  flat = flat && words <= 8 * 256;
  if (flat) {
    ff.woff[num_fields] = (int32_t)words;
    ff.n = num_fields;
    constexpr int R = PHC_COPY_RPB, R8 = R > 2 ? 2 : R;  // 8 words per thread: at most 2 rows in flight
    auto grid = [&](int rpb) { return dim3((unsigned)((n + rpb - 1) / rpb)); };
    const dim3 b(256);
    if (words <= 256) hipLaunchKernelGGL((k_copy_rows_flat<1, R>), grid(R), b, 0, st, ff, mask, n, counts, ws);
    else if (words <= 512) hipLaunchKernelGGL((k_copy_rows_flat<2, R>), grid(R), b, 0, st, ff, mask, n, counts, ws);
    else if (words <= 1024) hipLaunchKernelGGL((k_copy_rows_flat<4, R>), grid(R), b, 0, st, ff, mask, n, counts, ws);
    else hipLaunchKernelGGL((k_copy_rows_flat<8, R8>), grid(R8), b, 0, st, ff, mask, n, counts, ws);
  } else {
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)n), dim3(256), 0, st, fs, mask, n, counts, ws);
  }
  return check_launch("compact_rows");
}
