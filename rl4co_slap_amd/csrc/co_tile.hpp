// Tile engine shared by the TSP and SLAP step kernels: one 256-thread workgroup
// owns kTileRows consecutive instances; their [rows, N] byte mask is streamed
// through registers in 16-byte chunks (coalesced dwordx4), the byte at
// (row, action[row]) is cleared, and optionally the surviving bytes of each row
// are counted into LDS.  kTileRows * N is a multiple of 16 for every N, so each
// tile starts 16-byte aligned whenever the base pointers are.
#pragma once

#include "co_common.hpp"

namespace co {

constexpr int kTileRows = 64;
constexpr int kTileThreads = 256;

inline int tile_vec_ok(const void* a, const void* b) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
}

// One 16-byte chunk of the tile: clear the byte at (row, action[row]) and count the
// surviving bytes per row (LDS atomics, at most ~2 rows per chunk for N >= 16).
template <bool COUNT>
__device__ __forceinline__ void tile_chunk(uint4& v, int off, int nbytes, int N, int rows,
                                           const int* s_act, int* s_cnt) {
  union {
    uint4 v;
    uint8_t b[16];
  } u;
  u.v = v;
  int r = off / N;
  int col = off - r * N;
  int act = s_act[r];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint8_t x = u.b[j];
    if (col == act) x = 0;
    u.b[j] = x;
    if (COUNT) cnt += (x != 0);
    if (++col == N) {
      if (COUNT && cnt && off + j < nbytes) atomicAdd(&s_cnt[r], cnt);
      cnt = 0;
      col = 0;
      ++r;
      act = (r < rows) ? s_act[r] : -1;
    }
  }
  if (COUNT && cnt && r < rows) atomicAdd(&s_cnt[r], cnt);
  v = u.v;
}

__device__ __forceinline__ uint4 tile_load(const uint8_t* src, int off, int nbytes, bool vec) {
  if (vec && off + 16 <= nbytes) return *reinterpret_cast<const uint4*>(src + off);
  union {
    uint4 v;
    uint8_t b[16];
  } u;
#pragma unroll
  for (int j = 0; j < 16; ++j) u.b[j] = (off + j < nbytes) ? src[off + j] : 0;
  return u.v;
}

__device__ __forceinline__ void tile_store(uint8_t* dst, int off, int nbytes, bool vec, uint4 v) {
  if (vec && off + 16 <= nbytes) {
    *reinterpret_cast<uint4*>(dst + off) = v;
    return;
  }
  union {
    uint4 v;
    uint8_t b[16];
  } u;
  u.v = v;
  for (int j = 0; j < 16; ++j)
    if (off + j < nbytes) dst[off + j] = u.b[j];
}

// WRAP: negative actions index from the end (python indexing, SLAP); otherwise they
// are out of range (torch.scatter, TSP).  Every global load of the tile (the action,
// the epilogue's row scalars and the first PF mask chunks) is issued before the
// single barrier, so a workgroup pays one memory latency, not three.
// Epilogue: `typename E::Row row = epi.load(b)` early, `epi.store(b, action, count, row)`.
template <bool COUNT, bool WRAP = false, typename Epilogue>
__device__ __forceinline__ void mask_clear_tile(int64_t B, int N, const int64_t* __restrict__ action,
                                                const uint8_t* mask_in, uint8_t* mask_out,
                                                int32_t* status, bool vec, const Epilogue& epi) {
  constexpr int PF = 2;
  __shared__ int s_act[kTileRows];
  __shared__ int s_cnt[kTileRows];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows;
  const int rows = (int)((B - row0) < kTileRows ? (B - row0) : kTileRows);
  const uint8_t* src = mask_in + row0 * N;
  uint8_t* dst = mask_out + row0 * N;
  const int nbytes = rows * N;
  const int nchunks = (nbytes + 15) >> 4;

  int64_t a_reg = 0;
  typename Epilogue::Row rowv{};
  if (tid < rows) {
    a_reg = action[row0 + tid];
    rowv = epi.load(row0 + tid);
  }
  uint4 pf[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int c = tid + k * kTileThreads;
    if (c < nchunks) pf[k] = tile_load(src, c << 4, nbytes, vec);
  }
  if (tid < rows) {
    int64_t a = a_reg;
    if (WRAP && a < 0) a += N;
    if (a < 0 || a >= N) {
      set_status(status, CO_ST_INDEX_RANGE);
      a = -1;
    }
    s_act[tid] = (int)a;
    s_cnt[tid] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int c = tid + k * kTileThreads;
    if (c < nchunks) {
      tile_chunk<COUNT>(pf[k], c << 4, nbytes, N, rows, s_act, s_cnt);
      tile_store(dst, c << 4, nbytes, vec, pf[k]);
    }
  }
  for (int c = tid + PF * kTileThreads; c < nchunks; c += kTileThreads) {
    uint4 v = tile_load(src, c << 4, nbytes, vec);
    tile_chunk<COUNT>(v, c << 4, nbytes, N, rows, s_act, s_cnt);
    tile_store(dst, c << 4, nbytes, vec, v);
  }
  if (COUNT) __syncthreads();
  if (tid < rows) epi.store(row0 + tid, a_reg, COUNT ? s_cnt[tid] : 0, rowv);
}

}  // namespace co
