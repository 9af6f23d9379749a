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

// WRAP: negative actions index from the end (python indexing, SLAP);
// otherwise they are out of range (torch.scatter, TSP).
template <bool COUNT, bool WRAP = false, typename Epilogue>
__device__ __forceinline__ void mask_clear_tile(int64_t B, int N, const int64_t* __restrict__ action,
                                                const uint8_t* mask_in, uint8_t* mask_out,
                                                int32_t* status, bool vec, const Epilogue& epi) {
  __shared__ int s_act[kTileRows];
  __shared__ int s_cnt[kTileRows];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows;
  const int rows = (int)((B - row0) < kTileRows ? (B - row0) : kTileRows);
  int64_t a_reg = 0;
  if (tid < rows) {
    a_reg = action[row0 + tid];
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

  const uint8_t* src = mask_in + row0 * N;
  uint8_t* dst = mask_out + row0 * N;
  const int nbytes = rows * N;
  const int nchunks = (nbytes + 15) >> 4;
  for (int c = tid; c < nchunks; c += kTileThreads) {
    const int off = c << 4;
    const bool full = vec && (off + 16 <= nbytes);
    union {
      uint4 v;
      uint8_t b[16];
    } u;
    if (full) {
      u.v = *reinterpret_cast<const uint4*>(src + off);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) u.b[j] = (off + j < nbytes) ? src[off + j] : 0;
    }
    int r = off / N;
    int col = off - r * N;
    int act = s_act[r];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint8_t v = u.b[j];
      if (col == act) v = 0;
      u.b[j] = v;
      if (COUNT) cnt += (v != 0);
      if (++col == N) {
        if (COUNT && cnt && off + j < nbytes) atomicAdd(&s_cnt[r], cnt);
        cnt = 0;
        col = 0;
        ++r;
        act = (r < rows) ? s_act[r] : -1;
      }
    }
    if (COUNT && cnt && r < rows) atomicAdd(&s_cnt[r], cnt);
    if (full) {
      *reinterpret_cast<uint4*>(dst + off) = u.v;
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (off + j < nbytes) dst[off + j] = u.b[j];
    }
  }
  __syncthreads();
  if (tid < rows) epi(row0 + tid, a_reg, COUNT ? s_cnt[tid] : 0);
}

}  // namespace co
