// Shared device helpers for the gfx950 CO-env kernels.
// Wave = 64 lanes (CDNA4); every cross-lane helper here assumes it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/co_env.h"

namespace co {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ int wave_min_int(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return v;
}

// torch.argmax ordering: NaN beats everything, equal values keep the lower index.
__device__ __forceinline__ bool argmax_better(float a, int ia, float b, int ib) {
  const bool na = a != a, nb = b != b;
  if (na || nb) return na && (!nb || ia < ib);
  return a > b || (a == b && ia < ib);
}

__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(idx, off, kWave);
    if (argmax_better(ov, oi, v, idx)) { v = ov; idx = oi; }
  }
}

// argmin with lowest-index tie break (values are never NaN for our callers).
__device__ __forceinline__ void wave_argmin(float& v, int& idx) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(idx, off, kWave);
    if (ov < v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
}

__device__ __forceinline__ void set_status(int32_t* status, int32_t bits) {
  if (status) atomicOr(status, bits);
}

// Euclidean edge exactly as torch evaluates norm(p=2) over a size-2 dim in f32:
// sqrt(dx*dx + dy*dy) with no fused multiply-add (built with -ffp-contract=off).
__device__ __forceinline__ float edge_len(float x0, float y0, float x1, float y1) {
  const float dx = x1 - x0, dy = y1 - y0;
  return sqrtf(dx * dx + dy * dy);
}

// Grid size for grid-stride kernels: enough blocks to fill 256 CUs several times.
inline unsigned grid_for(int64_t work_items, int per_block, int64_t cap = 256 * 16) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? CO_OK : (int)e;
}

}  // namespace co

// internal (not part of the public C ABI): rollout.hip's thread-per-instance reward
int co_internal_tsp_reward_stepmajor(int64_t B, int64_t N, const float* locs,
                                     const int64_t* acts, int64_t st, int check, float* reward,
                                     int32_t* status, void* stream);
