// Shared device helpers for the gfx950 CO-env kernels.
// Wave = 64 lanes (CDNA4); every cross-lane helper here assumes it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/co_env.h"

namespace co {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
// the wave's index in its block as a wave-uniform (SGPR) value.  `threadIdx.x >> 6` alone is
// a VGPR to the compiler, and everything derived from it (row bases, LDS-DMA counts, m0 and
// global addresses) becomes per-lane VALU work and exec-masked loops.
__device__ __forceinline__ int wave_in_block() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// Streaming accesses (round 6): data a launch reads once or writes once goes through the
// non-temporal path (`nt` loads / stores: gfx950 streams them past the caches' normal
// retention).  Measured: a 2 GiB copy 6.2 -> 6.6 TB/s, the headline launch 23.0 -> 20.7
// us.  NT = false gives the plain access (kernels pass their own switch).
template <bool NT, typename T>
__device__ __forceinline__ T ld_s(const T* p) {
  if constexpr (NT && (sizeof(T) == 4 || sizeof(T) == 8) && !__is_class(T)) {
    return __builtin_nontemporal_load(p);
  } else if constexpr (NT && sizeof(T) == 8) {  // float2 and other 8-byte structs
    const unsigned long long u = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(p));
    T v;
    __builtin_memcpy(&v, &u, 8);
    return v;
  } else if constexpr (NT && sizeof(T) == 16) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    T v;
    __builtin_memcpy(&v, &u, 16);
    return v;
  } else {
    return *p;
  }
}
template <bool NT, typename T>
__device__ __forceinline__ void st_s(T* p, T v) {
  if constexpr (NT && (sizeof(T) == 1 || sizeof(T) == 4 || sizeof(T) == 8) && !__is_class(T)) {
    __builtin_nontemporal_store(v, p);
  } else if constexpr (NT && sizeof(T) == 8) {
    unsigned long long u;
    __builtin_memcpy(&u, &v, 8);
    __builtin_nontemporal_store(u, reinterpret_cast<unsigned long long*>(p));
  } else if constexpr (NT && sizeof(T) == 16) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 u;
    __builtin_memcpy(&u, &v, 16);
    __builtin_nontemporal_store(u, reinterpret_cast<u32x4*>(p));
  } else {
    *p = v;
  }
}

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

// ---------------------------------------------------------------------------
// Lane-group reductions for RL-lane groups (RL = 2 ... 64, 64/RL groups per wave),
// without LDS traffic: DPP quad_perm (xor 1, xor 2), row_half_mirror and row_mirror
// inside each 16-lane row, then gfx950's v_permlane16_swap / v_permlane32_swap across
// rows.  The mirrors are not xor partners but pair every lane with one in the other
// half, which is all a commutative reduction needs.  Every lane of the wave must be
// active (callers keep wave-uniform loop counts).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

// Reduce (value, aux) pairs with `take(ov, oa, v, a)` = "the other pair wins".
template <int RL, class Take>
__device__ __forceinline__ void grp_reduce2(uint32_t& v, uint32_t& a, Take take) {
  uint32_t ov, oa;
#define CO_DPP_STAGE(C)                      \
  ov = dpp_u<C>(v);                          \
  oa = dpp_u<C>(a);                          \
  if (take(ov, oa, v, a)) { v = ov; a = oa; }
  if (RL >= 2) { CO_DPP_STAGE(0xB1); }   // quad_perm [1,0,3,2]
  if (RL >= 4) { CO_DPP_STAGE(0x4E); }   // quad_perm [2,3,0,1]
  if (RL >= 8) { CO_DPP_STAGE(0x141); }  // row_half_mirror
  if (RL >= 16) { CO_DPP_STAGE(0x140); } // row_mirror
#undef CO_DPP_STAGE
  if (RL >= 32) {
    const auto rv = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const auto ra = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    v = rv[0]; a = ra[0];
    if (take(rv[1], ra[1], v, a)) { v = rv[1]; a = ra[1]; }
  }
  if (RL >= 64) {
    const auto rv = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    const auto ra = __builtin_amdgcn_permlane32_swap(a, a, false, false);
    v = rv[0]; a = ra[0];
    if (take(rv[1], ra[1], v, a)) { v = rv[1]; a = ra[1]; }
  }
}

template <int RL, class Op>
__device__ __forceinline__ uint32_t grp_reduce(uint32_t v, Op op) {
  if (RL >= 2) v = op(v, dpp_u<0xB1>(v));
  if (RL >= 4) v = op(v, dpp_u<0x4E>(v));
  if (RL >= 8) v = op(v, dpp_u<0x141>(v));
  if (RL >= 16) v = op(v, dpp_u<0x140>(v));
  if (RL >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = op(r[0], r[1]);
  }
  if (RL >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = op(r[0], r[1]);
  }
  return v;
}

// f64 sum over the group (each stage moves the two halves): exact enough that the f32
// rounding of a sum of f32 terms does not depend on the terms' order
template <int RL>
__device__ __forceinline__ double grp_sum_f64(double v) {
  uint32_t lo = (uint32_t)__double_as_longlong(v), hi = (uint32_t)(__double_as_longlong(v) >> 32);
  auto join = [](uint32_t l, uint32_t h) {
    return __longlong_as_double((long long)(((uint64_t)h << 32) | l));
  };
#define CO_DPP_F64(C)                                   \
  {                                                     \
    v = v + join(dpp_u<C>(lo), dpp_u<C>(hi));           \
    lo = (uint32_t)__double_as_longlong(v);             \
    hi = (uint32_t)(__double_as_longlong(v) >> 32);     \
  }
  if (RL >= 2) CO_DPP_F64(0xB1);
  if (RL >= 4) CO_DPP_F64(0x4E);
  if (RL >= 8) CO_DPP_F64(0x141);
  if (RL >= 16) CO_DPP_F64(0x140);
#undef CO_DPP_F64
  if (RL >= 32) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = join(rl[0], rh[0]) + join(rl[1], rh[1]);
    lo = (uint32_t)__double_as_longlong(v);
    hi = (uint32_t)(__double_as_longlong(v) >> 32);
  }
  if (RL >= 64) {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = join(rl[0], rh[0]) + join(rl[1], rh[1]);
  }
  return v;
}

template <int RL>
__device__ __forceinline__ float grp_max(float v) {
  return __uint_as_float(grp_reduce<RL>(__float_as_uint(v), [](uint32_t x, uint32_t y) {
    return __float_as_uint(fmaxf(__uint_as_float(x), __uint_as_float(y)));
  }));
}
// max over the group on order-preserving ints (one DPP max per stage; the float max needs
// a canonicalising move per stage).  A NaN member may win (the callers' sums go NaN anyway)
template <int RL>
__device__ __forceinline__ float grp_max_ord(float v) {
  const int b = __float_as_int(v);
  int o = b ^ ((b >> 31) & 0x7fffffff);
  o = (int)grp_reduce<RL>((uint32_t)o, [](uint32_t x, uint32_t y) {
    return (uint32_t)max((int)x, (int)y);
  });
  return __int_as_float(o ^ ((o >> 31) & 0x7fffffff));
}
template <int RL>
__device__ __forceinline__ float grp_sum(float v) {
  return __uint_as_float(grp_reduce<RL>(__float_as_uint(v), [](uint32_t x, uint32_t y) {
    return __float_as_uint(__uint_as_float(x) + __uint_as_float(y));
  }));
}
template <int RL>
__device__ __forceinline__ void grp_argmax(float& v, int& idx) {
  uint32_t uv = __float_as_uint(v), ui = (uint32_t)idx;
  grp_reduce2<RL>(uv, ui, [](uint32_t ov, uint32_t oi, uint32_t cv, uint32_t ci) {
    return argmax_better(__uint_as_float(ov), (int)oi, __uint_as_float(cv), (int)ci);
  });
  v = __uint_as_float(uv);
  idx = (int)ui;
}
template <int RL>
__device__ __forceinline__ int grp_min_int(int v) {
  return (int)grp_reduce<RL>((uint32_t)v, [](uint32_t x, uint32_t y) {
    return (uint32_t)min((int)x, (int)y);
  });
}
template <int RL>
__device__ __forceinline__ int grp_max_int(int v) {
  return (int)grp_reduce<RL>((uint32_t)v, [](uint32_t x, uint32_t y) {
    return (uint32_t)max((int)x, (int)y);
  });
}

template <int RL>
__device__ __forceinline__ void grp_argmin(float& v, int& idx) {
  uint32_t uv = __float_as_uint(v), ui = (uint32_t)idx;
  grp_reduce2<RL>(uv, ui, [](uint32_t ov, uint32_t oi, uint32_t cv, uint32_t ci) {
    const float a = __uint_as_float(ov), b = __uint_as_float(cv);
    return a < b || (a == b && (int)oi < (int)ci);
  });
  v = __uint_as_float(uv);
  idx = (int)ui;
}

// Exact group argmin for NaN-free values in two cheap passes: a float group min (one DPP
// move + v_min per stage), then the group min of the indices of the lanes that hold it
// (ties -> lowest index, as torch.argmin).  About half the VALU of a (value, index)
// pair reduction.  A lane without a candidate passes (+inf, 0x7fffffff).
template <int RL>
__device__ __forceinline__ void grp_argmin_split(float& v, int& idx) {
  const float m = __uint_as_float(grp_reduce<RL>(__float_as_uint(v), [](uint32_t a, uint32_t b) {
    return __float_as_uint(fminf(__uint_as_float(a), __uint_as_float(b)));
  }));
  const int cand = v == m ? idx : 0x7fffffff;
  idx = (int)grp_reduce<RL>((uint32_t)cand, [](uint32_t a, uint32_t b) {
    return (uint32_t)min((int)a, (int)b);
  });
  v = m;
}

typedef __attribute__((address_space(3))) void lds_void;

// Copy `nbytes` contiguous bytes global -> LDS with LDS-DMA (global_load_lds_dwordx4):
// every wave-instruction moves 1 KiB to a wave-uniform LDS base + lane*16, no VGPR
// round trip, all pieces in flight before the single wait.  `src` and `dst` must be
// 16-byte aligned; a tail of < 16 bytes is copied with plain loads.  Ends with the
// vmcnt drain + workgroup barrier that make the tile visible.
#ifndef CO_STAGE_AUX
#define CO_STAGE_AUX 0  // cache-policy bits of stage_bytes_lds's LDS-DMA (2 = nt)
#endif
template <int AUX = CO_STAGE_AUX>
__device__ __forceinline__ void stage_bytes_lds(const unsigned char* __restrict__ src, int nbytes,
                                                unsigned char* dst) {
  const int lane = threadIdx.x & 63, wave = wave_in_block(), nw = blockDim.x >> 6;
  const int n16 = nbytes & ~15;
  for (int base = wave * 1024; base < n16; base += nw * 1024) {
    const int off = base + lane * 16;
    if (off < n16)
      __builtin_amdgcn_global_load_lds((const void*)(src + off), (lds_void*)(dst + base), 16, 0,
                                       AUX);
  }
  for (int k = n16 + (int)threadIdx.x; k < nbytes; k += blockDim.x) dst[k] = src[k];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}

// The wave copies `nbytes` (16-byte aligned source and destination) global -> LDS with
// LDS-DMA, 1 KiB per instruction; the caller waits (vmcnt) before reading.
template <int AUX = 0>  // the loads' cache-policy bits (sc0 / nt / sc1)
__device__ __forceinline__ void wave_dma(const unsigned char* __restrict__ src, int nbytes,
                                         unsigned char* dst) {
  const int lane = lane_id(), n16 = nbytes & ~15;
  for (int base = 0; base < n16; base += 1024) {
    if (base + lane * 16 < n16)
      __builtin_amdgcn_global_load_lds((const void*)(src + base + lane * 16),
                                       (lds_void*)(dst + base), 16, 0, AUX);
  }
  if (lane < ((nbytes - n16) >> 2))  // a tail of whole dwords (< 16 B): plain loads
    reinterpret_cast<uint32_t*>(dst + n16)[lane] = reinterpret_cast<const uint32_t*>(src + n16)[lane];
}

// After wave_dma: drain the wave's loads and make its LDS writes (DMA and the tail's plain
// stores) visible to all of its lanes; no workgroup barrier.
__device__ __forceinline__ void wave_dma_wait() {
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Zero a device int32 (flags / counters).  A kernel, not hipMemsetAsync: memset nodes
// captured into HIP graphs were observed on MI355X to replay with a wrong fill byte
// (0x10101010 after a 4-byte memset to 0), which corrupted counters in replays.
namespace {  // one copy per translation unit
__global__ void zero_i32_kernel(int32_t* p) { *p = 0; }
}  // namespace
inline int zero_i32(int32_t* p, hipStream_t s) {
  hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(1), 0, s, p);
  return (int)hipGetLastError();
}

// Grid size for grid-stride kernels: enough blocks to fill 256 CUs several times.
inline unsigned grid_for(int64_t work_items, int per_block, int64_t cap = 256 * 16) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// A grid that covers the work exactly (kernels without a grid-stride loop: every row group
// gets its wave), or 0 when it would exceed HIP's limit of 2^32 - 1 threads per grid
// dimension -- the entry point then returns CO_E_INVAL instead of launching a grid that
// skips rows.
constexpr int64_t kMaxCoverThreads = ((int64_t)1 << 32) - 1;
inline unsigned cover_grid(int64_t work_items, int per_block, int block_threads = 256) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g * (int64_t)block_threads > kMaxCoverThreads) return 0;
  return (unsigned)g;
}

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? CO_OK : (int)e;
}

}  // namespace co

// internal (not part of the public C ABI): rollout.hip's thread-per-instance reward
int co_internal_tsp_reward_stepmajor(int64_t B, int64_t N, const float* locs,
                                     int64_t locs_batch, const int64_t* acts, int64_t st,
                                     int check, float* reward, int32_t* status, void* stream);
// internal: rollout.hip's lane-group reward for row-major actions (T == N <= 1024)
int co_internal_tsp_reward_rows(int64_t B, int64_t N, const float* locs, int64_t locs_batch,
                                const int64_t* acts, int64_t sb, int check, float* reward,
                                int32_t* status, void* stream);
// internal: nearest.hip's register-resident nearest-policy TSP episode
int co_internal_tsp_nearest_rollout(int64_t B, int64_t N, const float* locs, int64_t* acts_out,
                                    uint8_t* mask_out, int64_t* first_out, int64_t* cur_out,
                                    int64_t* i_out, uint8_t* done_out, uint8_t* step_reward_out,
                                    float* reward_out, void* stream);
