// utils.ops kernels for gfx950: gather_by_index (rl4co/utils/ops.py:65-77),
// the batch-wide "any i == 0" test of tsp/env.py:70, the not-done counter used
// by the rollout engine's done poll, and the build-info string.
#include "co_common.hpp"

using namespace co;

namespace {

// One thread per VW-byte unit of the output; the index of a unit's row is read
// once per unit (L1/L2 hit for the 2nd..k-th unit of the same row).
template <typename V>
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* src, int64_t outer,
                                                     int64_t src_len, int64_t units_per_elem,
                                                     int64_t s_outer, int64_t s_len,
                                                     const int64_t* idx, int64_t idx_len,
                                                     int64_t i_outer, int64_t i_len, V* dst,
                                                     int32_t* status) {
  const int64_t total = outer * idx_len * units_per_elem;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += stride) {
    const int64_t e = u / units_per_elem;
    const int64_t k = u - e * units_per_elem;
    const int64_t o = e / idx_len;
    const int64_t m = e - o * idx_len;
    const int64_t j = idx[o * i_outer + m * i_len];
    V v{};
    if (j < 0 || j >= src_len) {
      bad = true;
    } else {
      v = reinterpret_cast<const V*>(src + o * s_outer + j * s_len)[k];
    }
    dst[u] = v;
  }
  if (__any(bad) && lane_id() == 0) set_status(status, CO_ST_INDEX_RANGE);
}

// One 1024-thread workgroup reduces the whole vector and writes the result itself: no
// zeroing launch and no atomics (these feed per-step host polls inside graphs, where a
// launch costs ~4-5 us of its own).  16-byte loads when the base is aligned.
constexpr int kReduceThreads = 1024;

__device__ __forceinline__ int block_sum_int(int v) {
  __shared__ int s_part[kReduceThreads / 64];
  v = wave_sum(v);
  if (lane_id() == 0) s_part[threadIdx.x >> 6] = v;
  __syncthreads();
  int t = 0;
  if (threadIdx.x < 64) {
    t = threadIdx.x < kReduceThreads / 64 ? s_part[threadIdx.x] : 0;
    t = wave_sum(t);
  }
  return t;  // valid in wave 0
}

__global__ __launch_bounds__(kReduceThreads) void any_eq_kernel(const int64_t* x, int64_t n,
                                                                int64_t value, int32_t* flag) {
  int hit = 0;
  for (int64_t k = threadIdx.x; k < n; k += kReduceThreads) hit |= x[k] == value;
  hit = block_sum_int(hit);
  if (threadIdx.x == 0) *flag = hit != 0;
}

__global__ __launch_bounds__(kReduceThreads) void count_not_done_kernel(const uint8_t* done,
                                                                        int64_t n, int32_t* count) {
  int c = 0;
  const bool vec = (reinterpret_cast<uintptr_t>(done) & 15) == 0;
  const int64_t n16 = vec ? (n & ~(int64_t)15) : 0;
  for (int64_t k = (int64_t)threadIdx.x * 16; k < n16; k += (int64_t)kReduceThreads * 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(done + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) c += ((w[q] >> (8 * j)) & 0xffu) == 0u;
  }
  for (int64_t k = n16 + threadIdx.x; k < n; k += kReduceThreads) c += done[k] == 0;
  c = block_sum_int(c);
  if (threadIdx.x == 0) *count = c;
}

// One wave per instance: lanes over the S starts (strided by `instances`).
__global__ __launch_bounds__(256) void pomo_baseline_kernel(int64_t B, int S, const float* reward,
                                                            const float* ll, float* bl,
                                                            float* maxr, int64_t* best,
                                                            float* adv, float* lterm) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    float sum = 0.f, mv = -__builtin_inff();
    int mi = 0x7fffffff;
    for (int s = lane; s < S; s += 64) {
      const float r = reward[(int64_t)s * B + b];
      sum += r;
      if (argmax_better(r, s, mv, mi)) { mv = r; mi = s; }
    }
    sum = wave_sum(sum);
    wave_argmax(mv, mi);
    const float mean = sum / (float)S;
    float lt = 0.f;
    for (int s = lane; s < S; s += 64) {
      const int64_t e = (int64_t)s * B + b;
      const float a = reward[e] - mean;
      if (adv) adv[e] = a;
      if (ll) lt += a * ll[e];
    }
    lt = wave_sum(lt);
    if (lane == 0) {
      bl[b] = mean;
      if (maxr) maxr[b] = mv;
      if (best) best[b] = mi;
      if (lterm) lterm[b] = lt;
    }
  }
}

// The decode loop's epilogue on step-major rows: a 256-thread workgroup owns 64 instances
// (columns b0 .. b0+63 of the step rows) and walks the steps in chunks of kStackChunk:
// the chunk's action / log-probability rows are loaded coalesced (a wave reads one step's
// 64 values; the next chunk's loads in flight during this chunk's stores) into LDS, then
// written out transposed -- consecutive threads on consecutive
// steps of an instance's [B, T] row -- while thread b sums its row's
// log-probabilities in step order in f64 (ll) and tests `> -1000` (decoding.py:57-58).
constexpr int kStackChunk = 32;

__global__ __launch_bounds__(256) void episode_stack_kernel(
    int64_t B, int64_t T, const int64_t* __restrict__ act_sm, int64_t act_rs,
    const float* __restrict__ logp_sm, int64_t logp_rs, int64_t* __restrict__ actions,
    float* __restrict__ logprobs, float* __restrict__ ll, int32_t* status) {
  __shared__ int64_t s_act[kStackChunk][65];  // +1: the stores read down a column too
  __shared__ float s_lp[kStackChunk][65];  // +1: the row-wise sum reads down a column
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t b0 = (int64_t)blockIdx.x * 64;
  const int nb = (int)(B - b0 < 64 ? B - b0 : 64);
  double acc = 0.0;
  bool bad = false;
  // wave w loads steps w, w + 4, ... of a chunk into registers (one coalesced row piece
  // each; indices clamped into the rows, so every load is unconditional); the next chunk's
  // loads are issued before this chunk's stores, so they are in flight while it stores
  constexpr int KW = kStackChunk / 4;
  int64_t ra[KW];
  float rl[KW];
  const int64_t bb = b0 + (lane < nb ? lane : nb - 1);
  auto fetch = [&](int64_t t0) {
#pragma unroll
    for (int i = 0; i < KW; ++i) {
      const int64_t tt = t0 + w + 4 * i < T ? t0 + w + 4 * i : T - 1;
      if (act_sm) ra[i] = act_sm[tt * act_rs + bb];
      if (logp_sm) rl[i] = logp_sm[tt * logp_rs + bb];
    }
  };
  fetch(0);
  for (int64_t t0 = 0; t0 < T; t0 += kStackChunk) {
    const int nt = (int)(T - t0 < kStackChunk ? T - t0 : kStackChunk);
#pragma unroll
    for (int i = 0; i < KW; ++i) {
      const int k = w + 4 * i;
      if (k < nt && lane < nb) {
        if (act_sm) s_act[k][lane] = ra[i];
        if (logp_sm) s_lp[k][lane] = rl[i];
      }
    }
    __syncthreads();
    if (t0 + kStackChunk < T) fetch(t0 + kStackChunk);
    // transposed stores: element i of the chunk's 64 x nt output block is row i / nt, step
    // i % nt, so consecutive threads write consecutive addresses of a row (r05: 4 threads
    // x 8 values per row left every store instruction 64 separate 8-byte pieces)
    for (int i = tid; i < nb * nt; i += 256) {
      const int r = i / nt, j = i - r * nt;
      const int64_t o = (b0 + r) * T + t0 + j;
      if (actions) actions[o] = s_act[j][r];
      if (logprobs) logprobs[o] = s_lp[j][r];
    }
    if (logp_sm && tid < nb) {  // thread b: its row, in step order
      if (nt == kStackChunk) {
        float v[kStackChunk];
#pragma unroll
        for (int j = 0; j < kStackChunk; ++j) v[j] = s_lp[j][tid];  // reads ahead of the chain
#pragma unroll
        for (int j = 0; j < kStackChunk; ++j) {
          acc += (double)v[j];
          bad |= !(v[j] > -1000.f);
        }
      } else {
        for (int j = 0; j < nt; ++j) {
          const float v = s_lp[j][tid];
          acc += (double)v;
          bad |= !(v > -1000.f);
        }
      }
    }
    __syncthreads();  // the next chunk overwrites the tile
  }
  if (logp_sm && tid < nb && ll) ll[b0 + tid] = (float)acc;
  if (__any(bad) && lane == 0) set_status(status, CO_ST_LOGP_NEG_INF);
}

}  // namespace

extern "C" int co_episode_stack(int64_t B, int64_t T, const int64_t* act_sm, int64_t act_rs,
                                const float* logp_sm, int64_t logp_rs, int64_t* actions,
                                float* logprobs, float* ll, int32_t* status, void* stream) {
  if (B < 0 || T < 0 || (act_sm && act_rs < B) || (logp_sm && logp_rs < B)) return CO_E_INVAL;
  if (B == 0 || T == 0) return CO_OK;
  if ((act_sm && !actions) || (logp_sm && (!logprobs || !status)) || (ll && !logp_sm))
    return CO_E_INVAL;
  const unsigned grid = cover_grid(B, 64);
  if (grid == 0) return CO_E_INVAL;
  hipLaunchKernelGGL(episode_stack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, T,
                     act_sm, act_rs, logp_sm, logp_rs, actions, logprobs, ll, status);
  return launch_status();
}

extern "C" int co_pomo_shared_baseline(int64_t B, int64_t S, const float* reward, const float* ll,
                                       float* bl, float* maxr, int64_t* best, float* adv,
                                       float* lterm, void* stream) {
  if (B < 0 || S <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!reward || !bl || (lterm && !ll)) return CO_E_INVAL;
  hipLaunchKernelGGL(pomo_baseline_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)S, reward, ll, bl, maxr, best, adv, lterm);
  return launch_status();
}

extern "C" const char* co_build_info(void) {
  return "rl4co_slap_amd co_env: gfx950 (CDNA4), wave64";
}

extern "C" int co_gather_by_index(const void* src, int64_t outer, int64_t src_len,
                                  int64_t inner_bytes, int64_t s_outer, int64_t s_len,
                                  const int64_t* idx, int64_t idx_len, int64_t i_outer,
                                  int64_t i_len, void* dst, int32_t* status, void* stream) {
  if (outer < 0 || src_len < 0 || idx_len < 0 || inner_bytes <= 0) return CO_E_INVAL;
  if (outer == 0 || idx_len == 0) return CO_OK;
  if (!src || !idx || !dst) return CO_E_INVAL;
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                       (uintptr_t)s_outer | (uintptr_t)s_len | (uintptr_t)inner_bytes;
  const int64_t units = outer * idx_len;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* sp = static_cast<const uint8_t*>(src);
#define CO_GATHER(V, W)                                                                        \
  hipLaunchKernelGGL(gather_kernel<V>, dim3(grid_for(units * (inner_bytes / W), 256)),        \
                     dim3(256), 0, s, sp, outer, src_len, inner_bytes / W, s_outer, s_len, idx, \
                     idx_len, i_outer, i_len, static_cast<V*>(dst), status)
  if ((al & 15) == 0) {
    CO_GATHER(uint4, 16);
  } else if ((al & 7) == 0) {
    CO_GATHER(uint2, 8);
  } else if ((al & 3) == 0) {
    CO_GATHER(uint32_t, 4);
  } else {
    CO_GATHER(uint8_t, 1);
  }
#undef CO_GATHER
  return launch_status();
}

extern "C" int co_any_eq_i64(const int64_t* x, int64_t n, int64_t value, int32_t* flag,
                             void* stream) {
  if (n < 0 || !flag || (n > 0 && !x)) return CO_E_INVAL;
  hipLaunchKernelGGL(any_eq_kernel, dim3(1), dim3(kReduceThreads), 0, (hipStream_t)stream, x, n,
                     value, flag);
  return launch_status();
}

// co_row_deficit_max: out = max(0, max_b(width - sum of row b's bytes)): 16 lanes per row
// (consecutive bytes: coalesced row pieces), 4 rows per wave, a fixed grid of 1,024-thread
// workgroups striding over the rows, one atomicMax per workgroup (same-address atomics
// from every wave serialise: 8,192 of them took 37 us at B = 32,768).  The decode loop's
// done poll for CVRP: a row whose visited bytes sum to width - d cannot be done within
// d - 1 more steps (a step adds at most one to the sum), so the loop skips those polls.
__global__ __launch_bounds__(1024) void row_deficit_kernel(const uint8_t* __restrict__ rows,
                                                           int64_t n_rows, int width,
                                                           int64_t stride, int32_t* out) {
  __shared__ int s_best[16];
  const int lane = lane_id(), sl = lane & 15, w = wave_in_block();
  int best = 0;
  for (int64_t base = ((int64_t)blockIdx.x * 16 + w) * 4; base < n_rows;
       base += (int64_t)gridDim.x * 64) {  // wave-uniform: the group reduction needs all lanes
    const int64_t r = base + (lane >> 4);
    uint32_t sum = 0;
    if (r < n_rows) {
      const uint8_t* row = rows + r * stride;
      for (int c = sl; c < width; c += 16) sum += row[c];
    }
    sum = grp_reduce<16>(sum, [](uint32_t x, uint32_t y) { return x + y; });
    if (r < n_rows) best = max(best, width - (int)sum);
  }
  best = (int)grp_reduce<64>((uint32_t)best, [](uint32_t x, uint32_t y) {
    return (uint32_t)max((int)x, (int)y);
  });
  if (lane == 0) s_best[w] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    int m = 0;
    for (int q = 0; q < 16; ++q) m = max(m, s_best[q]);
    if (m > 0) atomicMax(out, m);
  }
}

extern "C" int co_row_deficit_max(const uint8_t* rows, int64_t n_rows, int64_t width,
                                  int64_t row_stride, int32_t* out, void* stream) {
  if (n_rows < 0 || width <= 0 || width > (1 << 24) || !out || (n_rows > 0 && !rows))
    return CO_E_INVAL;
  int rc = zero_i32(out, (hipStream_t)stream);
  if (rc != 0 || n_rows == 0) return rc == 0 ? CO_OK : rc;
  hipLaunchKernelGGL(row_deficit_kernel, dim3(grid_for(n_rows, 64, 256)), dim3(1024), 0,
                     (hipStream_t)stream, rows, n_rows, (int)width, row_stride, out);
  return launch_status();
}

extern "C" int co_count_not_done(const uint8_t* done, int64_t n, int32_t* count, void* stream) {
  if (n < 0 || !count || (n > 0 && !done)) return CO_E_INVAL;
  hipLaunchKernelGGL(count_not_done_kernel, dim3(1), dim3(kReduceThreads), 0,
                     (hipStream_t)stream, done, n, count);
  return launch_status();
}

// ------------------------------------------------------------------ instance generation
// Device instance generator for throughput runs: the reference's
// Uniform samplers (tsp/generator.py:51-60, cvrp/generator.py:116-143) on a counter-based
// stream instead of torch's CPU Mersenne Twister.  One Philox-4x32-10 block (key = seed,
// counter = (offset + i/4, 0)) gives elements 4*(i/4) .. 4*(i/4)+3; u = (x >> 8) * 2^-24
// is torch's f32 uniform grid, out = low + u * (high - low) as Uniform.sample (two
// roundings, no contraction); demand mode: out = ((int)(low + u * (high - low)) + 1) / cap.
namespace {
__device__ __forceinline__ uint4 philox4(uint64_t seed, uint64_t ctr) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0u, c3 = 0u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

template <bool DEMAND>
__device__ __forceinline__ float uniform_value(uint32_t x, float low, float range, float cap) {
  const float u = (float)(x >> 8) * 0x1p-24f;
  const float v = low + u * range;
  return DEMAND ? (float)((int)v + 1) / cap : v;
}

template <bool DEMAND>
__global__ __launch_bounds__(256) void uniform_fill_kernel(float* __restrict__ out, int64_t n,
                                                           float low, float range, float cap,
                                                           uint64_t seed, uint64_t offset) {
  const int64_t nb = (n + 3) / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 x = philox4(seed, offset + (uint64_t)i);
    const float4 v = make_float4(uniform_value<DEMAND>(x.x, low, range, cap),
                                 uniform_value<DEMAND>(x.y, low, range, cap),
                                 uniform_value<DEMAND>(x.z, low, range, cap),
                                 uniform_value<DEMAND>(x.w, low, range, cap));
    const int64_t e = 4 * i;
    if (e + 4 <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
      *reinterpret_cast<float4*>(out + e) = v;
    } else {
      const float w[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; j < 4 && e + j < n; ++j) out[e + j] = w[j];
    }
  }
}
// integers in [low, low + range): low + (x * range) >> 32 (multiply-shift; the bias is
// below range / 2^32, e.g. 5e-9 for range 20)
__global__ __launch_bounds__(256) void randint_fill_kernel(int64_t* __restrict__ out, int64_t n,
                                                           int64_t low, uint32_t range,
                                                           uint64_t seed, uint64_t offset) {
  const int64_t nb = (n + 3) / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 x = philox4(seed, offset + (uint64_t)i);
    const int64_t w[4] = {low + (int64_t)(((uint64_t)x.x * range) >> 32),
                          low + (int64_t)(((uint64_t)x.y * range) >> 32),
                          low + (int64_t)(((uint64_t)x.z * range) >> 32),
                          low + (int64_t)(((uint64_t)x.w * range) >> 32)};
    const int64_t e = 4 * i;
    if (e + 4 <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
      *reinterpret_cast<longlong2*>(out + e) = make_longlong2(w[0], w[1]);
      *reinterpret_cast<longlong2*>(out + e + 2) = make_longlong2(w[2], w[3]);
    } else {
      for (int j = 0; j < 4 && e + j < n; ++j) out[e + j] = w[j];
    }
  }
}
}  // namespace

extern "C" int co_randint_fill(int64_t* out, int64_t n, int64_t low, int64_t high, uint64_t seed,
                               uint64_t offset, void* stream) {
  if (n < 0 || (n > 0 && !out) || !(high > low) || high - low > (int64_t)0xffffffffLL)
    return CO_E_INVAL;
  if (n == 0) return CO_OK;
  hipLaunchKernelGGL(randint_fill_kernel, dim3(grid_for((n + 3) / 4, 256, 256 * 64)), dim3(256),
                     0, (hipStream_t)stream, out, n, low, (uint32_t)(high - low), seed, offset);
  return launch_status();
}

extern "C" int co_uniform_fill(float* out, int64_t n, float low, float high, float capacity,
                               int demand, uint64_t seed, uint64_t offset, void* stream) {
  if (n < 0 || (n > 0 && !out) || !(high >= low) || (demand && !(capacity > 0.f)))
    return CO_E_INVAL;
  if (n == 0) return CO_OK;
  const unsigned grid = grid_for((n + 3) / 4, 256, 256 * 64);
  if (demand)
    hipLaunchKernelGGL(uniform_fill_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       out, n, low, high - low, capacity, seed, offset);
  else
    hipLaunchKernelGGL(uniform_fill_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       out, n, low, high - low, 1.f, seed, offset);
  return launch_status();
}

// ------------------------------------------------------------------ measurement probe
namespace {
// one 16-B unit per thread over a full grid (the float4-copy shape of the guide's 6.29 TB/s
// measurement; grid-stride variants with 1 or 4 units in flight measured 5.07 / 4.25 TB/s)
#ifndef CO_PROBE_NT
#define CO_PROBE_NT 1  // non-temporal loads and stores (r06: 2 GiB 6.2 -> 6.6 TB/s, the best copy)
#endif
__global__ __launch_bounds__(256) void probe_copy_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) {
    if (CO_PROBE_NT) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(
          __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i),
          reinterpret_cast<u32x4*>(dst) + i);
    } else
      dst[i] = src[i];
  }
}
}  // namespace

extern "C" int co_probe_copy(const void* src, void* dst, int64_t nbytes, void* stream) {
  if (nbytes < 0 || (nbytes & 15) || (nbytes > 0 && (!src || !dst))) return CO_E_INVAL;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) != 0)
    return CO_E_ALIGN;
  if (nbytes == 0) return CO_OK;
  const int64_t blocks = (nbytes / 16 + 255) / 256;
  if (blocks > 0x7fffffff) return CO_E_INVAL;
  hipLaunchKernelGGL(probe_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst),
                     nbytes / 16);
  return launch_status();
}

// ------------------------------------------------------------------ augmentation
// data/transforms.py:15-37 dihedral_8_augmentation: out[r*B*N + i] = transform r of
// in[i] (i = b*N + c), r = 0..7 in the reference's order z0..z7; the [8B, N, 2] output is
// the batchify layout (row r*B + b).  1 - x in f32, exactly as the reference.
namespace {
__global__ __launch_bounds__(256) void dihedral8_kernel(int64_t BN, const float2* __restrict__ in,
                                                        float2* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < BN;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float2 p = in[i];
    const float x = p.x, y = p.y, nx = 1.f - x, ny = 1.f - y;
    out[i] = make_float2(x, y);
    out[BN + i] = make_float2(nx, y);
    out[2 * BN + i] = make_float2(x, ny);
    out[3 * BN + i] = make_float2(nx, ny);
    out[4 * BN + i] = make_float2(y, x);
    out[5 * BN + i] = make_float2(ny, x);
    out[6 * BN + i] = make_float2(y, nx);
    out[7 * BN + i] = make_float2(ny, nx);
  }
}

// data/transforms.py:49-71 symmetric_transform: per row b, rotate (x, y) - offset by
// phi[b], swap the axes when phi[b] > 2*pi (f32 compare), add the offset back.  f32
// separately rounded products as ATen evaluates them (-ffp-contract=off).
__global__ __launch_bounds__(256) void symmetric_kernel(int64_t B, int64_t N,
                                                        const float2* __restrict__ in,
                                                        const float* __restrict__ phi,
                                                        float offset, float2* __restrict__ out) {
  const float two_pi = (float)(2.0 * 3.14159265358979323846);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B * N;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float f = phi[i / N];
    const float c = cosf(f), s = sinf(f);
    const float2 p = in[i];
    const float x = p.x - offset, y = p.y - offset;
    const float xp = c * x - s * y, yp = s * x + c * y;
    const bool flip = f > two_pi;
    out[i] = make_float2((flip ? yp : xp) + offset, (flip ? xp : yp) + offset);
  }
}
}  // namespace

extern "C" int co_dihedral8_augment(int64_t B, int64_t N, const float* xy, float* out,
                                    void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!xy || !out) return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(xy) | reinterpret_cast<uintptr_t>(out)) & 7) return CO_E_ALIGN;
  const int64_t bn = B * N;
  hipLaunchKernelGGL(dihedral8_kernel, dim3(grid_for(bn, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, bn, reinterpret_cast<const float2*>(xy),
                     reinterpret_cast<float2*>(out));
  return launch_status();
}

extern "C" int co_symmetric_augment(int64_t B, int64_t N, const float* xy, const float* phi,
                                    float offset, float* out, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!xy || !phi || !out) return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(xy) | reinterpret_cast<uintptr_t>(out)) & 7) return CO_E_ALIGN;
  hipLaunchKernelGGL(symmetric_kernel, dim3(grid_for(B * N, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, B, N, reinterpret_cast<const float2*>(xy), phi, offset,
                     reinterpret_cast<float2*>(out));
  return launch_status();
}

// utils/ops.py:104-111 get_distance_matrix: out[b, i, j] = |locs[b,i] - locs[b,j]|_2 in
// f32 (sqrt(dx*dx + dy*dy), correctly rounded).  Four j per thread, float4 stores when
// N % 4 == 0; the instance's coordinates come from L2 after the first touch.
namespace {
__global__ __launch_bounds__(256) void distance_matrix_kernel(int64_t B, int N,
                                                              const float2* __restrict__ locs,
                                                              float* __restrict__ out) {
  const int64_t NN = (int64_t)N * N;
  const bool vec = (N & 3) == 0;
  const int64_t units = vec ? B * (NN / 4) : B * NN;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units;
       u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = vec ? u * 4 : u;
    const int64_t b = e / NN, r = e - b * NN;
    const int i = (int)(r / N), j = (int)(r - (int64_t)i * N);
    const float2* row = locs + b * N;
    const float2 p = row[i];
    if (vec) {
      float d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 o = row[j + q];
        const float dx = p.x - o.x, dy = p.y - o.y;
        d[q] = sqrtf(dx * dx + dy * dy);
      }
      *reinterpret_cast<float4*>(out + e) = make_float4(d[0], d[1], d[2], d[3]);
    } else {
      const float2 o = row[j];
      const float dx = p.x - o.x, dy = p.y - o.y;
      out[e] = sqrtf(dx * dx + dy * dy);
    }
  }
}
}  // namespace

extern "C" int co_distance_matrix(int64_t B, int64_t N, const float* locs, float* out,
                                  void* stream) {
  if (B < 0 || N <= 0 || N > (1 << 15)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !out) return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(locs) & 7) || (reinterpret_cast<uintptr_t>(out) & 15))
    return CO_E_ALIGN;
  hipLaunchKernelGGL(distance_matrix_kernel, dim3(grid_for(B * N * N / 4 + 1, 256, 16384)),
                     dim3(256), 0, (hipStream_t)stream, B, (int)N,
                     reinterpret_cast<const float2*>(locs), out);
  return launch_status();
}
