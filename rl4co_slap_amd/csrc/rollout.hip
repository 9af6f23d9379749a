// Fused episode rollouts for gfx950: reset + every env step + episode reward in ONE
// launch, with the policy in-kernel (teacher-forced actions = Evaluate mode, or a
// cheap deterministic policy).  The per-step state transition is the reference's
// (tsp/env.py:67-93, slap/env.py:38-93) applied step by step; only the state a
// caller can observe after `rollout()` (rl4co/utils/decoding.py:88-109) is written:
// the final TensorDict columns, the actions (when chosen in-kernel) and the reward.
//
// TSP layout: one thread per instance, 64 instances per workgroup.  The tile's node
// coordinates are staged once into LDS (coalesced 16-byte loads; rows padded to an
// odd number of 8-byte slots so the 32 lanes of a ds_read_b64 half-wave hit distinct
// banks when they read the same column), the visited set lives in NW 64-bit
// registers, each step's action is one coalesced [B] row of the step-major action
// matrix, and the tour length accumulates in f64 as the steps go.  The final mask is
// expanded from the bit registers through LDS and stored as coalesced 16-byte rows.
#include "co_common.hpp"

using namespace co;

namespace {

constexpr int kRollT = 64;  // instances per workgroup (one wave)

__device__ __forceinline__ int odd_stride(int n) { return n | 1; }

template <int NW>
__device__ __forceinline__ bool bit_test(const uint64_t (&m)[NW], int a) {
  uint64_t w = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k)
    if ((a >> 6) == k) w = m[k];
  return (w >> (a & 63)) & 1ull;
}

template <int NW>
__device__ __forceinline__ void bit_clear(uint64_t (&m)[NW], int a) {
#pragma unroll
  for (int k = 0; k < NW; ++k)
    if ((a >> 6) == k) m[k] &= ~(1ull << (a & 63));
}

// Stage rows [row0, row0+rows) of a [*, n] float2 array into LDS with row stride S.
__device__ __forceinline__ void stage_rows(const float2* __restrict__ src, int64_t row0, int rows,
                                           int n, int S, float2* dst) {
  const int64_t nodes = (int64_t)rows * n;
  const float2* s = src + row0 * n;
  const bool al16 = ((reinterpret_cast<uintptr_t>(s) & 15) == 0);
  if (al16) {
    const int64_t pairs = nodes >> 1;
    for (int64_t k = threadIdx.x; k < pairs; k += blockDim.x) {
      const float4 v = reinterpret_cast<const float4*>(s)[k];
      const int64_t e0 = 2 * k;
      const int r0 = (int)(e0 / n), c0 = (int)(e0 - (int64_t)r0 * n);
      dst[r0 * S + c0] = make_float2(v.x, v.y);
      const int c1 = c0 + 1 == n ? 0 : c0 + 1, r1 = c0 + 1 == n ? r0 + 1 : r0;
      dst[r1 * S + c1] = make_float2(v.z, v.w);
    }
    if ((nodes & 1) && threadIdx.x == 0) {
      const int64_t e = nodes - 1;
      dst[(int)(e / n) * S + (int)(e % n)] = s[e];
    }
  } else {
    for (int64_t e = threadIdx.x; e < nodes; e += blockDim.x)
      dst[(int)(e / n) * S + (int)(e % n)] = s[e];
  }
}

// Expand per-row visited bits (LDS, [rows][NW]) into the [rows, n] bool tile in HBM.
template <int NW>
__device__ __forceinline__ void store_mask_tile(const uint64_t* bits, int rows, int n,
                                                uint8_t* __restrict__ dst) {
  const int nbytes = rows * n;
  const bool al16 = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
  const int nch = (nbytes + 15) >> 4;
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
    const int off = c << 4;
    union {
      uint4 v;
      uint8_t b[16];
    } u;
    int r = off / n, col = off - r * n;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint8_t v = 0;
      if (off + j < nbytes) v = (uint8_t)((bits[r * NW + (col >> 6)] >> (col & 63)) & 1ull);
      u.b[j] = v;
      if (++col == n) { col = 0; ++r; }
    }
    if (al16 && off + 16 <= nbytes) {
      *reinterpret_cast<uint4*>(dst + off) = u.v;
    } else {
      for (int j = 0; j < 16 && off + j < nbytes; ++j) dst[off + j] = u.b[j];
    }
  }
}

template <int NW, bool NEAREST>
__global__ __launch_bounds__(kRollT) void tsp_rollout_kernel(
    int64_t B, int N, const float2* __restrict__ locs, const int64_t* __restrict__ acts_in,
    int64_t* __restrict__ acts_out, uint8_t* __restrict__ mask_out, int64_t* __restrict__ first_out,
    int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out, int check,
    int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = odd_stride(N);
  float2* s_xy = reinterpret_cast<float2*>(smem);
  uint64_t* s_bits = reinterpret_cast<uint64_t*>(smem + (size_t)kRollT * S * sizeof(float2));
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kRollT;
  const int rows = (int)((B - row0) < kRollT ? (B - row0) : kRollT);
  const int64_t b = row0 + tid;
  const bool live = tid < rows;

  stage_rows(locs, row0, rows, N, S, s_xy);
  __syncthreads();

  const float2* xy = s_xy + tid * S;
  uint64_t m[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int lo = k * 64;
    m[k] = (N >= lo + 64) ? ~0ull : (N > lo ? ((1ull << (N - lo)) - 1ull) : 0ull);
  }
  bool bad = false;
  int first = 0, a = 0;
  float px = 0.f, py = 0.f, fx = 0.f, fy = 0.f;
  double len = 0.0;
  // one env step of tsp/env.py:67-93 on the register state + the tour-length edge
  auto step = [&](int t, int64_t a64) {
    if (a64 < 0 || a64 >= N) {  // the reference's scatter would raise
      bad = true;
      a64 = 0;
    }
    a = (int)a64;
    if (!bit_test(m, a)) bad = true;  // revisit: not a permutation (tsp/env.py:168-173)
    bit_clear(m, a);
    const float2 q = xy[a];
    if (t == 0) {
      first = a;
      fx = q.x;
      fy = q.y;
    } else {
      len += (double)edge_len(px, py, q.x, q.y);
    }
    px = q.x;
    py = q.y;
  };
  if (live) {
    if (NEAREST) {
      for (int t = 0; t < N; ++t) {
        int bi = 0;
        if (t > 0) {
          float best = __builtin_inff();
#pragma unroll
          for (int k = 0; k < NW; ++k) {
            uint64_t w = m[k];
            while (w) {
              const int j = k * 64 + __builtin_ctzll(w);
              w &= w - 1;
              const float2 q = xy[j];
              const float d = edge_len(px, py, q.x, q.y);
              if (d < best) { best = d; bi = j; }
            }
          }
        }
        acts_out[(int64_t)t * B + b] = bi;
        step(t, bi);
      }
    } else {
      // teacher-forced: 8 coalesced action loads in flight ahead of the dependent steps
      constexpr int U = 8;
      for (int t0 = 0; t0 < N; t0 += U) {
        int64_t av[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          av[u] = (t0 + u < N) ? acts_in[(int64_t)(t0 + u) * B + b] : 0;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (t0 + u < N) step(t0 + u, av[u]);
      }
    }
    len += (double)edge_len(px, py, fx, fy);  // closing edge (roll by -1)
  }
#pragma unroll
  for (int k = 0; k < NW; ++k) s_bits[tid * NW + k] = live ? m[k] : 0ull;
  __syncthreads();
  store_mask_tile<NW>(s_bits, rows, N, mask_out + row0 * N);
  if (live) {
    bool empty = true;
#pragma unroll
    for (int k = 0; k < NW; ++k) empty &= (m[k] == 0);
    first_out[b] = first;
    cur_out[b] = a;
    i_out[b] = N;
    done_out[b] = empty;
    step_reward_out[b] = 0;
    reward_out[b] = -(float)len;
  }
  if (__any(bad && check) && tid == 0) set_status(status, CO_ST_INVALID_TOUR);
}

}  // namespace

extern "C" int co_tsp_rollout(int64_t B, int64_t N, const float* locs, const int64_t* acts_in,
                              int64_t* acts_out, uint8_t* mask_out, int64_t* first_out,
                              int64_t* cur_out, int64_t* i_out, uint8_t* done_out,
                              uint8_t* step_reward_out, float* reward_out, int check,
                              int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > 256) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  const bool nearest = acts_in == nullptr;
  if (!locs || !mask_out || !first_out || !cur_out || !i_out || !done_out || !step_reward_out ||
      !reward_out || (nearest && !acts_out) || (check && !status))
    return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  const int S = (int)N | 1;
  const int NW = (int)((N + 63) / 64);
  const size_t shmem = (size_t)kRollT * S * 8 + (size_t)kRollT * NW * 8;
  const dim3 grid((unsigned)((B + kRollT - 1) / kRollT)), block(kRollT);
  hipStream_t s = (hipStream_t)stream;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
#define CO_ROLL(W, NEAR)                                                                       \
  do {                                                                                         \
    if (shmem > 64 * 1024)                                                                     \
      (void)hipFuncSetAttribute((const void*)tsp_rollout_kernel<W, NEAR>,                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);       \
    hipLaunchKernelGGL((tsp_rollout_kernel<W, NEAR>), grid, block, shmem, s, B, (int)N, l2,    \
                       acts_in, acts_out, mask_out, first_out, cur_out, i_out, done_out,       \
                       step_reward_out, reward_out, check, status);                            \
  } while (0)
  if (nearest) {
    if (NW == 1) CO_ROLL(1, true);
    else if (NW == 2) CO_ROLL(2, true);
    else CO_ROLL(4, true);
  } else {
    if (NW == 1) CO_ROLL(1, false);
    else if (NW == 2) CO_ROLL(2, false);
    else CO_ROLL(4, false);
  }
#undef CO_ROLL
  return launch_status();
}
