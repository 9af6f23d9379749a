// Fused episode rollouts for gfx950: reset + every env step + episode reward in ONE
// launch, with the policy in-kernel (teacher-forced actions = Evaluate mode, or a
// cheap deterministic policy).  The per-step state transition is the reference's
// (tsp/env.py:67-93, slap/env.py:38-93) applied step by step; only the state a
// caller can observe after `rollout()` (rl4co/utils/decoding.py:88-109) is written:
// the final TensorDict columns, the actions (when chosen in-kernel) and the reward.
//
// TSP layout: one thread per instance, 64 instances per workgroup.  The tile's node
// coordinates are staged once into LDS by LDS-DMA (global_load_lds_dwordx4, the whole
// 51 KB tile in flight at once), the visited set lives in NW 64-bit
// registers, each step's action is one coalesced [B] row of the step-major action
// matrix, and the tour length accumulates in f64 as the steps go.  The final mask is
// expanded from the bit registers through LDS and stored as coalesced 16-byte rows.
#include "co_common.hpp"

using namespace co;

namespace {

constexpr int kRollT = 64;  // instances per workgroup (one wave)

// Visited-set bit ops on NW 64-bit registers, written as value selects (v_cndmask):
// a data-dependent `if` here becomes an exec-masked branch per step.
template <int NW>
__device__ __forceinline__ bool bit_test(const uint64_t (&m)[NW], int a) {
  const uint64_t bit = 1ull << (a & 63);
  const int w = a >> 6;
  uint64_t hit = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) hit |= m[k] & (w == k ? bit : 0ull);
  return hit != 0;
}

template <int NW>
__device__ __forceinline__ void bit_clear(uint64_t (&m)[NW], int a) {
  const uint64_t bit = 1ull << (a & 63);
  const int w = a >> 6;
#pragma unroll
  for (int k = 0; k < NW; ++k) m[k] &= ~(w == k ? bit : 0ull);
}

typedef __attribute__((address_space(3))) void lds_void;

// NW template value the launchers pick for N (1, 2 or 4 words of 64 bits)
inline int NW_launch(int64_t n) {
  const int w = (int)((n + 63) / 64);
  return w <= 1 ? 1 : (w == 2 ? 2 : 4);
}

// Copy `nbytes` contiguous bytes global -> LDS with LDS-DMA (global_load_lds_dwordx4):
// every wave-instruction moves 1 KiB to a wave-uniform LDS base + lane*16, no VGPR
// round trip, all pieces in flight before the single wait.  `src` and `dst` must be
// 16-byte aligned; a tail of < 16 bytes is copied with plain loads.  Ends with the
// vmcnt drain + workgroup barrier that make the tile visible.
__device__ __forceinline__ void stage_bytes_lds(const unsigned char* __restrict__ src, int nbytes,
                                                unsigned char* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n16 = nbytes & ~15;
  for (int base = wave * 1024; base < n16; base += nw * 1024) {
    const int off = base + lane * 16;
    if (off < n16)
      __builtin_amdgcn_global_load_lds((const void*)(src + off), (lds_void*)(dst + base), 16, 0, 0);
  }
  for (int k = n16 + (int)threadIdx.x; k < nbytes; k += blockDim.x) dst[k] = src[k];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}

// Stage a [rows, n] float2 tile into LDS with an ODD row stride S (in float2 slots) so
// that a half-wave reading the same column of 32 different rows hits 32 distinct bank
// pairs.  LDS-DMA writes lane-linear dwords, so the padding is produced on the SOURCE
// side: LDS dword w of the tile receives source dword (row r, dword d) with
// w = r*2S + d; pad dwords (d >= 2n) re-read the row's first dword.  Ends with the
// vmcnt drain + workgroup barrier.
__device__ __forceinline__ void stage_rows_padded_lds(const float2* __restrict__ src, int rows,
                                                      int n, int S, float2* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int W = 2 * S;  // dwords per padded row
  const int total = rows * W;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
  unsigned char* d8 = reinterpret_cast<unsigned char*>(dst);
  int w = wave * 64 + lane;
  int r = w / W, d = w - r * W;
  const int step = nw * 64;  // < W is not required: the wrap loop handles any step
  for (int base = wave * 64; base < total; base += step) {
    if (w < total) {
      const int sd = d < 2 * n ? d : 0;
      __builtin_amdgcn_global_load_lds((const void*)(s32 + (int64_t)r * 2 * n + sd),
                                       (lds_void*)(d8 + (size_t)base * 4), 4, 0, 0);
    }
    w += step;
    d += step;
    while (d >= W) {
      d -= W;
      ++r;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}

// Per-thread row of visited bits -> its row of the [rows, n] byte tile in LDS
// (dword writes when n % 4 == 0: conflict-free for odd n/4), then the whole tile is
// stored with coalesced 16-byte writes.  `scratch` must hold rows*n bytes, 16-aligned.
template <int NW>
__device__ __forceinline__ void store_mask_rows(const uint64_t (&m)[NW], bool live, int rows,
                                                int n, unsigned char* scratch,
                                                uint8_t* __restrict__ dst) {
  const int tid = threadIdx.x;
  if (live) {
    unsigned char* row = scratch + tid * n;
    if ((n & 3) == 0) {
      for (int c = 0; c < n; c += 4) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cc = c + j;
          uint64_t w = 0;
#pragma unroll
          for (int k = 0; k < NW; ++k)
            if ((cc >> 6) == k) w = m[k];
          v |= (uint32_t)((w >> (cc & 63)) & 1ull) << (8 * j);
        }
        *reinterpret_cast<uint32_t*>(row + c) = v;
      }
    } else {
      for (int c = 0; c < n; ++c) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k)
          if ((c >> 6) == k) w = m[k];
        row[c] = (unsigned char)((w >> (c & 63)) & 1ull);
      }
    }
  }
  __syncthreads();
  const int nbytes = rows * n;
  const int n16 = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? (nbytes & ~15) : 0;
  for (int off = tid * 16; off < n16; off += blockDim.x * 16)
    *reinterpret_cast<uint4*>(dst + off) = *reinterpret_cast<const uint4*>(scratch + off);
  for (int k = n16 + tid; k < nbytes; k += blockDim.x) dst[k] = scratch[k];
}

// STATE = false: reward + validity only (co_tsp_reward on step-major actions).
template <int NW, bool NEAREST, bool STATE = true>
__global__ __launch_bounds__(kRollT) void tsp_rollout_kernel(
    int64_t B, int N, const float2* __restrict__ locs, const int64_t* __restrict__ acts_in,
    int64_t* __restrict__ acts_out, uint8_t* __restrict__ mask_out, int64_t* __restrict__ first_out,
    int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out, int check,
    int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* s_xy = reinterpret_cast<float2*>(smem);  // [64][S] coordinates, then the mask bytes
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kRollT;
  const int rows = (int)((B - row0) < kRollT ? (B - row0) : kRollT);
  const int64_t b = row0 + tid;
  const bool live = tid < rows;

  const int S = NEAREST ? (N | 1) : N;  // padded rows only where lanes read one column
  // teacher: step 0 and the first action batch are loaded before the LDS-DMA drain
  constexpr int U = 16;
  int64_t bufA[U], bufB[U];
  int64_t a0_pref = 0;
  const int64_t* ap = acts_in + (live ? b : row0);  // this lane's column of [N, B]
  // rows [t0, t0+U) of the lane's column; the start is clamped so a prefetch past the
  // last full batch still reads in-bounds rows (its values are never used)
  auto load = [&](int64_t (&dst)[U], int t0) {
    const int tc = t0 + U <= N ? t0 : N - U;
    const int64_t* p = ap + (int64_t)tc * B;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dst[u] = *p;
      p += B;
    }
  };
  const int nfull = NEAREST ? 0 : (N - 1) / U;  // full batches after step 0
  if (!NEAREST) {
    a0_pref = ap[0];
    if (nfull > 0) load(bufA, 1);
  }
  if (NEAREST) {
    stage_rows_padded_lds(locs + row0 * N, rows, N, S, s_xy);
  } else {
    stage_bytes_lds(reinterpret_cast<const unsigned char*>(locs + row0 * N), rows * N * 8,
                    reinterpret_cast<unsigned char*>(s_xy));
  }
#if defined(CO_DIAG_PHASE) && CO_DIAG_PHASE == 1
  if (tid < rows && s_xy[tid].x == 12345.f) reward_out[b] = 1.f;
  return;
#endif

  const float2* xy = s_xy + tid * S;
  uint64_t m[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int lo = k * 64;
    m[k] = (N >= lo + 64) ? ~0ull : (N > lo ? ((1ull << (N - lo)) - 1ull) : 0ull);
  }
  // teacher mode keeps the visited set as 32-bit LDS words (odd stride VS per lane)
  constexpr int VS = 2 * NW + 1;
  uint32_t* s_vis = reinterpret_cast<uint32_t*>(smem + (size_t)kRollT * S * sizeof(float2));
  if (!NEAREST) {
#pragma unroll
    for (int kk = 0; kk < NW; ++kk) {
      s_vis[tid * VS + 2 * kk] = (uint32_t)m[kk];
      s_vis[tid * VS + 2 * kk + 1] = (uint32_t)(m[kk] >> 32);
    }
  }
  bool bad = false;
  int first = 0, a = 0;
  float px = 0.f, py = 0.f, fx = 0.f, fy = 0.f;
  double len = 0.0;
  // state transition of tsp/env.py:67-93 on the register state (mask bits + validity)
  auto visit = [&](int64_t a64) -> int {
    const bool in = (a64 >= 0) & (a64 < N);  // the reference's scatter would raise otherwise
    const int x = in ? (int)a64 : 0;
    bad |= (!in) | (!bit_test(m, x));        // revisit: not a permutation (tsp/env.py:168-173)
    bit_clear(m, x);
    return x;
  };
  if (live) {
    // step 0 (peeled): i == 0 -> first_node = action
    {
      int64_t a0;
      if (NEAREST) {
        a0 = 0;
        acts_out[b] = 0;
      } else {
        a0 = a0_pref;
      }
      a = first = visit(a0);
      if (!NEAREST) {  // mirror step 0 into the LDS words
        s_vis[tid * VS + (a >> 5)] &= ~(1u << (a & 31));
      }
      const float2 q = xy[a];
      px = fx = q.x;
      py = fy = q.y;
    }
    if (NEAREST) {
      for (int t = 1; t < N; ++t) {
        // nearest unvisited: argmin_j sqrt(dx*dx + dy*dy) with the lowest index on ties.
        // Ascending scan on squared distances; sqrt (correctly rounded, as ATen's) only
        // when a squared distance improves, and the switch needs a STRICTLY smaller
        // sqrt, so rounding ties keep the lower index exactly like torch.argmin.
        float best_sq = __builtin_inff(), best_r = __builtin_inff();
        int bi = 0;
        for (int j0 = 0; j0 < N; j0 += 8) {
          float sq[8];
          bool ok[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = j0 + u < N ? j0 + u : N - 1;
            const float2 q = xy[j];
            const float dx = q.x - px, dy = q.y - py;
            sq[u] = dx * dx + dy * dy;
            ok[u] = (j0 + u < N) & bit_test(m, j);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (ok[u] && sq[u] < best_sq) {
              const float r = sqrtf(sq[u]);
              if (r < best_r) {
                best_r = r;
                best_sq = sq[u];
                bi = j0 + u;
              }
            }
          }
        }
        acts_out[(int64_t)t * B + b] = bi;
        a = visit(bi);
        const float2 q = xy[a];
        len += (double)edge_len(px, py, q.x, q.y);
        px = q.x;
        py = q.y;
      }
    } else {
      // Teacher-forced.  Full batches of U = 16 steps, double-buffered (A/B alternate
      // without register copies, so the waits stay counted and one batch's coalesced
      // [B]-row action loads are in flight while the other batch runs).  A batch is one
      // basic block: U test-and-clear LDS atomics on the lane's visited words
      // (ds_and_rtn: the returned old word says whether the node was already visited),
      // U LDS coordinate reads, U independent edge lengths summed in f32, then one f64
      // add.  Edge lengths use the hardware v_sqrt_f32 (<= 1 ulp; reward parity is 1e-5
      // relative).
      uint32_t* vw = s_vis + tid * VS;
      uint32_t badw = 0;
      auto run = [&](const int64_t (&src)[U], int cnt) {  // cnt: steps used (uniform)
        int av[U];
        uint32_t old[U], bitv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < cnt) {
            const uint32_t lo = (uint32_t)src[u];
            const uint32_t in = ((uint32_t)(src[u] >> 32) == 0u) & (lo < (uint32_t)N);
            badw |= in ^ 1u;
            av[u] = in ? (int)lo : 0;
            bitv[u] = 1u << (av[u] & 31);
            old[u] = atomicAnd(&vw[av[u] >> 5], ~bitv[u]);
          }
        }
        float2 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u < cnt) q[u] = xy[av[u]];
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < cnt) {
            const float ox = u ? q[u - 1].x : px, oy = u ? q[u - 1].y : py;
            const float dx = q[u].x - ox, dy = q[u].y - oy;
            acc += __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
            badw |= ((old[u] & bitv[u]) == 0u);  // revisit (tsp/env.py:168-173)
          }
        }
        len += (double)acc;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u + 1 == cnt) {
            px = q[u].x;
            py = q[u].y;
            a = av[u];
          }
      };
      int k = 0;
      for (; k + 1 < nfull; k += 2) {
        load(bufB, 1 + (k + 1) * U);
        run(bufA, U);
        load(bufA, 1 + (k + 2) * U);
        run(bufB, U);
      }
      if (k < nfull) run(bufA, U);
      const int tail = N - 1 - nfull * U;  // < U steps left
      if (tail > 0) {
        const int t0 = 1 + nfull * U;
#pragma unroll
        for (int u = 0; u < U; ++u) bufB[u] = (u < tail) ? ap[(int64_t)(t0 + u) * B] : 0;
        run(bufB, tail);
      }
      bad |= badw != 0u;
      // the visited words back into the register bit set used by the state store
#pragma unroll
      for (int kk = 0; kk < NW; ++kk)
        m[kk] = (uint64_t)vw[2 * kk] | ((uint64_t)vw[2 * kk + 1] << 32);
    }
    len += (double)edge_len(px, py, fx, fy);  // closing edge (roll by -1)
  }
#if defined(CO_DIAG_PHASE) && CO_DIAG_PHASE == 2
  if (live) reward_out[b] = -(float)len + (float)(m[0] & 1) + (bad ? 1.f : 0.f);
  return;
#endif
  if (!STATE) {
    if (live) reward_out[b] = -(float)len;
    if (__any(bad && check) && tid == 0) set_status(status, CO_ST_INVALID_TOUR);
    return;
  }
  __syncthreads();  // every lane is done reading the coordinate tile
  store_mask_rows<NW>(m, live, rows, N, reinterpret_cast<unsigned char*>(s_xy),
                      mask_out + row0 * N);
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


// ----------------------------------------------------------------------------- SLAP
// One thread per instance for the P steps (slap/env.py:38-93: product p_t = the
// reset's to_choose[t] = t, assignment[p_t] = a_t, location a_t masked, done when
// i == P-1), the visited locations in NW bit registers and the assignment row in LDS
// (row stride P|1 dwords: conflict-free).  The reward (slap/env.py:131-143) is then
// computed one thread per (instance, order): the order's K picklist entries are a
// coalesced 8K-byte segment, product -> location through the LDS assignment, the
// closed pick tour summed in pick order (f32), and the orders of an instance added in
// order by the instance's thread.
template <int NW, bool CLOSEST>
__global__ __launch_bounds__(kRollT) void slap_rollout_kernel(
    int64_t B, int L, int P, int O, int K, const float2* __restrict__ locs,
    const int64_t* __restrict__ picklist, const float* __restrict__ depot_dist,
    const int32_t* __restrict__ assign_in, const int64_t* __restrict__ acts_in,
    int64_t* __restrict__ acts_out, uint8_t* __restrict__ mask_out,
    int32_t* __restrict__ assign_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out,
    float* __restrict__ ratio_out, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int PS = P | 1, LS = L | 1;  // odd row strides: conflict-free column access
  unsigned char* s_mask = smem;                                             // [64][L] bytes
  int32_t* s_asg = reinterpret_cast<int32_t*>(smem + ((kRollT * L + 15) & ~15));  // [64][PS]
  float* s_len = reinterpret_cast<float*>(s_asg + kRollT * PS);             // [64][O]
  float* s_dd = s_len + kRollT * O;                                         // [64][LS] (CLOSEST)
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kRollT;
  const int rows = (int)((B - row0) < kRollT ? (B - row0) : kRollT);
  const int64_t b = row0 + tid;
  const bool live = tid < rows;

  // stage the tile's initial assignment (the generator's -1s) and, for the policy,
  // the depot distances
  for (int k = tid; k < rows * P; k += kRollT) {
    const int r = k / P, c = k - r * P;
    s_asg[r * PS + c] = assign_in[row0 * P + k];
  }
  if (CLOSEST)
    for (int k = tid; k < rows * L; k += kRollT) {
      const int r = k / L, c = k - r * L;
      s_dd[r * LS + c] = depot_dist[row0 * L + k];
    }
  __syncthreads();

  uint64_t m[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int lo = k * 64;
    m[k] = (L >= lo + 64) ? ~0ull : (L > lo ? ((1ull << (L - lo)) - 1ull) : 0ull);
  }
  m[0] &= ~1ull;  // the depot (location 0) is never available (slap/env.py:115-116)
  bool range = false;
  if (live) {
    int32_t* arow = s_asg + tid * PS;
    const float* dd = s_dd + tid * LS;
    for (int t = 0; t < P; ++t) {
      int64_t a64;
      if (CLOSEST) {
        // ascending branch-free scan, strict < keeps the lowest index (torch.argmin)
        float best = __builtin_inff();
        int bi = 0;
        for (int j0 = 0; j0 < L; j0 += 8) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = j0 + u < L ? j0 + u : L - 1;
            const float d = dd[j];
            const bool take = (j0 + u < L) & bit_test(m, j) & (d < best);
            best = take ? d : best;
            bi = take ? j0 + u : bi;
          }
        }
        a64 = bi;
        acts_out[(int64_t)t * B + b] = a64;
      } else {
        a64 = acts_in[(int64_t)t * B + b];
      }
      arow[t] = (int32_t)a64;        // product t (to_choose[t] = t after reset)
      int64_t a = a64 < 0 ? a64 + L : a64;  // python indexing wraps negatives
      if (a < 0 || a >= L) {
        range = true;
      } else {
        bit_clear(m, (int)a);
      }
    }
  }
  __syncthreads();

  // reward: one thread per (instance, order)
  const int units = rows * O;
  for (int u = tid; u < units; u += kRollT) {
    const int r = u / O, o = u - r * O;
    const int64_t* pk = picklist + (row0 + r) * (int64_t)O * K + (int64_t)o * K;
    const int32_t* arow = s_asg + r * PS;
    const float2* lrow = locs + (row0 + r) * (int64_t)L;
    float2 p0 = make_float2(0.f, 0.f), prev = p0;
    float len = 0.f;
    for (int k = 0; k < K; ++k) {
      int64_t p = pk[k];
      if (p < 0) p += P;
      int64_t loc = 0;
      if (p < 0 || p >= P) {
        range = true;
      } else {
        loc = arow[p];
        if (loc < 0) loc += L;
        if (loc < 0 || loc >= L) {
          range = true;
          loc = 0;
        }
      }
      const float2 q = lrow[loc];
      if (k == 0) {
        p0 = q;
      } else {
        len += edge_len(prev.x, prev.y, q.x, q.y);
      }
      prev = q;
    }
    len += edge_len(prev.x, prev.y, p0.x, p0.y);
    s_len[r * O + o] = len;
  }
  __syncthreads();

  store_mask_rows<NW>(m, live, rows, L, s_mask, mask_out + row0 * L);
  for (int k = tid; k < rows * P; k += kRollT) {
    const int r = k / P, c = k - r * P;
    assign_out[row0 * P + k] = s_asg[r * PS + c];
  }
  if (ratio_out)
    for (int k = tid; k < rows * L; k += kRollT) ratio_out[row0 * L + k] = 0.f;
  if (live) {
    // f32 order-by-order accumulation of slap/env.py:135-142
    float total = 0.f;
    for (int o = 0; o < O; ++o) total += -s_len[tid * O + o];
    reward_out[b] = total;
    i_out[b] = P;
    done_out[b] = 1;  // the P-th step has i == P-1
    step_reward_out[b] = 0;
  }
  if (__any(range) && tid == 0) set_status(status, CO_ST_INDEX_RANGE);
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
  if (nearest)  // register-resident lane-group episode (nearest.hip)
    return co_internal_tsp_nearest_rollout(B, N, locs, acts_out, mask_out, first_out, cur_out,
                                           i_out, done_out, step_reward_out, reward_out, stream);
  if (reinterpret_cast<uintptr_t>(locs) & 15) return CO_E_ALIGN;  // LDS-DMA staging
  const int NW = (int)((N + 63) / 64);
  const size_t shmem = (size_t)kRollT * (nearest ? (N | 1) : N) * 8 +
                       (nearest ? 0 : (size_t)kRollT * (2 * NW_launch(N) + 1) * 4);
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
  if (NW == 1) CO_ROLL(1, false);
  else if (NW == 2) CO_ROLL(2, false);
  else CO_ROLL(4, false);
#undef CO_ROLL
  return launch_status();
}

// Reward + permutation check for step-major actions (element (b, t) at acts[t*st + b]),
// T == N: the thread-per-instance rollout body without the state outputs.  Called by
// co_tsp_reward when the actions come from the stepwise engine.
int co_internal_tsp_reward_stepmajor(int64_t B, int64_t N, const float* locs,
                                     const int64_t* acts, int64_t st, int check, float* reward,
                                     int32_t* status, void* stream) {
  if (st != B || N > 256 || (reinterpret_cast<uintptr_t>(locs) & 15)) return CO_E_INVAL;
  const int NW = (int)((N + 63) / 64);
  const size_t shmem = (size_t)kRollT * N * 8 + (size_t)kRollT * (2 * NW_launch(N) + 1) * 4;
  const dim3 grid((unsigned)((B + kRollT - 1) / kRollT)), block(kRollT);
  hipStream_t s = (hipStream_t)stream;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
#define CO_RW(W)                                                                               \
  do {                                                                                         \
    if (shmem > 64 * 1024)                                                                     \
      (void)hipFuncSetAttribute((const void*)tsp_rollout_kernel<W, false, false>,              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);       \
    hipLaunchKernelGGL((tsp_rollout_kernel<W, false, false>), grid, block, shmem, s, B,        \
                       (int)N, l2, acts, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, \
                       nullptr, reward, check, status);                                        \
  } while (0)
  if (NW == 1) CO_RW(1);
  else if (NW == 2) CO_RW(2);
  else CO_RW(4);
#undef CO_RW
  return launch_status();
}

extern "C" int co_slap_rollout(int64_t B, int64_t L, int64_t P, int64_t O, int64_t K,
                               const float* locs, const int64_t* picklist,
                               const float* depot_dist, const int32_t* assign_in,
                               const int64_t* acts_in, int64_t* acts_out, uint8_t* mask_out,
                               int32_t* assign_out, int64_t* i_out, uint8_t* done_out,
                               uint8_t* step_reward_out, float* reward_out, float* ratio_out,
                               int32_t* status, void* stream) {
  if (B < 0 || L <= 1 || L > 256 || P <= 0 || O <= 0 || K <= 0 || P > 4096) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  const bool closest = acts_in == nullptr;
  if (!locs || !picklist || !assign_in || !mask_out || !assign_out || !i_out || !done_out ||
      !step_reward_out || !reward_out || !status || (closest && (!acts_out || !depot_dist)))
    return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  const int NW = (int)((L + 63) / 64);
  const int PS = (int)P | 1;
  size_t shmem = (((size_t)kRollT * L + 15) & ~(size_t)15) + (size_t)kRollT * PS * 4 +
                 (size_t)kRollT * O * 4 + (closest ? (size_t)kRollT * ((int)L | 1) * 4 : 0);
  if (shmem > 160 * 1024) return CO_E_INVAL;
  const dim3 grid((unsigned)((B + kRollT - 1) / kRollT)), block(kRollT);
  hipStream_t s = (hipStream_t)stream;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
#define CO_SLAP(W, C)                                                                          \
  do {                                                                                         \
    if (shmem > 64 * 1024)                                                                     \
      (void)hipFuncSetAttribute((const void*)slap_rollout_kernel<W, C>,                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);       \
    hipLaunchKernelGGL((slap_rollout_kernel<W, C>), grid, block, shmem, s, B, (int)L, (int)P,  \
                       (int)O, (int)K, l2, picklist, depot_dist, assign_in, acts_in, acts_out, \
                       mask_out, assign_out, i_out, done_out, step_reward_out, reward_out,     \
                       ratio_out, status);                                                     \
  } while (0)
  if (closest) {
    if (NW == 1) CO_SLAP(1, true);
    else if (NW == 2) CO_SLAP(2, true);
    else CO_SLAP(4, true);
  } else {
    if (NW == 1) CO_SLAP(1, false);
    else if (NW == 2) CO_SLAP(2, false);
    else CO_SLAP(4, false);
  }
#undef CO_SLAP
  return launch_status();
}
