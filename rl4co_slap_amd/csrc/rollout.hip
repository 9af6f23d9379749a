// Fused episode rollouts for gfx950: reset + every env step + episode reward in ONE
// launch, with the policy in-kernel (teacher-forced actions = Evaluate mode, or a
// cheap deterministic policy).  The per-step state transition is the reference's
// (tsp/env.py:67-93, slap/env.py:38-93) applied step by step; only the state a
// caller can observe after `rollout()` (rl4co/utils/decoding.py:88-109) is written:
// the final TensorDict columns, the actions (when chosen in-kernel) and the reward.
//
// TSP (teacher-forced): 64 instances per workgroup over Q waves; coordinates staged by
// LDS-DMA, visited words in LDS shared by the waves, step-major action rows
// double-buffered.  SLAP: G-lane groups per instance with the free-location set in
// VGPRs.  The nearest-policy TSP and the CVRP episodes are in nearest.hip.
#include "co_common.hpp"

using namespace co;

namespace {


// NW template value the launchers pick for N (1, 2 or 4 words of 64 bits)
inline int NW_launch(int64_t n) {
  const int w = (int)((n + 63) / 64);
  return w <= 1 ? 1 : (w == 2 ? 2 : 4);
}

// Columns [c_lo, c_hi) of a row of visited bits -> mask bytes (1 = still feasible) of
// `row` in LDS (dword writes when n % 4 == 0 and c_lo % 4 == 0: conflict-free for odd
// n/4).
template <int NW>
__device__ __forceinline__ void mask_row_to_lds(const uint64_t (&m)[NW], int n,
                                                unsigned char* row, int c_lo = 0,
                                                int c_hi = -1) {
  if (c_hi < 0) c_hi = n;
  if ((n & 3) == 0 && (c_lo & 3) == 0) {
    for (int c = c_lo; c < c_hi; c += 4) {
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
    for (int c = c_lo; c < c_hi; ++c) {
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < NW; ++k)
        if ((c >> 6) == k) w = m[k];
      row[c] = (unsigned char)((w >> (c & 63)) & 1ull);
    }
  }
}

// The whole block copies an LDS byte tile to global memory with coalesced 16-byte
// stores (byte stores for a misaligned destination or the tail).
__device__ __forceinline__ void copy_tile_out(const unsigned char* scratch, int nbytes,
                                              uint8_t* __restrict__ dst) {
  const int tid = threadIdx.x;
  const int n16 = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? (nbytes & ~15) : 0;
  for (int off = tid * 16; off < n16; off += blockDim.x * 16)
    *reinterpret_cast<uint4*>(dst + off) = *reinterpret_cast<const uint4*>(scratch + off);
  for (int k = n16 + tid; k < nbytes; k += blockDim.x) dst[k] = scratch[k];
}

// The whole block writes zeros over a tile of mask bytes (16-byte stores when aligned).
__device__ __forceinline__ void zero_tile_out(int nbytes, uint8_t* __restrict__ dst) {
  const int tid = threadIdx.x;
  const int n16 = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? (nbytes & ~15) : 0;
  for (int off = tid * 16; off < n16; off += blockDim.x * 16)
    *reinterpret_cast<uint4*>(dst + off) = make_uint4(0u, 0u, 0u, 0u);
  for (int k = n16 + tid; k < nbytes; k += blockDim.x) dst[k] = 0;
}

#ifndef CO_TEACH_ZFAST
#define CO_TEACH_ZFAST 1  // all-visited tiles store zero mask rows without the LDS expansion
#endif

// LDS bytes of the TSP teacher kernel's coordinate tile region: [64][N] float2, or the
// post-episode scratch (mask bytes, Q x 64 partial sums, last node) if larger.
__host__ __device__ inline size_t tsp_tile_bytes(int N, int Q) {
  const size_t xy = (size_t)64 * N * 8;
  const size_t scr = (((size_t)64 * N + 15) & ~(size_t)15) + (size_t)Q * 64 * 8 + 64 * 8 + 64 * 4 +
                     16 * 4;  // + per-wave "all visited" flags
  return ((xy > scr ? xy : scr) + 15) & ~(size_t)15;
}

// Teacher-forced TSP episode (Evaluate mode): 64 instances per workgroup, Q waves.
// The tile's coordinates are staged once into LDS by LDS-DMA; the visited set of
// instance `lane` is 32-bit LDS words shared by the Q waves (ds_and_rtn: the returned
// old word says whether the node was already visited, in whichever wave).  Wave q
// walks steps [1 + q*R, 1 + (q+1)*R) of the lane's instance (wave 0 also step 0), so
// a tile's serial step chain is Q times shorter and a CU holds 3Q waves; each step's
// action is one coalesced [B] row of the step-major action matrix, double-buffered in
// batches of U.  Partial tour lengths (f32 per batch, f64 across batches) are added in
// wave order after a barrier, then the closing edge.  STATE = false: reward + validity
// only (co_tsp_reward on step-major actions).
#ifndef CO_TEACH_Q
#define CO_TEACH_Q 4
#endif
#ifndef CO_TEACH_U
#define CO_TEACH_U 8
#endif
// NB > 0: a wave's whole step range (<= NB*U steps) is loaded into registers at the
// kernel's start, in flight together with the coordinate staging, so the walk itself
// waits on LDS only; NB == 0: U-step batches double-buffered during the walk (long N).
#ifndef CO_TEACH_NB
#define CO_TEACH_NB 0
#endif
template <int NW, int Q, bool STATE, int NB = 0>
__global__ __launch_bounds__(64 * Q) void tsp_teacher_kernel(
    int64_t B, int N, const float2* __restrict__ locs, int64_t LB,
    const int64_t* __restrict__ acts_in, uint8_t* __restrict__ mask_out,
    int64_t* __restrict__ first_out, int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out,
    uint8_t* __restrict__ done_out, uint8_t* __restrict__ step_reward_out,
    float* __restrict__ reward_out, int check, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* s_xy = reinterpret_cast<float2*>(smem);  // [64][N] coordinates, later scratch
  constexpr int VS = 2 * NW + 1;                    // visited words per instance (odd)
  uint32_t* s_vis = reinterpret_cast<uint32_t*>(smem + tsp_tile_bytes(N, Q));
  const int lane = threadIdx.x & 63, q = wave_in_block();
  const int64_t row0 = (int64_t)blockIdx.x * 64;
  const int rows = (int)((B - row0) < 64 ? (B - row0) : 64);
  const int64_t b = row0 + lane;
  const bool live = lane < rows;

  const int R = (N - 1 + Q - 1) / Q;  // steps per wave after step 0
  const int t_lo = 1 + q * R < N ? 1 + q * R : N;
  const int t_hi = t_lo + R < N ? t_lo + R : N;
  constexpr int U = CO_TEACH_U;
  int64_t bufA[U], bufB[U];
  const int64_t* ap = acts_in + (live ? b : row0);  // this lane's column of [N, B]
  // rows [t0, t0+U) of the lane's column, start clamped into [t_lo, t_hi - U] so a
  // prefetch past the last full batch reads in-bounds rows (its values are never used)
  auto load = [&](int64_t (&dst)[U], int t0) {
    const int tc = t0 + U <= t_hi ? t0 : t_hi - U;
    const int64_t* p = ap + (int64_t)tc * B;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dst[u] = *p;
      p += B;
    }
  };
  const int nfull = (t_hi - t_lo) / U;
  // wave 0: step 0's action; wave q > 0: the action before its range (previous node)
  const int64_t a_prev = ap[(int64_t)(q == 0 ? 0 : t_lo - 1) * B];
  int64_t pre[NB > 0 ? NB * U : 1];
  if constexpr (NB > 0) {
    // every step of the range at once (rows past t_hi re-read the range's last row,
    // in bounds, never used); the walk below then waits on LDS only
#pragma unroll
    for (int j = 0; j < NB * U; ++j) {
      const int tj = t_lo + j < t_hi ? t_lo + j : (t_hi > 0 ? t_hi - 1 : 0);
      pre[j] = ap[(int64_t)tj * B];
    }
  } else if (nfull > 0) {
    load(bufA, t_lo);
  }
  if (q == 0) {
    for (int k = 0; k < NW; ++k) {
      const int lo = k * 64;
      const uint64_t w = (N >= lo + 64) ? ~0ull : (N > lo ? ((1ull << (N - lo)) - 1ull) : 0ull);
      s_vis[lane * VS + 2 * k] = (uint32_t)w;
      s_vis[lane * VS + 2 * k + 1] = (uint32_t)(w >> 32);
    }
  }
  // env e uses coordinate row e % LB (POMO: the S starts share an instance's row); the
  // launcher guarantees LB == B or LB % 64 == 0, so a tile never wraps
  stage_bytes_lds(reinterpret_cast<const unsigned char*>(locs + (row0 % LB) * N), rows * N * 8,
                  reinterpret_cast<unsigned char*>(s_xy));  // ends with a barrier
  const float2* xy = s_xy + lane * N;
  uint32_t* vw = s_vis + lane * VS;
  uint32_t badw = 0;
  int a = 0;
  float px = 0.f, py = 0.f, fx = 0.f, fy = 0.f;  // (fx, fy): wave 0's first node
  double len = 0.0;
  if (live) {
    const uint32_t lo = (uint32_t)a_prev;
    const uint32_t in = ((uint32_t)(a_prev >> 32) == 0u) & (lo < (uint32_t)N);
    a = in ? (int)lo : 0;
    if (q == 0) {  // step 0 (i == 0 -> first_node = action)
      badw |= in ^ 1u;
      // no-return clear: a revisit leaves some node's bit set (N steps, N nodes), which
      // the final visited words show -- the permutation check of tsp/env.py:168-173
      __hip_atomic_fetch_and(&vw[a >> 5], ~(1u << (a & 31)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const float2 p0 = xy[a];
    px = fx = p0.x;
    py = fy = p0.y;
    // A batch is one basic block: U LDS coordinate reads, U no-return visited-bit clears
    // (a revisit shows in the final visited words: N steps over N nodes clear them all
    // exactly when the actions are a permutation), U independent edge lengths, each added
    // in f64 (the f32 length then does not depend on the order: a tour and its reverse
    // score the same) -- one LDS round trip per batch.  Edge lengths use the hardware
    // v_sqrt_f32 (<= 1 ulp; reward parity is 1e-5 relative).
    auto run = [&](const int64_t (&src)[U], int cnt) {  // cnt: steps used (uniform)
      int av[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < cnt) {
          const uint32_t l32 = (uint32_t)src[u];
          const uint32_t ok = ((uint32_t)(src[u] >> 32) == 0u) & (l32 < (uint32_t)N);
          badw |= ok ^ 1u;
          av[u] = ok ? (int)l32 : 0;
        }
      }
      float2 qq[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < cnt) qq[u] = xy[av[u]];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < cnt)
          __hip_atomic_fetch_and(&vw[av[u] >> 5], ~(1u << (av[u] & 31)), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      // keep the batch's LDS operations issued back to back (the scheduler otherwise
      // splits the reads into groups with a full wait between them)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < cnt) {
          const float ox = u ? qq[u - 1].x : px, oy = u ? qq[u - 1].y : py;
          const float dx = qq[u].x - ox, dy = qq[u].y - oy;
          len += (double)__builtin_amdgcn_sqrtf(dx * dx + dy * dy);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u + 1 == cnt) {
          px = qq[u].x;
          py = qq[u].y;
          a = av[u];
        }
    };
    if constexpr (NB > 0) {
      const int cnt = t_hi - t_lo;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
        for (int u = 0; u < U; ++u) bufA[u] = pre[kb * U + u];
        if (cnt >= (kb + 1) * U)
          run(bufA, U);  // full batch: straight-line code (a compile-time count)
        else if (cnt > kb * U)
          run(bufA, cnt - kb * U);
      }
    } else {
      int k = 0;
      for (; k + 1 < nfull; k += 2) {
        load(bufB, t_lo + (k + 1) * U);
        run(bufA, U);
        load(bufA, t_lo + (k + 2) * U);
        run(bufB, U);
      }
      if (k < nfull) run(bufA, U);
      const int tail = t_hi - t_lo - nfull * U;  // < U steps left
      if (tail > 0) {
        const int t0 = t_lo + nfull * U;
#pragma unroll
        for (int u = 0; u < U; ++u) bufB[u] = (u < tail) ? ap[(int64_t)(t0 + u) * B] : 0;
        run(bufB, tail);
      }
    }
  }
  // out-of-range actions seen by this wave (revisits: from the final words below)
  if (__any(badw != 0u && check) && lane == 0) set_status(status, CO_ST_INVALID_TOUR);
  __syncthreads();  // steps done: the coordinate tile is free, the visited words final
  // scratch in the tile region: [64][N] mask bytes, then per-wave partial sums and the
  // last wave's final node
  const int qlast = N >= 2 ? (N - 2) / R : 0;
  const size_t mbytes = ((size_t)64 * N + 15) & ~(size_t)15;
  double* s_len = reinterpret_cast<double*>(smem + mbytes);  // [Q][64]
  float2* s_last = reinterpret_cast<float2*>(s_len + Q * 64);  // [64]
  int* s_lasta = reinterpret_cast<int*>(s_last + 64);          // [64]
  s_len[q * 64 + lane] = len;
  if (q == qlast) {
    s_last[lane] = make_float2(px, py);
    s_lasta[lane] = a;
  }
  uint64_t m[NW];
#pragma unroll
  for (int kk = 0; kk < NW; ++kk) m[kk] = (uint64_t)vw[2 * kk] | ((uint64_t)vw[2 * kk + 1] << 32);
  bool empty = true;
#pragma unroll
  for (int kk = 0; kk < NW; ++kk) empty &= (m[kk] == 0);
  // a node left unvisited after N steps = some node visited twice (or an out-of-range
  // action, already flagged): not a permutation
  if (q == 0 && __any(live && !empty && check) && lane == 0)
    set_status(status, CO_ST_INVALID_TOUR);
  // Every instance of the tile fully visited (any valid tour): its mask rows are all zero
  // and are stored as zeros, without the LDS expansion and its read-back.
  int* s_flag = s_lasta + 64;  // [Q]
  bool all_empty = false;
  if (STATE && CO_TEACH_ZFAST) {
    const bool wave_empty = __ballot(live && !empty) == 0ull;
    if (lane == 0) s_flag[q] = wave_empty;
    __syncthreads();
    all_empty = true;
#pragma unroll
    for (int w = 0; w < Q; ++w) all_empty &= s_flag[w] != 0;
  }
  if (STATE && !all_empty) {
    if (live) {  // the Q waves expand column quarters of the lane's mask row
      const int per = ((N + 4 * Q - 1) / (4 * Q)) * 4;
      const int c_lo = q * per < N ? q * per : N;
      const int c_hi = c_lo + per < N ? c_lo + per : N;
      mask_row_to_lds<NW>(m, N, smem + (size_t)lane * N, c_lo, c_hi);
    }
    __syncthreads();
  } else if (!STATE) {
    __syncthreads();
  }
  if (q == 0 && live) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < Q; ++w) tot += s_len[w * 64 + lane];
    const float2 pl = s_last[lane];
    const int first = ((uint64_t)a_prev < (uint64_t)N) ? (int)a_prev : 0;  // step 0's action
    tot += (double)edge_len(pl.x, pl.y, fx, fy);  // closing edge (roll by -1)
    reward_out[b] = -(float)tot;
    if (STATE) {
      first_out[b] = first;
      cur_out[b] = s_lasta[lane];
      i_out[b] = N;
      done_out[b] = empty;
      step_reward_out[b] = 0;
    }
  }
  if (STATE) {
    if (all_empty)
      zero_tile_out(rows * N, mask_out + row0 * N);
    else
      copy_tile_out(smem, rows * N, mask_out + row0 * N);
  }
}

// Teacher-forced TSP episode on ROW-MAJOR actions [B, N] (element (b, t) at
// acts[b*sb + t]: the reference's own [B, T] layout, ConstructivePolicy's `actions`):
// G lanes per instance, lane sl owns the EPL consecutive steps t = sl*EPL + k.  Every
// input is read as a contiguous row: MODE 2 (the headline's) stages a wave's GPW action
// rows and GPW coordinate rows by LDS-DMA as two contiguous blocks and reads steps and
// coordinate gathers from LDS; MODE 0 / 1 read the instance's 8N bytes of actions from
// memory (scalar / 16-byte vectors) and gather its coordinates within one row (whole
// lines, L2).  One block of instances per wave, all of B in flight.  The visited set
// is a per-group LDS bitmap (no-return ds_or per step); the actions are a permutation iff
// all N bits are set after the N steps (and every action is in range).  Edge lengths in
// f32 (hardware sqrt, <= 1 ulp; reward parity is 1e-5 relative): within a lane, to the
// next lane's first step (lane shuffle) and the closing edge, lane sums added in f64.
// STATE = false: reward + validity only (co_tsp_reward on row-major actions, T == N);
// coordinates of env e come from row e % LB (POMO multistart).
#ifndef CO_ROWS_EPL112
#define CO_ROWS_EPL112 7  // steps per lane for 96 < N <= 112 (16 lanes)
#endif
#ifndef CO_ROWS_DMA
#define CO_ROWS_DMA 1  // the row kernel stages a wave's rows by LDS-DMA when it can
#endif

// LDS bytes per wave of the LDS-DMA variant: the wave's GPW coordinate rows and action
// rows, contiguous in memory, land in LDS as two blocks of GPW*N*8 bytes.
__host__ __device__ inline size_t tsp_rows_wave_bytes(int gpw, int N) {
  return (((size_t)gpw * N * 8 + 15) & ~(size_t)15) * 2;
}

// MODE 0: scalar 8-byte action loads; 1: 16-byte vectors (16-byte aligned rows); 2: the
// wave's GPW action and coordinate rows (contiguous: sb == N, consecutive coordinate
// rows) staged by LDS-DMA as two contiguous blocks, steps and gathers then read from LDS.
#ifndef CO_ROWS_WPB
#define CO_ROWS_WPB 4  // waves per workgroup of the row kernel (r06: 2 / 8 / 16 slower)
#endif
// Round 6: the inputs are read once and the outputs written once, so the row kernel's
// LDS-DMA loads carry the non-temporal hint (nt: streamed past the caches' normal
// retention) and its mask rows are non-temporal stores -- 23.0 -> 20.7 us per launch at
// B = 65,536 (HIP events, same box A/B; sc0 / sc1 variants measured no better).
#ifndef CO_ROWS_AUX
#define CO_ROWS_AUX 2  // cache-policy bits of the row kernel's LDS-DMA loads (2 = nt)
#endif
#ifndef CO_ROWS_NTST
#define CO_ROWS_NTST 1  // non-temporal mask-row stores
#endif
#ifndef CO_ROWS_MODE3
#define CO_ROWS_MODE3 1  // coordinates by LDS-DMA, actions loaded straight into registers
                         // (r06: half the LDS per wave; 20.7 -> 19.1 us, same-box A/B)
#endif
#ifndef CO_ROWS_AV4
#define CO_ROWS_AV4 0  // MODE 3: the actions as 16-byte pieces (odd EPL; r06: no faster, off)
#endif
#ifndef CO_ROWS_ANT
#define CO_ROWS_ANT 0  // MODE 3: the action loads non-temporal (r06: 19.1 -> 35.7 us, partial lines)
#endif
template <int G, int EPL, int MODE, bool STATE>
__global__ __launch_bounds__(64 * CO_ROWS_WPB) void tsp_teacher_rows_kernel(
    int64_t B, int N, const float2* __restrict__ locs, int64_t LB,
    const int64_t* __restrict__ acts, int64_t sb, uint8_t* __restrict__ mask_out,
    int64_t* __restrict__ first_out, int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out,
    uint8_t* __restrict__ done_out, uint8_t* __restrict__ step_reward_out,
    float* __restrict__ reward_out, int check, int32_t* status) {
  constexpr int GPW = 64 / G;
  // 16-byte action pairs only when every lane's first step t0 = sl*EPL is even (the row
  // base is 16-byte aligned): an odd EPL takes the scalar loads
  // MODE 3: the coordinate rows by LDS-DMA (nt), the actions straight into registers
  constexpr bool VEC = MODE == 1 && EPL % 2 == 0, DMA = MODE == 2 || MODE == 3,
                 ADMA = MODE == 2;
  __shared__ uint32_t s_bits[CO_ROWS_WPB][GPW][(G * EPL + 31) / 32];
  extern __shared__ __attribute__((aligned(16))) unsigned char s_rows[];  // DMA: per wave
  constexpr int NWB = (G * EPL + 31) / 32;
  const int lane = lane_id(), sl = lane % G, grp = lane / G, w = wave_in_block();
  uint32_t* bits = s_bits[w][grp];
  const size_t half = DMA ? tsp_rows_wave_bytes(GPW, N) / 2 : 0;
  unsigned char* s_w = s_rows + (DMA ? (size_t)w * (ADMA ? 2 : 1) * half : 0);
  const float2* s_xy = reinterpret_cast<const float2*>(s_w);
  const int64_t* s_act = reinterpret_cast<const int64_t*>(s_w + half);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
  const int nwords = (N + 31) >> 5;
  const int t0 = sl * EPL;
  // one block of GPW instances per wave (the grid covers B: no loop, short live ranges)
  {
    const int64_t base = wid * GPW;
    if (base >= B) return;
    const int64_t r = base + grp;
    const bool valid = r < B;
    const int64_t rr = valid ? r : 0;
    const int64_t* arow = acts + rr * sb;
    if constexpr (DMA) {
      // the previous rows' LDS reads are done before the DMA overwrites them
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      const int rows = (int)(B - base < GPW ? B - base : GPW);
      const int64_t lb = LB == B ? base : base % LB;
      wave_dma<CO_ROWS_AUX>(reinterpret_cast<const unsigned char*>(locs + lb * N), rows * N * 8,
                            s_w);
      if constexpr (ADMA)
        wave_dma<CO_ROWS_AUX>(reinterpret_cast<const unsigned char*>(acts + base * (int64_t)N),
                              rows * N * 8, s_w + half);
    }
    int64_t av[EPL];
    if constexpr (MODE == 3) {  // in flight with the DMA
      if constexpr (CO_ROWS_AV4 && EPL % 2 == 1) {
        // 16-byte pieces (8-byte aligned: gfx950 loads them whole), branch-free and inside
        // the row: pair j starts at p = min(t0 + 2j, N - 2); when clamped, step t0 + 2j is
        // N - 1 (its .y) or past N (masked below like every slot past N)
        typedef long long i64x2a8 __attribute__((ext_vector_type(2), aligned(8)));
#pragma unroll
        for (int k = 0; k + 1 < EPL; k += 2) {
          const int p = t0 + k < N - 2 ? t0 + k : N - 2;
          const i64x2a8 v = *reinterpret_cast<const i64x2a8*>(arow + p);
          av[k] = p == t0 + k ? v.x : v.y;
          av[k + 1] = v.y;
        }
        av[EPL - 1] = arow[t0 + EPL - 1 < N ? t0 + EPL - 1 : N - 1];
      } else {  // slots past N re-read step N-1
#pragma unroll
        for (int k = 0; k < EPL; ++k)
          av[k] = ld_s<CO_ROWS_ANT>(arow + (t0 + k < N ? t0 + k : N - 1));
      }
    }
    if constexpr (DMA) {
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // the lane's EPL actions: 16-byte vectors when the row is 16-byte aligned
    if constexpr (ADMA) {
      // branch-free: slots past N re-read step N-1 (in the staged block); their
      // contributions are masked below
#pragma unroll
      for (int k = 0; k < EPL; ++k) av[k] = s_act[grp * N + (t0 + k < N ? t0 + k : N - 1)];
    } else if constexpr (MODE == 3) {
    } else if constexpr (VEC) {
#pragma unroll
      for (int k = 0; k < EPL; k += 2) {
        if (valid && t0 + k + 1 < N) {
          const longlong2 v = *reinterpret_cast<const longlong2*>(arow + t0 + k);
          av[k] = v.x;
          av[k + 1] = v.y;
        } else {
          av[k] = (valid && t0 + k < N) ? arow[t0 + k] : 0;
          av[k + 1] = 0;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) av[k] = (valid && t0 + k < N) ? arow[t0 + k] : 0;
    }
    for (int j = sl; j < NWB; j += G) bits[j] = 0u;
    uint32_t bad = 0;
    int node[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const uint32_t l32 = (uint32_t)av[k];
      const bool ok = ((uint32_t)(av[k] >> 32) == 0u) & (l32 < (uint32_t)N);
      const bool in = t0 + k < N;
      bad |= (in && !ok) ? 1u : 0u;
      node[k] = ok ? (int)l32 : 0;
    }
    const float2* lrow = DMA ? s_xy + grp * N : locs + (LB == B ? rr : rr % LB) * (int64_t)N;
    float2 p[EPL];
    if constexpr (DMA) {  // node is always a valid LDS index
#pragma unroll
      for (int k = 0; k < EPL; ++k) p[k] = lrow[node[k]];
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        p[k] = (valid && t0 + k < N) ? lrow[node[k]] : make_float2(0.f, 0.f);
    }
    // the zeroed bitmap is visible to the group's other lanes (one wave, in order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < EPL; ++k)  // OR of 0 for slots past N: no branch
      __hip_atomic_fetch_or(&bits[node[k] >> 5],
                            (valid && t0 + k < N) ? 1u << (node[k] & 31) : 0u, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WAVEFRONT);
    // edges: within the lane, to the next lane's first step, and the closing edge; summed
    // in f64 so the f32 tour length does not depend on the summation order (a tour and its
    // reverse get the same reward, as the step-major kernel's f64 accumulation gives)
    double acc = 0.0;
#pragma unroll
    for (int k = 1; k < EPL; ++k) {
      const float dx = p[k].x - p[k - 1].x, dy = p[k].y - p[k - 1].y;
      const float e = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
      acc += t0 + k < N ? (double)e : 0.0;
    }
    const float nx = __shfl_down(p[0].x, 1, G), ny = __shfl_down(p[0].y, 1, G);
    const float fx = __shfl(p[0].x, 0, G), fy = __shfl(p[0].y, 0, G);  // step 0
    const int tl = N - 1 - t0;  // this lane's slot of step N-1 (if 0 <= tl < EPL)
    float lx = p[EPL - 1].x, ly = p[EPL - 1].y;
#pragma unroll
    for (int k = 0; k < EPL - 1; ++k)
      if (k == tl) {
        lx = p[k].x;
        ly = p[k].y;
      }
    {
      // edge (t0 + EPL - 1) -> (t0 + EPL), the next lane's first step; or, on the lane
      // holding step N-1, the closing edge N-1 -> 0 (roll by -1)
      const bool cross = t0 + EPL < N, closing = !cross && tl >= 0 && tl < EPL;
      const float tx = cross ? nx : fx, ty = cross ? ny : fy;
      const float dx = tx - lx, dy = ty - ly;
      const float e = __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
      acc += (cross || closing) ? (double)e : 0.0;
    }
    const float len = (float)grp_sum_f64<G>(acc);
    // visited words: all N bits set <=> the N actions are a permutation (given in range)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int cnt = 0;
    for (int j = sl; j < nwords; j += G) cnt += __popc(bits[j]);
    cnt = (int)grp_reduce<G>((uint32_t)cnt, [](uint32_t x, uint32_t y) { return x + y; });
    bad = grp_reduce<G>(bad, [](uint32_t x, uint32_t y) { return x | y; });
    const bool full = cnt == N;
    if (check && valid && sl == 0 && (bad || !full)) set_status(status, CO_ST_INVALID_TOUR);
    if (!valid) return;
    if constexpr (STATE) {
      // action_mask row: byte c = node c not visited (all zero for a permutation)
      uint8_t* mrow = mask_out + r * (int64_t)N;
      const bool wide = ((reinterpret_cast<uintptr_t>(mrow) | (uintptr_t)N) & 3) == 0;
      if (wide) {
        for (int c4 = sl; c4 < (N >> 2); c4 += G) {
          uint32_t v = 0;
          if (!full) {
            const uint32_t nib = ~(bits[c4 >> 3] >> (4 * (c4 & 7))) & 0xfu;
            v = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
          }
          if (CO_ROWS_NTST)
            __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(mrow + 4 * c4));
          else
            *reinterpret_cast<uint32_t*>(mrow + 4 * c4) = v;
        }
      } else {
        for (int c = sl; c < N; c += G)
          mrow[c] = full ? 0 : (uint8_t)(((bits[c >> 5] >> (c & 31)) & 1u) ^ 1u);
      }
      // row scalars spread over the group's lanes
      const int last_lane = (N - 1) / EPL;
      int lastnode = node[0];
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (k == tl) lastnode = node[k];
      if (sl == 0) {
        first_out[r] = node[0];
        i_out[r] = N;
        reward_out[r] = -(float)len;
      }
      if (sl == last_lane) cur_out[r] = lastnode;
      if (sl == (G > 2 ? 2 : 1) % G) {
        done_out[r] = full;
        step_reward_out[r] = 0;
      }
    } else {
      if (sl == 0) reward_out[r] = -(float)len;
    }
  }
}

#ifndef CO_SLAP_CSWAP
#define CO_SLAP_CSWAP 1  // one-compare comparator (asm selects) in the key sort (r06: -0.5 us)
#endif
#ifndef CO_SLAP_KEY2
#define CO_SLAP_KEY2 1  // distance keys by an add of +0.0 and a sign mask (4 VALU instead of 6;
                        // r06: -0.7 us at B = 65,536)
#endif
#ifndef CO_SLAP_OWNW
#define CO_SLAP_OWNW 0  // the popping lane writes the assignment; free bits cleared after the
                        // loop (r06: 43.4 -> 45.3 us at B = 65,536: off)
#endif
__device__ __forceinline__ uint32_t sel_u32(uint64_t m, uint32_t t, uint32_t f) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
// compare-exchange with one v_cmp_lt_u64 and four selects on its lane mask (written as
// two ternaries the compiler emits a second, `gt`, compare for the max)
__device__ __forceinline__ void cswap_u64(uint64_t& a, uint64_t& b) {
  const uint64_t lt = __builtin_amdgcn_ballot_w64(a < b);
  const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b,
                 bhi = (uint32_t)(b >> 32);
  a = ((uint64_t)sel_u32(lt, ahi, bhi) << 32) | sel_u32(lt, alo, blo);
  b = ((uint64_t)sel_u32(lt, bhi, ahi) << 32) | sel_u32(lt, blo, alo);
}

// ascending sort of EPL u64 keys in registers (Batcher odd-even merge network)
template <int EPL>
__device__ __forceinline__ void sort_keys(uint64_t (&k)[EPL]) {
  static_assert((EPL & (EPL - 1)) == 0, "EPL must be a power of two");
#pragma unroll
  for (int p = 1; p < EPL; p <<= 1)
#pragma unroll
    for (int q = p; q > 0; q >>= 1)
#pragma unroll
      for (int j = q % p; j + q < EPL; j += 2 * q)
#pragma unroll
        for (int i = 0; i < q; ++i)
          if (i + j + q < EPL && (i + j) / (2 * p) == (i + j + q) / (2 * p)) {
#if CO_SLAP_CSWAP
            cswap_u64(k[i + j], k[i + j + q]);
#else
            const uint64_t a = k[i + j], b = k[i + j + q];
            k[i + j] = a < b ? a : b;
            k[i + j + q] = a < b ? b : a;
#endif
          }
}

// ----------------------------------------------------------------------------- SLAP
// SLAP episode (slap/env.py:38-143), G lanes per instance, 256/G instances per
// workgroup.  Lane `sl` keeps locations c = sl + G*k (k < EPL): their depot distance
// and a free bit in VGPRs.  Step t assigns product t (to_choose after reset is
// 0..P-1) to the step's location: the closest-free policy is a DPP min over the
// lanes' sorted candidate heads (ties -> lowest index, torch.argmin on depot_loc_dist
// masked to inf), a
// teacher action is one broadcast load of the step-major action row; python's
// negative-index wrap applies to the mask write and the reward's location lookup
// (the int32 assignment keeps the raw value, slap/env.py:50-62).  The reward then runs
// one lane per order over the LDS-staged assignment row and coordinates: K picks, the
// closed pick tour in f32 in pick order, and the orders added in order by lane 0.
// SLAP reward helpers: a pick's location (python wrap of the int32 assignment; -1 /
// out of range -> flagged, location 0) and the closed tour of one order's KU picks in
// pick order (f32, hardware sqrt: <= 1 ulp per edge, reward parity is 1e-5 relative).
__device__ __forceinline__ float edge_len_hw(float x0, float y0, float x1, float y1) {
  const float dx = x1 - x0, dy = y1 - y0;
  return __builtin_amdgcn_sqrtf(dx * dx + dy * dy);
}
__device__ __forceinline__ int slap_pick_loc(int pp, const int32_t* asg, int L, bool& range) {
  // branch-free (r06): the assignment entry is read at a clamped index and every test is
  // a select; the wave runs one straight-line path per pick
  const bool neg = pp < 0;
  int64_t loc = asg[neg ? 0 : pp];
  loc = loc < 0 ? loc + L : loc;
  const bool bad = neg || loc < 0 || loc >= L;
  range |= bad;
  return bad ? 0 : (int)loc;
}
template <int KU, typename PK>
__device__ __forceinline__ float slap_order_len(const PK* pk, const int32_t* asg,
                                                const float2* xy, int L, bool& range,
                                                int K = KU) {
  int pp[KU], lc[KU];
  float2 q[KU];
#pragma unroll
  for (int k = 0; k < KU; ++k) pp[k] = k < K ? pk[k] : 0;
#pragma unroll
  for (int k = 0; k < KU; ++k) lc[k] = k < K ? slap_pick_loc(pp[k], asg, L, range) : 0;
#pragma unroll
  for (int k = 0; k < KU; ++k) q[k] = xy[lc[k]];
  float len = 0.f;
#pragma unroll
  for (int k = 1; k < KU; ++k)
    if (k < K) len += edge_len_hw(q[k - 1].x, q[k - 1].y, q[k].x, q[k].y);
  float2 ql = q[0];
#pragma unroll
  for (int k = 1; k < KU; ++k) ql = (k == K - 1) ? q[k] : ql;
  return len + edge_len_hw(ql.x, ql.y, q[0].x, q[0].y);
}

__host__ __device__ inline size_t slap_asg_bytes(int ipb, int P) {
  return ((size_t)ipb * P * 4 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t slap_wave_bytes(int gpw, int epl, int L, int O, int K) {
  const size_t keys = (size_t)epl * 64 * 8;
  // coordinates f32x2, order lengths f32, picklist products int16 (P <= 4,096)
  const size_t data = (size_t)gpw * (L * 8 + O * 4 + O * K * 2);
  return ((keys > data ? keys : data) + 15) & ~(size_t)15;
}
// The LDS-DMA staging layout (SD = true): the wave's coordinate rows [GPW][L] land at the
// region's start by DMA and stay there; after them one area holds, in turn, the DMA'd depot
// distances [GPW][L], the sorted keys 2..EPL-1 [EPL-2][64], and after the step loop the
// order lengths [GPW][O] and picklist products [GPW][O*K].
__host__ __device__ inline size_t slap_xy_bytes(int gpw, int L) {
  return ((size_t)gpw * L * 8 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t slap_wave_bytes_sd(int gpw, int epl, int L, int O, int K) {
  size_t area = (size_t)(epl - 2) * 64 * 8;
  const size_t dd = (size_t)gpw * L * 4, tail = (size_t)gpw * (O * 4 + O * K * 2);
  area = area > dd ? area : dd;
  area = area > tail ? area : tail;
  return slap_xy_bytes(gpw, L) + ((area + 15) & ~(size_t)15);
}

#ifndef CO_SLAP_LATE
#define CO_SLAP_LATE 0  // 1: the coordinates, 2: also the picklist loaded after the step loop
#endif

#ifndef CO_SLAP_POP
#define CO_SLAP_POP 0  // 1: branch-free pop in the closest-free step loop (r05: 43.9 against 42.0 us)
#endif

#ifndef CO_SLAP_WPE
#define CO_SLAP_WPE 0  // > 0: amdgpu_waves_per_eu floor (SGPRs cap the kernel at 7 waves)
#endif
#if CO_SLAP_WPE > 0
#define CO_SLAP_ATTR __attribute__((amdgpu_waves_per_eu(CO_SLAP_WPE)))
#else
#define CO_SLAP_ATTR
#endif

#ifndef CO_SLAP_NT
#define CO_SLAP_NT 0  // non-temporal loads / stores (r06: 47 -> 53 us at B = 65,536: partial-line
                      // accesses; nt pays only for whole-line streams such as LDS-DMA)
#endif

#ifndef CO_SLAP_SD
#define CO_SLAP_SD 1  // stage coordinates and depot distances by LDS-DMA (nt) when aligned
                      // (r06: B = 16,384 18.9 -> 17.0 us, 65,536 48.0 -> 45.1 us, A/B)
#endif
#ifndef CO_SLAP_PNT
#define CO_SLAP_PNT 0  // picklist loads non-temporal (r06: 44.8 -> 47.2 us at B = 65,536: off)
#endif

template <int G, int EPL, bool CLOSEST, bool SD>
__global__ __launch_bounds__(256) CO_SLAP_ATTR void slap_group_kernel(
    int64_t B, int L, int P, int O, int K, const float2* __restrict__ locs,
    const int64_t* __restrict__ picklist, const float* __restrict__ depot_dist,
    const int32_t* __restrict__ assign_in, const int64_t* __restrict__ acts_in,
    int64_t* __restrict__ acts_out, uint8_t* __restrict__ mask_out,
    int32_t* __restrict__ assign_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out,
    float* __restrict__ ratio_out, int32_t* status) {
  constexpr int IPB = 256 / G, GPW = 64 / G;
  constexpr bool NT = CO_SLAP_NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // [IPB][P] assignment rows, then one region per wave that holds the sorted candidate
  // keys [EPL][64] during the step loop and, after it (same wave, program order), the
  // coordinates [GPW][L], order lengths [GPW][O] and picklist products [GPW][O*K]
  const int lane = lane_id(), sl = lane % G, g = threadIdx.x / G, gw = lane / G;
  int32_t* s_asg = reinterpret_cast<int32_t*>(smem);
  unsigned char* wreg =
      smem + slap_asg_bytes(IPB, P) +
      (size_t)wave_in_block() * (SD ? slap_wave_bytes_sd(GPW, EPL, L, O, K)
                                    : slap_wave_bytes(GPW, EPL, L, O, K));
  // SD: keys 2..EPL-1 at slots 0..EPL-3 of the area after the coordinates; else slots
  // 2..EPL-1 of the region's start (overwritten by the coordinates after the loop)
  unsigned char* area = wreg + (SD ? slap_xy_bytes(GPW, L) : 0);
  uint64_t* s_keys = reinterpret_cast<uint64_t*>(area) - (SD ? 2 * 64 : 0);
  const int64_t b = (int64_t)blockIdx.x * IPB + g;
  const bool live = b < B;
  const int64_t bb = live ? b : 0;
  float2* xy = reinterpret_cast<float2*>(wreg) + gw * L;
  int32_t* asg = s_asg + g * P;
  unsigned char* obase = SD ? area : wreg + (size_t)GPW * L * 8;
  float* olen = reinterpret_cast<float*>(obase) + gw * O;
  int16_t* pks = reinterpret_cast<int16_t*>(obase + (size_t)GPW * O * 4) + gw * O * K;
  // SD: the wave's GPW depot-distance rows and coordinate rows (contiguous in memory) by
  // LDS-DMA with the non-temporal hint, the distances first: the wait for them (the sort
  // needs them) is the only one before the step loop; the coordinates are waited for after
  // it
  const int64_t wbase = (int64_t)blockIdx.x * IPB + (int64_t)wave_in_block() * GPW;
  const int wrows = (int)(B - wbase < GPW ? (B - wbase > 0 ? B - wbase : 0) : GPW);
  if constexpr (SD) {
    wave_dma<2>(reinterpret_cast<const unsigned char*>(depot_dist + wbase * L), wrows * L * 4,
                area);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  // Loads are issued in the order they are needed: the depot distances (the step loop),
  // then the coordinates and up to G*EPL picklist entries, which stay in registers during
  // the step loop and go to LDS after it, so their latency hides behind the loop.  The
  // initial assignment is not read: the P steps overwrite every entry (product t <- step t).
  float dd[EPL];
  uint32_t avail = 0;  // bit k: location sl + G*k is free (the mask output)
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
    const bool ok = c < L && c != 0;  // the depot is never free (slap/env.py:115-116)
    if (ok) avail |= 1u << k;
    if constexpr (SD)
      dd[k] = (CLOSEST && ok) ? reinterpret_cast<const float*>(area)[gw * L + c] : __builtin_inff();
    else
      dd[k] = (CLOSEST && ok) ? ld_s<NT>(depot_dist + bb * L + c) : __builtin_inff();
  }
  if constexpr (SD) {  // the coordinates stream in behind the sort and the step loop
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the distance reads are back
    wave_dma<2>(reinterpret_cast<const unsigned char*>(locs + wbase * L), wrows * L * 8, wreg);
  }
  // ratio (slap/env.py:114, zeros) depends on nothing: its stores go out first and
  // drain while the loads are in flight
  if (live && ratio_out) {
    float* rrow = ratio_out + bb * L;
    if (((reinterpret_cast<uintptr_t>(ratio_out) | ((uintptr_t)L * 4)) & 15) == 0) {
      // 16-byte stores (r06): 2 store instructions per lane at L = 100 instead of 7
      for (int c4 = sl; c4 < (L >> 2); c4 += G)
        *reinterpret_cast<float4*>(rrow + 4 * c4) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int c = sl; c < L; c += G) st_s<NT>(rrow + c, 0.f);
    }
  }
  const float2* lrow = locs + bb * L;
  const int64_t* prow = picklist + bb * (int64_t)O * K;
  float2 xr[EPL];
  int64_t pr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
#if !CO_SLAP_LATE
    if constexpr (!SD) xr[k] = c < L ? ld_s<NT>(lrow + c) : make_float2(0.f, 0.f);
#endif
#if CO_SLAP_LATE < 2
    pr[k] = c < O * K ? ld_s<NT || CO_SLAP_PNT>(prow + c) : 0;
#endif
  }
  // closest-free = the free locations in increasing (distance, index) order.  Each lane
  // sorts its EPL candidates once (keys: order-preserving u32 of the distance, then the
  // location); a step is then a group min over the lanes' heads and a pop by the owner,
  // instead of an EPL-wide scan + argmin and a slot clear.  A distance that is not below
  // +inf (taken, depot, pad, NaN) is never chosen; with no candidate left the action is 0.
  // picklist entries as wrapped product indices (-1 = out of range), int32 before the
  // step loop so the int64 loads do not stay live through it
  auto wrap_product = [&](int64_t pp) -> int32_t {
    if (pp < 0) pp += P;
    return (pp < 0 || pp >= P) ? -1 : (int32_t)pp;
  };
  int32_t pw[EPL];
#if CO_SLAP_LATE < 2
#pragma unroll
  for (int k = 0; k < EPL; ++k) pw[k] = wrap_product(pr[k]);
#endif
  uint64_t key[EPL];
  if (CLOSEST) {
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
#if CO_SLAP_KEY2
      // -0.0 keyed as +0.0 (d + 0.0 is +0.0 for d = -0.0, d otherwise): they tie as in
      // argmin's float compare, and the index decides
      const uint32_t u = __float_as_uint(dd[k] + 0.0f);
      const uint32_t ord = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
#else
      // -0.0 keyed as +0.0: they tie (argmin's float compare), the index decides
      const uint32_t u = dd[k] == 0.f ? 0u : __float_as_uint(dd[k]);
      const uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
#endif
      key[k] = ((uint64_t)ord << 32) | (uint32_t)(sl + G * k);
    }
    sort_keys<EPL>(key);
  }
#if defined(CO_SLAP_CUT) && CO_SLAP_CUT == 1
  if (live && sl == 0 && (uint32_t)key[0] == 12345u + (uint32_t)pr[0] + (uint32_t)__float_as_uint(xr[0].x))
    reward_out[bb] = 1.f;
  return;
#endif
  constexpr uint32_t kOrdInf = 0xff800000u;  // ordered key of +inf
  bool range = false;
  if (CLOSEST) {
    // The lane's head and next key stay in registers, the rest of its sorted list in
    // LDS; a pop (owner lane only) is two moves and one LDS read that is waited for only
    // at the lane's next pop.  The owner also clears its own free bit (the chosen
    // location gi is slot gi / G of lane gi % G).
    uint64_t hk = key[0], nk = EPL > 1 ? key[1] : ~0ull;
#pragma unroll
    for (int k = 2; k < EPL; ++k) s_keys[k * 64 + lane] = key[k];
    int h = 2;
#if CO_SLAP_POP
    // branch-free pop: every lane reads the key after its `next` each step (issued before
    // the two group reductions, so its latency hides behind them) and the owner's head /
    // next / free bit move by selects -- no divergent branch and exec-mask juggling per step
    for (int t = 0; t < P; ++t) {
      const uint64_t nn = h < EPL ? s_keys[h * 64 + lane] : ~0ull;
      const uint32_t hh = (uint32_t)(hk >> 32);
      const uint32_t gm = grp_reduce<G>(hh, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      const uint32_t cand = hh == gm ? (uint32_t)hk : 0xffffffffu;
      const uint32_t gi =
          grp_reduce<G>(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      const bool any = gm < kOrdInf;
      const bool pop = any && (uint32_t)hk == gi;  // the owner's head is the chosen location
      avail &= pop ? ~(1u << (gi / G)) : ~0u;
      hk = pop ? nk : hk;
      nk = pop ? nn : nk;
      h += pop ? 1 : 0;
      if (sl == 0) asg[t] = any ? (int32_t)gi : 0;  // product t
    }
#else
#if CO_SLAP_OWNW
    // r06: the owner of the chosen location writes assignment[t] in its pop (a step with no
    // candidate leaves the pre-stored 0), and the popped keys' free bits are cleared after
    // the loop from their slots -- 2 VALU and an exec switch fewer per step
    for (int t = sl; t < P; t += G) asg[t] = 0;
    uint32_t slots = 0;  // nibble j: the register slot (location / G) of sorted key j
#pragma unroll
    for (int j = 0; j < EPL && j < 8; ++j) slots |= (((uint32_t)key[j] - sl) / G) << (4 * j);
    __builtin_amdgcn_wave_barrier();  // (one wave: the zeros land before any pop's write)
    for (int t = 0; t < P; ++t) {
      const uint32_t hh = (uint32_t)(hk >> 32);
      const uint32_t gm = grp_reduce<G>(hh, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      const uint32_t cand = hh == gm ? (uint32_t)hk : 0xffffffffu;
      const uint32_t gi =
          grp_reduce<G>(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      if (gm < kOrdInf && (uint32_t)hk == gi) {  // the owner's head is the chosen location
        asg[t] = (int32_t)gi;  // product t
        hk = nk;
        nk = h < EPL ? s_keys[h * 64 + lane] : ~0ull;
        ++h;
      }
    }
#pragma unroll
    for (int j = 0; j < EPL && j < 8; ++j)
      if (j < h - 2) avail &= ~(1u << ((slots >> (4 * j)) & 15u));
#else
    for (int t = 0; t < P; ++t) {
      const uint32_t hh = (uint32_t)(hk >> 32);
      const uint32_t gm = grp_reduce<G>(hh, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      const uint32_t cand = hh == gm ? (uint32_t)hk : 0xffffffffu;
      const uint32_t gi =
          grp_reduce<G>(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      const bool any = gm < kOrdInf;
      if (any && (uint32_t)hk == gi) {  // the owner's head is the chosen location
        avail &= ~(1u << (gi / G));
        hk = nk;
        nk = h < EPL ? s_keys[h * 64 + lane] : ~0ull;
        ++h;
      }
      if (sl == 0) asg[t] = any ? (int32_t)gi : 0;  // product t
    }
#endif
#endif
  } else {
    // teacher actions: lane sl loads steps t = sl, sl + G, ... (all loads in flight at
    // once, a few VGPRs), writes the int32 assignment entry and the wrapped location (-1
    // when out of range) to LDS; after a wave fence every lane scans the P locations for
    // the free bits it owns.  The wrapped locations use the wave's key region (unused by
    // the teacher path); P*GPW ints always fit it for P <= 256.
    int32_t* s_w = reinterpret_cast<int32_t*>(wreg) + gw * P;
    if (P * GPW <= EPL * 128) {
#pragma unroll 4
      for (int t = sl; t < P; t += G) {
        const int64_t a64 = acts_in[(int64_t)t * B + bb];
        asg[t] = (int32_t)a64;  // product t
        const int64_t a = a64 < 0 ? a64 + L : a64;
        const bool bad = a < 0 || a >= L;
        range |= bad;
        s_w[t] = bad ? -1 : (int)a;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int t = 0; t < P; ++t) {
        const int a = s_w[t];
        if (a >= 0 && sl == a % G) avail &= ~(1u << (a / G));
      }
    } else {
      for (int t = 0; t < P; ++t) {
        const int64_t a64 = acts_in[(int64_t)t * B + bb];
        if (sl == 0) asg[t] = (int32_t)a64;  // product t
        const int64_t a = a64 < 0 ? a64 + L : a64;
        if (a < 0 || a >= L) {
          range = true;
        } else if (sl == (int)(a % G)) {
          avail &= ~(1u << (int)(a / G));
        }
      }
    }
  }
#if defined(CO_SLAP_CUT) && CO_SLAP_CUT == 2
  {
    uint32_t sink = avail;
#pragma unroll
    for (int k = 0; k < EPL; ++k)
      sink += (uint32_t)pw[k] + __float_as_uint(xr[k].x) + __float_as_uint(xr[k].y);
    if (live && sink == 12345u) reward_out[bb] = 1.f;
    return;
  }
#endif
  if constexpr (SD) {  // the DMA'd coordinates have landed in place
    __builtin_amdgcn_s_waitcnt(0);
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const int c = sl + G * k;
#if CO_SLAP_LATE
      xr[k] = c < L ? lrow[c] : make_float2(0.f, 0.f);
#endif
      if (c < L) xy[c] = xr[k];
    }
  }
  // picklist entries as wrapped product indices (-1 = out of range)
#if CO_SLAP_LATE >= 2
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
    pw[k] = c < O * K ? wrap_product(prow[c]) : 0;
  }
#endif
#pragma unroll
  for (int k = 0; k < EPL; ++k) {  // entry sl + G*k is register pw[k]
    const int c = sl + G * k;
    if (c < O * K) pks[c] = (int16_t)pw[k];
  }
  for (int c = sl + G * EPL; c < O * K; c += G) pks[c] = (int16_t)wrap_product(ld_s<NT>(prow + c));
  // the group's LDS rows are written and read by lanes of the same wave: a wave-level
  // fence orders them, no workgroup barrier (groups do not wait for other waves)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // closest policy: the step-major action rows of the wave's 64/G instances, written
  // once from the LDS assignment rows (P x 64/G int64 values, 2 store instructions
  // instead of one per step)
  if (CLOSEST) {
    constexpr int IPW = 64 / G;
    const int w0 = wave_in_block() * IPW;  // first group of this wave
    for (int idx = lane; idx < IPW * P; idx += 64) {
      const int t = idx / IPW, gi = idx - t * IPW;
      const int64_t be = (int64_t)blockIdx.x * IPB + w0 + gi;
      if (be < B) st_s<NT>(acts_out + (int64_t)t * B + be, (int64_t)s_asg[(w0 + gi) * P + t]);
    }
  }
  // one lane per order; for K <= 8 the K picks' LDS lookups (product -> location ->
  // coordinates) are three independent batches, not a K-long dependent chain
  for (int o = sl; o < O; o += G) {
    const int16_t* pk = pks + o * K;
    float len = 0.f;
    if (K == 5) {  // examples/slap.py: max_products_in_order = 5
      len = slap_order_len<5>(pk, asg, xy, L, range);
    } else if (K <= 8) {
      len = slap_order_len<8>(pk, asg, xy, L, range, K);
    } else {
      float2 p0 = make_float2(0.f, 0.f), prev = p0;
      for (int k = 0; k < K; ++k) {
        const float2 q = xy[slap_pick_loc(pk[k], asg, L, range)];
        if (k == 0) {
          p0 = q;
        } else {
          len += edge_len_hw(prev.x, prev.y, q.x, q.y);
        }
        prev = q;
      }
      len += edge_len_hw(prev.x, prev.y, p0.x, p0.y);
    }
    olen[o] = len;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

#if defined(CO_SLAP_CUT) && CO_SLAP_CUT == 3
  if (live && sl == 0) reward_out[bb] = olen[0] + (float)avail;
  return;
#endif
  if (live) {
    uint8_t* mrow = mask_out + bb * L;
    if (((reinterpret_cast<uintptr_t>(mask_out) | (uintptr_t)L) & 3) == 0) {
      // r06: the mask bytes go through the group's coordinate slot in LDS (free after the
      // reward) and out as dwords -- 2 store instructions per lane at L = 100, not 8 byte
      // stores
      uint8_t* sm = reinterpret_cast<uint8_t*>(xy);
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        const int c = sl + G * k;
        if (c < L) sm[c] = (uint8_t)((avail >> k) & 1u);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int d = sl; d < (L >> 2); d += G)
        *reinterpret_cast<uint32_t*>(mrow + 4 * d) = *reinterpret_cast<const uint32_t*>(sm + 4 * d);
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        const int c = sl + G * k;
        if (c < L) st_s<NT>(mrow + c, (uint8_t)((avail >> k) & 1u));
      }
    }
    if (((reinterpret_cast<uintptr_t>(assign_out) | ((uintptr_t)P * 4)) & 15) == 0) {
      for (int c4 = sl; c4 < (P >> 2); c4 += G)  // the row as 16-byte pieces
        *reinterpret_cast<int4*>(assign_out + bb * P + 4 * c4) =
            *reinterpret_cast<const int4*>(asg + 4 * c4);
    } else {
      // (not unrolled: the compiler's 16-way unroll of this loop set the kernel's VGPR peak)
#pragma unroll 2
      for (int c = sl; c < P; c += G) st_s<NT>(assign_out + bb * P + c, asg[c]);
    }
    if (sl == 0) {
      // f32 order-by-order accumulation of slap/env.py:135-142 (four lengths per LDS read
      // when the row allows it: the reads no longer wait one by one)
      float total = 0.f;
      int o = 0;
      if ((O & 3) == 0 && (reinterpret_cast<uintptr_t>(olen) & 15) == 0)
        for (; o < O; o += 4) {
          const float4 v = *reinterpret_cast<const float4*>(olen + o);
          total += -v.x;
          total += -v.y;
          total += -v.z;
          total += -v.w;
        }
      for (; o < O; ++o) total += -olen[o];
      reward_out[bb] = total;
      i_out[bb] = P;
      done_out[bb] = 1;  // the P-th step has i == P-1
      step_reward_out[bb] = 0;
    }
  }
  if (__any(range && live) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
}


template <bool STATE>
int launch_tsp_teacher(int64_t B, int64_t N, const float2* l2, int64_t LB, const int64_t* acts,
                       uint8_t* mask_out, int64_t* first_out, int64_t* cur_out, int64_t* i_out,
                       uint8_t* done_out, uint8_t* step_reward_out, float* reward_out, int check,
                       int32_t* status, hipStream_t s) {
  constexpr int Q = CO_TEACH_Q, PRE = CO_TEACH_NB;
  const int NW = NW_launch(N);
  const size_t shmem = tsp_tile_bytes((int)N, Q) + (size_t)64 * (2 * NW + 1) * 4;
  const dim3 grid(cover_grid(B, 64, 64 * Q)), block(64 * Q);
  if (grid.x == 0) return CO_E_INVAL;
  // a wave's step range fits the register prefetch: R = ceil((N - 1) / Q) <= PRE * U
  const bool pre = PRE > 0 && (N - 1 + Q - 1) / Q <= PRE * CO_TEACH_U;
#define CO_TEACH(W, P)                                                                         \
  do {                                                                                         \
    if (shmem > 64 * 1024)                                                                     \
      (void)hipFuncSetAttribute((const void*)tsp_teacher_kernel<W, Q, STATE, P>,               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);       \
    hipLaunchKernelGGL((tsp_teacher_kernel<W, Q, STATE, P>), grid, block, shmem, s, B, (int)N, \
                       l2, LB, acts, mask_out, first_out, cur_out, i_out, done_out,                \
                       step_reward_out, reward_out, check, status);                            \
  } while (0)
  if (NW == 1) {
    if (pre) CO_TEACH(1, PRE);
    else CO_TEACH(1, 0);
  } else if (NW == 2) {
    if (pre) CO_TEACH(2, PRE);
    else CO_TEACH(2, 0);
  } else {
    CO_TEACH(4, 0);
  }
#undef CO_TEACH
  return launch_status();
}

template <bool STATE>
int launch_tsp_rows(int64_t B, int64_t N, const float2* l2, int64_t LB, const int64_t* acts,
                    int64_t sb, uint8_t* mask_out, int64_t* first_out, int64_t* cur_out,
                    int64_t* i_out, uint8_t* done_out, uint8_t* step_reward_out,
                    float* reward_out, int check, int32_t* status, hipStream_t s) {
  const bool vec = ((reinterpret_cast<uintptr_t>(acts) & 15) == 0) && (sb % 2 == 0);
  // LDS-DMA staging: contiguous rows (sb == N), 16-byte aligned blocks (the wave's GPW rows
  // start at a multiple of 32N bytes), the multistart row map not wrapping inside a wave
  const bool dma_ok = CO_ROWS_DMA && sb == N &&
                      ((reinterpret_cast<uintptr_t>(acts) | reinterpret_cast<uintptr_t>(l2)) & 15) == 0;
#define CO_ROWS(GG, EE)                                                                        \
  do {                                                                                         \
    constexpr int WPB = CO_ROWS_WPB;                                                           \
    const dim3 grid(cover_grid((B + 64 / GG - 1) / (64 / GG), WPB, 64 * WPB)), block(64 * WPB); \
    if (grid.x == 0) return CO_E_INVAL;                                                        \
    const size_t dsh = WPB * tsp_rows_wave_bytes(64 / GG, (int)N);                             \
    /* the static visited bitmaps come on top of the dynamic staging (64 KiB default) */       \
    const size_t sbits = (size_t)WPB * (64 / GG) * ((GG * EE + 31) / 32) * 4;                  \
    if (CO_ROWS_MODE3 && dma_ok && (LB == B || LB % (64 / GG) == 0) &&                       \
        dsh / 2 + sbits <= 64 * 1024)                                                          \
      hipLaunchKernelGGL((tsp_teacher_rows_kernel<GG, EE, 3, STATE>), grid, block, dsh / 2, s,  \
                         B, (int)N, l2, LB, acts, sb, mask_out, first_out, cur_out, i_out,     \
                         done_out, step_reward_out, reward_out, check, status);                \
    else if (dma_ok && (LB == B || LB % (64 / GG) == 0) && dsh + sbits <= 64 * 1024)           \
      hipLaunchKernelGGL((tsp_teacher_rows_kernel<GG, EE, 2, STATE>), grid, block, dsh, s, B,   \
                         (int)N, l2, LB, acts, sb, mask_out, first_out, cur_out, i_out,        \
                         done_out, step_reward_out, reward_out, check, status);                \
    else if (vec)                                                                              \
      hipLaunchKernelGGL((tsp_teacher_rows_kernel<GG, EE, 1, STATE>), grid, block, 0, s, B,     \
                         (int)N, l2, LB, acts, sb, mask_out, first_out, cur_out, i_out,        \
                         done_out, step_reward_out, reward_out, check, status);                \
    else                                                                                       \
      hipLaunchKernelGGL((tsp_teacher_rows_kernel<GG, EE, 0, STATE>), grid, block, 0, s, B,     \
                         (int)N, l2, LB, acts, sb, mask_out, first_out, cur_out, i_out,        \
                         done_out, step_reward_out, reward_out, check, status);                \
  } while (0)
  if (N <= 32) CO_ROWS(4, 8);
  else if (N <= 64) CO_ROWS(8, 8);
  else if (N <= 16 * CO_ROWS_EPL112) CO_ROWS(16, CO_ROWS_EPL112);  // TSP-100: 7 steps a lane
  else if (N <= 128) CO_ROWS(16, 8);
  else if (N <= 256) CO_ROWS(32, 8);
  else if (N <= 512) CO_ROWS(64, 8);
  else CO_ROWS(64, 16);
#undef CO_ROWS
  return launch_status();
}

}  // namespace

// Reward + permutation check for row-major actions (element (b, t) at acts[b*sb + t]),
// T == N <= 1024: the row kernel without the state outputs.  Called by co_tsp_reward.
int co_internal_tsp_reward_rows(int64_t B, int64_t N, const float* locs, int64_t locs_batch,
                                const int64_t* acts, int64_t sb, int check, float* reward,
                                int32_t* status, void* stream) {
  if (N > 1024 || sb < N || (reinterpret_cast<uintptr_t>(locs) & 7)) return CO_E_INVAL;
  return launch_tsp_rows<false>(B, N, reinterpret_cast<const float2*>(locs), locs_batch, acts, sb,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, reward,
                                check, status, (hipStream_t)stream);
}

namespace {
// The episode beyond the fused engines' tiles (teacher N > 256: the coordinate tile no
// longer fits the LDS; nearest N > 1024: 64 lanes x 16 registers): the same outputs from
// the stepwise kernels, in place -- co_tsp_reset, then per step [co_tsp_nearest_action
// +] co_tsp_step (mask / i / first_node updated in place, current_node = the action),
// then co_tsp_reward on the step-major actions.  N + 2 (2N + 2) launches, no host sync.
int tsp_rollout_stepwise(int64_t B, int64_t N, const float* locs, const int64_t* acts_in,
                         int64_t* acts_out, uint8_t* mask_out, int64_t* first_out,
                         int64_t* cur_out, int64_t* i_out, uint8_t* done_out,
                         uint8_t* step_reward_out, float* reward_out, int check, int32_t* status,
                         void* stream) {
  // reset's reward[B,1] = 0 goes to reward_out, which the episode reward overwrites
  int rc = co_tsp_reset(B, N, mask_out, first_out, cur_out, i_out, reward_out, stream);
  const bool nearest = acts_in == nullptr;
  const int64_t* acts = nearest ? acts_out : acts_in;
  for (int64_t t = 0; t < N && rc == CO_OK; ++t) {
    if (nearest)
      rc = co_tsp_nearest_action(B, N, locs, mask_out, cur_out, t == 0, acts_out + t * B,
                                 stream);
    if (rc == CO_OK)
      rc = co_tsp_step(B, N, acts + t * B, mask_out, mask_out, i_out, i_out, first_out,
                       first_out, cur_out, done_out, step_reward_out, t == 0 ? 1 : 0, nullptr,
                       status, stream);
  }
  if (rc != CO_OK) return rc;
  return co_tsp_reward(B, N, N, locs, B, acts, 1, B, check, reward_out, status, stream);
}
}  // namespace

extern "C" int co_tsp_rollout_ex(int64_t B, int64_t N, const float* locs,
                                 const int64_t* acts_in, int64_t sb, int64_t st,
                                 int64_t* acts_out, uint8_t* mask_out, int64_t* first_out,
                                 int64_t* cur_out, int64_t* i_out, uint8_t* done_out,
                                 uint8_t* step_reward_out, float* reward_out, int check,
                                 int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > (1 << 24)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  const bool nearest = acts_in == nullptr;
  if (!locs || !mask_out || !first_out || !cur_out || !i_out || !done_out || !step_reward_out ||
      !reward_out || (nearest && !acts_out) || (check && !status))
    return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  if (!nearest && !(sb == 1 && st == B)) {
    // row-major teacher actions (the reference's [B, T]): one lane group per instance
    if (st != 1 || sb < N || N > 1024) return CO_E_INVAL;
    return launch_tsp_rows<true>(B, N, reinterpret_cast<const float2*>(locs), B, acts_in, sb,
                                 mask_out, first_out, cur_out, i_out, done_out, step_reward_out,
                                 reward_out, check, status, (hipStream_t)stream);
  }
  if (N > (nearest ? 1024 : 256))
    return tsp_rollout_stepwise(B, N, locs, acts_in, acts_out, mask_out, first_out, cur_out,
                                i_out, done_out, step_reward_out, reward_out, check, status,
                                stream);
  if (nearest)  // register-resident lane-group episode (nearest.hip)
    return co_internal_tsp_nearest_rollout(B, N, locs, acts_out, mask_out, first_out, cur_out,
                                           i_out, done_out, step_reward_out, reward_out, stream);
  if (reinterpret_cast<uintptr_t>(locs) & 15) return CO_E_ALIGN;  // LDS-DMA staging
  return launch_tsp_teacher<true>(B, N, reinterpret_cast<const float2*>(locs), B, acts_in,
                                  mask_out,
                                  first_out, cur_out, i_out, done_out, step_reward_out,
                                  reward_out, check, status, (hipStream_t)stream);
}

extern "C" int co_tsp_rollout(int64_t B, int64_t N, const float* locs, const int64_t* acts_in,
                              int64_t* acts_out, uint8_t* mask_out, int64_t* first_out,
                              int64_t* cur_out, int64_t* i_out, uint8_t* done_out,
                              uint8_t* step_reward_out, float* reward_out, int check,
                              int32_t* status, void* stream) {
  return co_tsp_rollout_ex(B, N, locs, acts_in, 1, B, acts_out, mask_out, first_out, cur_out,
                           i_out, done_out, step_reward_out, reward_out, check, status, stream);
}

// Reward + permutation check for step-major actions (element (b, t) at acts[t*st + b]),
// T == N: the teacher episode without the state outputs.  Called by co_tsp_reward when
// the actions come from the stepwise engine.
int co_internal_tsp_reward_stepmajor(int64_t B, int64_t N, const float* locs,
                                     int64_t locs_batch, const int64_t* acts, int64_t st,
                                     int check, float* reward, int32_t* status, void* stream) {
  if (st != B || N > 256 || (reinterpret_cast<uintptr_t>(locs) & 15)) return CO_E_INVAL;
  if (locs_batch != B && locs_batch % 64 != 0) return CO_E_INVAL;
  return launch_tsp_teacher<false>(B, N, reinterpret_cast<const float2*>(locs), locs_batch, acts,
                                   nullptr,
                                   nullptr, nullptr, nullptr, nullptr, nullptr, reward, check,
                                   status, (hipStream_t)stream);
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
  // G lanes x 8 locations per instance (16 lanes measured best for L = 100 on MI355X:
  // 8 lanes 33 us, 32 lanes 38 us, at B = 16,384)
  const int G = L <= 64 ? 8 : (L <= 128 ? 16 : 32);
  const int ipb = 256 / G;
  // LDS-DMA staging of the distance / coordinate rows: 16-byte aligned row blocks
  const bool sd = CO_SLAP_SD && closest && (L % 4) == 0 &&
                  ((reinterpret_cast<uintptr_t>(locs) | reinterpret_cast<uintptr_t>(depot_dist)) &
                   15) == 0;
  const size_t shmem =
      slap_asg_bytes(ipb, (int)P) +
      4 * (sd ? slap_wave_bytes_sd(64 / G, 8, (int)L, (int)O, (int)K)
              : slap_wave_bytes(64 / G, 8, (int)L, (int)O, (int)K));
  if (shmem > 160 * 1024) return CO_E_INVAL;
  const dim3 grid(cover_grid(B, ipb)), block(256);
  if (grid.x == 0) return CO_E_INVAL;
  hipStream_t s = (hipStream_t)stream;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
#define CO_SLAP(GG, EPL, C, SDD)                                                               \
  do {                                                                                         \
    if (shmem > 64 * 1024)                                                                     \
      (void)hipFuncSetAttribute((const void*)slap_group_kernel<GG, EPL, C, SDD>,               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);       \
    hipLaunchKernelGGL((slap_group_kernel<GG, EPL, C, SDD>), grid, block, shmem, s, B, (int)L, \
                       (int)P, (int)O, (int)K, l2, picklist, depot_dist, assign_in, acts_in,   \
                       acts_out, mask_out, assign_out, i_out, done_out, step_reward_out,       \
                       reward_out, ratio_out, status);                                         \
  } while (0)
#define CO_SLAP_G(C, SDD)                                       \
  if (G == 8) CO_SLAP(8, 8, C, SDD);                            \
  else if (G == 16) CO_SLAP(16, 8, C, SDD);                     \
  else CO_SLAP(32, 8, C, SDD)
  if (closest && sd) {
    CO_SLAP_G(true, true);
  } else if (closest) {
    CO_SLAP_G(true, false);
  } else {
    CO_SLAP_G(false, false);
  }
#undef CO_SLAP_G
#undef CO_SLAP
  return launch_status();
}
