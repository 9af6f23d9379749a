// TSP env kernels for gfx950: reset, step (mask scatter + done), episode reward,
// and the nearest-unvisited bench policy.
//
// Step layout: one 256-thread workgroup owns a tile of 64 consecutive instances.
// The tile's action_mask bytes (64*N, always a multiple of 16) are streamed with
// 16-byte coalesced loads/stores; each thread clears the byte of its chunk that
// matches its row's action and counts surviving bytes into a per-row LDS counter
// (done = count == 0).  Row scalars (action, i, first_node, ...) are read/written
// coalesced by the first 64 threads.
//
// Reward layout: one wavefront per instance (grid-stride); lanes walk the tour,
// gather both edge endpoints (L1/L2-resident row), accumulate edge lengths in
// f64 and wave-reduce; the permutation check uses a per-wave LDS bitmap.
#include "co_common.hpp"
#include "co_tile.hpp"

using namespace co;

namespace {

__global__ __launch_bounds__(256) void tsp_reset_kernel(int64_t B, int64_t N, uint8_t* mask,
                                                        int64_t* first, int64_t* cur,
                                                        int64_t* it, float* reward) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nbytes = B * N;
  // 16-byte fill of the mask (the tail is byte-filled).
  const int64_t nvec = nbytes >> 4;
  uint4 ones = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
  for (int64_t k = t0; k < nvec; k += stride) reinterpret_cast<uint4*>(mask)[k] = ones;
  for (int64_t k = (nvec << 4) + t0; k < nbytes; k += stride) mask[k] = 1;
  for (int64_t b = t0; b < B; b += stride) {
    first[b] = 0;
    cur[b] = 0;
    it[b] = 0;
    reward[b] = 0.f;
  }
}

struct TspRowEpilogue {
  const int64_t* i_in;
  int64_t* i_out;
  const int64_t* first_in;
  int64_t* first_out;
  int64_t* cur_out;
  uint8_t* done;
  uint8_t* reward;
  int take_first;
  struct Row {
    int64_t i, first;
  };
  __device__ Row load(int64_t b) const { return {i_in[b], take_first ? 0 : first_in[b]}; }
  __device__ void store(int64_t b, int64_t action, int remaining, const Row& r) const {
    first_out[b] = take_first ? action : r.first;
    i_out[b] = r.i + 1;
    if (cur_out) cur_out[b] = action;
    done[b] = remaining == 0;
    reward[b] = 0;
  }
};

__global__ __launch_bounds__(256) void tsp_step_kernel(int64_t B, int N, const int64_t* action,
                                                       const uint8_t* mask_in, uint8_t* mask_out,
                                                       TspRowEpilogue epi, int first_mode,
                                                       const int32_t* first_flag, int32_t* status,
                                                       int vec) {
  if (first_mode == 2) epi.take_first = (*first_flag != 0);
  mask_clear_tile<true>(B, N, action, mask_in, mask_out, status, vec != 0, epi);
}

// Lane-group step for rows of N % 4 == 0 bytes: G lanes per row, lane sl owns the
// 4 mask words [4*sl, 4*sl + 4) of its row (u32 loads/stores); the action's byte is
// cleared with a word select, the surviving entries are counted per word, done is a
// group ballot, and the group's lane 0 writes the row scalars.  64/G rows per wave.
#ifndef CO_TSP_STEP_GROUP
#define CO_TSP_STEP_GROUP 1
#endif

#ifndef CO_TSP_WPL
#define CO_TSP_WPL 4
#endif
#ifndef CO_TSP_LAYOUT
#define CO_TSP_LAYOUT 1
#endif
#ifndef CO_TSP_SCUT
#define CO_TSP_SCUT 0  // timing diagnostic only: 1 no row epilogue, 2 no mask store
#endif

#ifndef CO_TSP_NT
#define CO_TSP_NT 0  // variants: 1 mask words, 2 row scalars stored, 4 mask words loaded non-temporal
#endif
#ifndef CO_TSP_UNR
#define CO_TSP_UNR 1  // row groups per wave (all their loads issued before the first use)
#endif

template <int G>
__global__ __launch_bounds__(256) void tsp_step_group_kernel(int64_t B, int N,
                                                             const int64_t* __restrict__ action,
                                                             const uint32_t* __restrict__ mask_in,
                                                             uint32_t* __restrict__ mask_out,
                                                             TspRowEpilogue epi, int first_mode,
                                                             const int32_t* first_flag,
                                                             int32_t* status) {
  constexpr int WPL = CO_TSP_WPL, U = CO_TSP_UNR;
  const int lane = lane_id(), sl = lane % G, gbase = lane - sl;
  const int W = N >> 2;  // words per row
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
  if (first_mode == 2) epi.take_first = (*first_flag != 0);
  // U row groups per wave (the grid covers B; no grid-stride loop)
  const int64_t base = wid * (64 / G) * U;
  if (base >= B) return;  // wave-uniform
  int64_t rr[U], a_raw[U], rs[U];
  bool valid[U];
  uint32_t w[U][WPL];
  typename TspRowEpilogue::Row rv[U];
  // CO_TSP_LAYOUT 1: word c = sl + k*G (each load/store instruction covers G consecutive
  // words of a row); 0: c = sl*WPL + k (a lane's words adjacent)
#define CO_TSP_WORD(k) (CO_TSP_LAYOUT ? sl + (k) * G : sl * WPL + (k))
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t b = base + u * (64 / G) + lane / G;
    valid[u] = b < B;
    const int64_t r = rr[u] = valid[u] ? b : 0;
    a_raw[u] = action[r];
    // row scalars: with G >= 8 spread over the group's lanes (lane 0 reads i, lane 1
    // first_node: one load instruction; lanes 0-2 write i / first / current: one 8-B
    // store; lanes 3, 4 done / reward: one byte store), else lane 0 does all of them
    rv[u] = {};
    rs[u] = 0;
    if constexpr (G >= 8) {
      const int64_t* rsrc = sl == 0 ? epi.i_in : epi.first_in;
      if (valid[u] && (sl == 0 || (sl == 1 && !epi.take_first)) && !(CO_TSP_SCUT & 1))
        rs[u] = rsrc[r];
    } else if (valid[u] && !(CO_TSP_SCUT & 1)) {
      rv[u] = epi.load(r);
    }
    const uint32_t* src = mask_in + r * W;
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int c = CO_TSP_WORD(k);
      w[u][k] = (valid[u] && c < W)
                    ? ((CO_TSP_NT & 4) ? __builtin_nontemporal_load(src + c) : src[c])
                    : 0u;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = rr[u];
    int64_t a = a_raw[u];
    if (a < 0 || a >= N) {
      if (valid[u] && sl == 0) set_status(status, CO_ST_INDEX_RANGE);
      a = -1;
    }
    const int aw = a >= 0 ? (int)(a >> 2) : -1;  // the action's word and byte
    const uint32_t aclr = 0xffu << (8 * (int)(a & 3));
    int left = 0;
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const uint32_t clr = CO_TSP_WORD(k) == aw ? aclr : 0u;
      w[u][k] &= ~clr;
      // nonzero bytes of the word: high bit of each byte of (b & 0x7f) + 0x7f, or b
      const uint32_t nz = (((w[u][k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w[u][k]) & 0x80808080u;
      left += __builtin_popcount(nz);
    }
    uint32_t* dst = mask_out + r * W;
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int c = CO_TSP_WORD(k);
      if (valid[u] && c < W && !(CO_TSP_SCUT & 2)) {
        if (CO_TSP_NT & 1) __builtin_nontemporal_store(w[u][k], dst + c);
        else dst[c] = w[u][k];
      }
    }
    const bool any_left = (__ballot(left != 0) & gmask) != 0;
    if constexpr (G >= 8) {
      if (valid[u] && !(CO_TSP_SCUT & 1)) {
        int64_t* d8 = sl == 0 ? epi.i_out : sl == 1 ? epi.first_out : epi.cur_out;
        const int64_t v8 = sl == 0 ? rs[u] + 1 : (sl == 1 && !epi.take_first) ? rs[u] : a_raw[u];
        if (sl < 3 && d8) {
          if (CO_TSP_NT & 2) __builtin_nontemporal_store(v8, d8 + r);
          else d8[r] = v8;
        }
        if (sl == 3 || sl == 4) (sl == 3 ? epi.done : epi.reward)[r] = sl == 3 ? !any_left : 0;
      }
    } else if (valid[u] && sl == 0 && !(CO_TSP_SCUT & 1)) {
      epi.store(r, a_raw[u], any_left ? 1 : 0, rv[u]);
    }
  }
#undef CO_TSP_WORD
}

// K consecutive env steps in one launch (co_tsp_steps, round 6): exactly K co_tsp_step
// calls whose state ping-pongs between the buffers A and B (step k reads A for even k, B
// for odd k, and writes the other), every step's mask row, i, first node, current node,
// done and reward stored as that step's launch would store them.  The row's state is
// loaded once, then carried in registers from step to step (each step still writes its
// whole state).  G lanes per row, the group kernel's word layout (word c = sl + k*G,
// WPL words per lane); the K actions of the row are loaded up front (KB per batch).
template <int G>
__global__ __launch_bounds__(256) void tsp_steps_group_kernel(
    int64_t B, int N, int K, const int64_t* __restrict__ action, int64_t astride,
    uint32_t* __restrict__ mask_a, int64_t* __restrict__ i_a, int64_t* __restrict__ first_a,
    uint32_t* __restrict__ mask_b, int64_t* __restrict__ i_b, int64_t* __restrict__ first_b,
    int64_t* __restrict__ cur_out, uint8_t* __restrict__ done, uint8_t* __restrict__ reward,
    int first_mode, int32_t* status) {
  constexpr int WPL = CO_TSP_WPL, KB = 8;
  const int lane = lane_id(), sl = lane % G, gbase = lane - sl;
  const int W = N >> 2;
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
  const int64_t b0 = wid * (64 / G);
  if (b0 >= B) return;  // wave-uniform
  const int64_t bq = b0 + lane / G;
  const bool valid = bq < B;
  const int64_t r = valid ? bq : 0;
  uint32_t w[WPL];
#pragma unroll
  for (int k = 0; k < WPL; ++k) {
    const int c = sl + k * G;
    w[k] = (valid && c < W) ? mask_a[r * W + c] : 0u;
  }
  int64_t iv = valid ? i_a[r] : 0;
  int64_t fv = (valid && first_mode != 1) ? first_a[r] : 0;
  bool range = false;
  for (int t0 = 0; t0 < K; t0 += KB) {
    int64_t av[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u)
      av[u] = (valid && t0 + u < K) ? action[(int64_t)(t0 + u) * astride + r] : 0;
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int t = t0 + u;
      if (t >= K) break;  // wave-uniform
      const int64_t a_raw = av[u];
      int64_t a = a_raw;
      if (a < 0 || a >= N) {
        range |= valid;
        a = -1;
      }
      const int aw = a >= 0 ? (int)(a >> 2) : -1;
      const uint32_t aclr = 0xffu << (8 * (int)(a & 3));
      int left = 0;
#pragma unroll
      for (int k = 0; k < WPL; ++k) {
        const uint32_t clr = sl + k * G == aw ? aclr : 0u;
        w[k] &= ~clr;
        const uint32_t nz = (((w[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w[k]) & 0x80808080u;
        left += __builtin_popcount(nz);
      }
      const bool to_b = (t & 1) == 0;  // step t writes B when it read A
      uint32_t* mdst = (to_b ? mask_b : mask_a) + r * W;
#pragma unroll
      for (int k = 0; k < WPL; ++k) {
        const int c = sl + k * G;
        if (valid && c < W) mdst[c] = w[k];
      }
      const bool any_left = (__ballot(left != 0) & gmask) != 0;
      iv += 1;
      if (t == 0 && first_mode == 1) fv = a_raw;
      if (valid) {
        if (sl == 0) (to_b ? i_b : i_a)[r] = iv;
        else if (sl == 1) (to_b ? first_b : first_a)[r] = fv;
        else if (sl == 2 && cur_out) cur_out[r] = a_raw;
        else if (sl == 3) done[r] = !any_left;
        else if (sl == 4 % G) reward[r] = 0;
      }
    }
  }
  if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void tsp_reward_kernel(int64_t B, int N, int T,
                                                                const float2* locs, int64_t LB,
                                                                const int64_t* actions,
                                                                int64_t sb, int64_t st, int check,
                                                                float* reward, int32_t* status) {
  extern __shared__ uint32_t s_bits[];
  const int w = wave_in_block(), lane = lane_id();
  const int words = (T + 31) >> 5;
  uint32_t* bits = s_bits + w * words;
  for (int64_t b = (int64_t)blockIdx.x * WAVES + w; b < B; b += (int64_t)gridDim.x * WAVES) {
    if (check) {
      for (int k = lane; k < words; k += 64) bits[k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const int64_t* arow = actions + b * sb;
    const float2* lrow = locs + (LB == B ? b : b % LB) * (int64_t)N;  // multistart: e % B
    double acc = 0.0;
    bool bad = false, range = false;
    for (int t = lane; t < T; t += 64) {
      const int64_t a = arow[(int64_t)t * st];
      const int64_t an = arow[(int64_t)((t + 1 == T) ? 0 : t + 1) * st];
      if (check) {
        if (a < 0 || a >= T) {
          bad = true;
        } else {
          const uint32_t bit = 1u << (a & 31);
          if (atomicOr(&bits[a >> 5], bit) & bit) bad = true;
        }
      }
      if (a < 0 || a >= N || an < 0 || an >= N) {
        range = true;
        continue;
      }
      const float2 p = lrow[a], q = lrow[an];
      acc += (double)edge_len(p.x, p.y, q.x, q.y);
    }
    acc = wave_sum(acc);
    if (__any(bad) && lane == 0) set_status(status, CO_ST_INVALID_TOUR);
    if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    if (lane == 0) reward[b] = -(float)acc;
  }
}

// Bench policy: nearest unvisited node to current_node; step 0 -> node 0.
__global__ __launch_bounds__(256) void tsp_nearest_kernel(int64_t B, int N, const float2* locs,
                                                          const uint8_t* mask, const int64_t* cur,
                                                          int first_step, int64_t* out) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    if (first_step) {
      if (lane == 0) out[b] = 0;
      continue;
    }
    const float2* lrow = locs + b * (int64_t)N;
    const uint8_t* mrow = mask + b * (int64_t)N;
    int64_t c0 = cur[b];
    c0 = (c0 < 0 || c0 >= N) ? 0 : c0;
    const float2 p = lrow[c0];
    float best = __builtin_inff();
    int bi = 0x7fffffff;
    for (int c = lane; c < N; c += 64) {
      float d = __builtin_inff();
      if (mrow[c]) {
        const float2 q = lrow[c];
        d = edge_len(p.x, p.y, q.x, q.y);
      }
      if (d < best || (d == best && c < bi)) { best = d; bi = c; }
    }
    wave_argmin(best, bi);
    if (lane == 0) out[b] = bi;
  }
}

}  // namespace

extern "C" int co_tsp_reset(int64_t B, int64_t N, uint8_t* mask, int64_t* first, int64_t* cur,
                            int64_t* it, float* reward, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!mask || !first || !cur || !it || !reward) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(mask) & 15) return CO_E_ALIGN;
  hipLaunchKernelGGL(tsp_reset_kernel, dim3(grid_for(B * N / 16 + B, 256)), dim3(256), 0,
                     (hipStream_t)stream, B, N, mask, first, cur, it, reward);
  return launch_status();
}

extern "C" int co_tsp_step(int64_t B, int64_t N, const int64_t* action, const uint8_t* mask_in,
                           uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                           const int64_t* first_in, int64_t* first_out, int64_t* current_out,
                           uint8_t* done, uint8_t* reward, int first_mode,
                           const int32_t* first_flag, int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > (1 << 30)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !mask_in || !mask_out || !i_in || !i_out || !first_out || !done || !reward)
    return CO_E_INVAL;
  if (first_mode < 0 || first_mode > 2) return CO_E_MODE;
  if (first_mode != 1 && !first_in) return CO_E_INVAL;
  if (first_mode == 2 && !first_flag) return CO_E_INVAL;
  const int vec = tile_vec_ok(mask_in, mask_out);
  TspRowEpilogue epi{i_in, i_out, first_in, first_out, current_out, done, reward,
                     first_mode == 1};
  if (CO_TSP_STEP_GROUP && (N & 3) == 0 && (N >> 2) <= 64 * CO_TSP_WPL &&
      ((reinterpret_cast<uintptr_t>(mask_in) | reinterpret_cast<uintptr_t>(mask_out)) & 3) == 0) {
    const int W = (int)(N >> 2), WG = (W + CO_TSP_WPL - 1) / CO_TSP_WPL;
    const int G = WG <= 2 ? 2 : WG <= 4 ? 4 : WG <= 8 ? 8 : WG <= 16 ? 16 : WG <= 32 ? 32 : 64;
    const int64_t waves = (B * G + 64 * CO_TSP_UNR - 1) / (64 * CO_TSP_UNR);
    const dim3 grid(cover_grid(waves, 4));  // a wave per CO_TSP_UNR row groups
    if (grid.x == 0) return CO_E_INVAL;
    const uint32_t* mi = reinterpret_cast<const uint32_t*>(mask_in);
    uint32_t* mo = reinterpret_cast<uint32_t*>(mask_out);
    hipStream_t s = (hipStream_t)stream;
#define CO_TSG(GG)                                                                             \
  hipLaunchKernelGGL(tsp_step_group_kernel<GG>, grid, dim3(256), 0, s, B, (int)N, action, mi,  \
                     mo, epi, first_mode, first_flag, status)
    if (G == 2) CO_TSG(2);
    else if (G == 4) CO_TSG(4);
    else if (G == 8) CO_TSG(8);
    else if (G == 16) CO_TSG(16);
    else if (G == 32) CO_TSG(32);
    else CO_TSG(64);
#undef CO_TSG
    return launch_status();
  }
  const unsigned grid = cover_grid(B, kTileRows, kTileThreads);
  if (grid == 0) return CO_E_INVAL;
  hipLaunchKernelGGL(tsp_step_kernel, dim3(grid), dim3(kTileThreads), 0, (hipStream_t)stream, B,
                     (int)N, action, mask_in, mask_out, epi, first_mode, first_flag, status, vec);
  return launch_status();
}

extern "C" int co_tsp_steps(int64_t B, int64_t N, int64_t K, const int64_t* action,
                            int64_t astride, uint8_t* mask_a, int64_t* i_a, int64_t* first_a,
                            uint8_t* mask_b, int64_t* i_b, int64_t* first_b,
                            int64_t* current_out, uint8_t* done, uint8_t* reward,
                            int first_mode, int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > (1 << 30) || K < 0 || K > (1 << 20)) return CO_E_INVAL;
  if (B == 0 || K == 0) return CO_OK;
  if (first_mode < 0 || first_mode > 1) return CO_E_MODE;
  if (!action || astride < B || !mask_a || !i_a || !mask_b || !i_b || !first_b || !done ||
      !reward || !status || (first_mode == 0 && !first_a) || (K > 1 && !first_a))
    return CO_E_INVAL;
  const int W = (int)(N >> 2), WG = (W + CO_TSP_WPL - 1) / CO_TSP_WPL;
  const bool group = (N & 3) == 0 && W <= 64 * CO_TSP_WPL && WG >= 5 &&
                     ((reinterpret_cast<uintptr_t>(mask_a) | reinterpret_cast<uintptr_t>(mask_b)) &
                      3) == 0;
  if (!group) {  // the K single steps (rows the group kernel does not take)
    for (int64_t t = 0; t < K; ++t) {
      const bool even = (t & 1) == 0;
      const int rc = co_tsp_step(B, N, action + t * astride, even ? mask_a : mask_b,
                                 even ? mask_b : mask_a, even ? i_a : i_b, even ? i_b : i_a,
                                 even ? first_a : first_b, even ? first_b : first_a,
                                 current_out, done, reward, t == 0 ? first_mode : 0, nullptr,
                                 status, stream);
      if (rc != CO_OK) return rc;
    }
    return CO_OK;
  }
  // G >= 8: the row scalars go out from lanes 0-4 of the group
  const int G = WG <= 8 ? 8 : WG <= 16 ? 16 : WG <= 32 ? 32 : 64;
  const int64_t waves = (B * G + 63) / 64;
  const dim3 grid(cover_grid(waves, 4));
  if (grid.x == 0) return CO_E_INVAL;
  uint32_t* ma = reinterpret_cast<uint32_t*>(mask_a);
  uint32_t* mb = reinterpret_cast<uint32_t*>(mask_b);
  hipStream_t s = (hipStream_t)stream;
#define CO_TSK(GG)                                                                             \
  hipLaunchKernelGGL(tsp_steps_group_kernel<GG>, grid, dim3(256), 0, s, B, (int)N, (int)K,     \
                     action, astride, ma, i_a, first_a, mb, i_b, first_b, current_out, done,  \
                     reward, first_mode, status)
  if (G == 8) CO_TSK(8);
  else if (G == 16) CO_TSK(16);
  else if (G == 32) CO_TSK(32);
  else CO_TSK(64);
#undef CO_TSK
  return launch_status();
}

extern "C" int co_tsp_reward(int64_t B, int64_t N, int64_t T, const float* locs,
                             int64_t locs_batch, const int64_t* actions, int64_t sb, int64_t st,
                             int check, float* reward, int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || T <= 0 || T > (1 << 24)) return CO_E_INVAL;
  if (locs_batch <= 0 || (B > 0 && B % locs_batch != 0)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !actions || !reward || (check && !status)) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  // step-major actions ([T, B], the stepwise engine's layout): thread per instance,
  // coalesced [B]-row loads, LDS-staged coordinates (rollout.hip)
  if (sb == 1 && st == B && T == N && N <= 256 && B > 1 &&
      (locs_batch == B || locs_batch % 64 == 0) && (reinterpret_cast<uintptr_t>(locs) & 15) == 0)
    return co_internal_tsp_reward_stepmajor(B, N, locs, locs_batch, actions, st, check, reward,
                                            status, stream);
  // row-major actions ([B, T], the reference's layout), T == N: lane group per instance,
  // contiguous rows (rollout.hip)
  if (st == 1 && sb >= T && T == N && N <= 1024 &&
      (locs_batch == B || B % locs_batch == 0))
    return co_internal_tsp_reward_rows(B, N, locs, locs_batch, actions, sb, check, reward,
                                       status, stream);
  const size_t words = (size_t)((T + 31) / 32);
  constexpr int W = 4;
  const size_t shmem = check ? W * words * sizeof(uint32_t) : 0;
  if (shmem > 64 * 1024) return CO_E_INVAL;
  hipLaunchKernelGGL(tsp_reward_kernel<W>, dim3(grid_for(B, W, 256 * 32)), dim3(W * 64), shmem,
                     (hipStream_t)stream, B, (int)N, (int)T,
                     reinterpret_cast<const float2*>(locs), locs_batch, actions, sb, st, check,
                     reward, status);
  return launch_status();
}

extern "C" int co_tsp_nearest_action(int64_t B, int64_t N, const float* locs,
                                     const uint8_t* mask, const int64_t* cur, int first_step,
                                     int64_t* out, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!out || (!first_step && (!locs || !mask || !cur))) return CO_E_INVAL;
  hipLaunchKernelGGL(tsp_nearest_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, reinterpret_cast<const float2*>(locs), mask,
                     cur, first_step, out);
  return launch_status();
}
