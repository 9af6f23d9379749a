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

#ifndef CO_TSP_FLAT_ROWS
#define CO_TSP_FLAT_ROWS 0  // rows per wave of the flat step kernel (0: the lane-group kernel)
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

template <int G>
__global__ __launch_bounds__(256) void tsp_step_group_kernel(int64_t B, int N,
                                                             const int64_t* __restrict__ action,
                                                             const uint32_t* __restrict__ mask_in,
                                                             uint32_t* __restrict__ mask_out,
                                                             TspRowEpilogue epi, int first_mode,
                                                             const int32_t* first_flag,
                                                             int32_t* status) {
  constexpr int WPL = CO_TSP_WPL;
  const int lane = lane_id(), sl = lane % G, gbase = lane - sl;
  const int W = N >> 2;  // words per row
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
  if (first_mode == 2) epi.take_first = (*first_flag != 0);
  // one row group per wave (the grid covers B; no grid-stride loop)
  const int64_t base = wid * (64 / G);
  if (base >= B) return;  // wave-uniform
  {
    const int64_t b = base + lane / G;
    const bool valid = b < B;
    const int64_t r = valid ? b : 0;
    const int64_t a_raw = action[r];
    int64_t a = a_raw;
    // row scalars: with G >= 8 spread over the group's lanes (lane 0 reads i, lane 1
    // first_node: one load instruction; lanes 0-2 write i / first / current: one 8-B
    // store; lanes 3, 4 done / reward: one byte store), else lane 0 does all of them
    typename TspRowEpilogue::Row rv{};
    int64_t rs = 0;
    if constexpr (G >= 8) {
      const int64_t* rsrc = sl == 0 ? epi.i_in : epi.first_in;
      if (valid && (sl == 0 || (sl == 1 && !epi.take_first)) && !(CO_TSP_SCUT & 1)) rs = rsrc[r];
    } else if (valid && !(CO_TSP_SCUT & 1)) {
      rv = epi.load(r);
    }
    const uint32_t* src = mask_in + r * W;
    uint32_t w[WPL];
    // CO_TSP_LAYOUT 1: word c = sl + k*G (each load/store instruction covers G consecutive
    // words of a row); 0: c = sl*WPL + k (a lane's words adjacent)
#define CO_TSP_WORD(k) (CO_TSP_LAYOUT ? sl + (k) * G : sl * WPL + (k))
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int c = CO_TSP_WORD(k);
      w[k] = (valid && c < W) ? src[c] : 0u;
    }
    if (a < 0 || a >= N) {
      if (valid && sl == 0) set_status(status, CO_ST_INDEX_RANGE);
      a = -1;
    }
    const int aw = a >= 0 ? (int)(a >> 2) : -1;  // the action's word and byte
    const uint32_t aclr = 0xffu << (8 * (int)(a & 3));
    int left = 0;
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const uint32_t clr = CO_TSP_WORD(k) == aw ? aclr : 0u;
      w[k] &= ~clr;
      // nonzero bytes of the word: high bit of each byte of (b & 0x7f) + 0x7f, or b
      const uint32_t nz = (((w[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w[k]) & 0x80808080u;
      left += __builtin_popcount(nz);
    }
    uint32_t* dst = mask_out + r * W;
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
      const int c = CO_TSP_WORD(k);
      if (valid && c < W && !(CO_TSP_SCUT & 2)) dst[c] = w[k];
    }
#undef CO_TSP_WORD
    const bool any_left = (__ballot(left != 0) & gmask) != 0;
    if constexpr (G >= 8) {
      if (valid && !(CO_TSP_SCUT & 1)) {
        int64_t* d8 = sl == 0 ? epi.i_out : sl == 1 ? epi.first_out : epi.cur_out;
        const int64_t v8 = sl == 0 ? rs + 1 : (sl == 1 && !epi.take_first) ? rs : a_raw;
        if (sl < 3 && d8) d8[r] = v8;
        if (sl == 3 || sl == 4) (sl == 3 ? epi.done : epi.reward)[r] = sl == 3 ? !any_left : 0;
      }
    } else if (valid && sl == 0 && !(CO_TSP_SCUT & 1)) {
      epi.store(r, a_raw, any_left ? 1 : 0, rv);
    }
  }
}

// Flat step (round 4): a wave owns R consecutive rows, i.e. the contiguous R*N mask bytes
// [b0*N, (b0+R)*N) (16-byte aligned: R*N % 16 == 0 and an aligned base), moved as 16-byte
// chunks -- lane l holds chunks l + 64u (u < CPL) -- so each load / store instruction
// covers 1 KiB of the rows (the lane-group kernel's dword instructions: 256 B in 8 row
// pieces), and the row scalars of the R rows are one coalesced access per column (lane r
// owns row b0 + r).  A chunk holds bytes of at most two rows (N >= 16): r0 = 16j / N and
// r1 = (16j + 15) / N; their actions come from the row lanes by ds_bpermute and clear the
// chunk's byte of each (SWAR on the four words).  Row r's "anything left" is the OR of
// its chunks' nonzero tests, evaluated on two ballots per chunk slot (f0: the chunk's
// part in row r0, f1: the part in row r1): row r's first chunk contributes its f1 part
// when it starts in row r - 1, the following ones their f0 part.  The last wave's
// partial rows (B % R) leave a tail of < 16 bytes, moved as dwords (N % 4 == 0).
template <int R, int CPL>
__global__ __launch_bounds__(256) void tsp_step_flat_kernel(int64_t B, int N,
                                                            const int64_t* __restrict__ action,
                                                            const uint8_t* mask_in,
                                                            uint8_t* mask_out, TspRowEpilogue epi,
                                                            int first_mode,
                                                            const int32_t* first_flag,
                                                            int32_t* status) {
  static_assert(R <= 64, "one row per lane for the row scalars");
  const int lane = lane_id();
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t b0 = wid * R;
  if (b0 >= B) return;  // wave-uniform
  if (first_mode == 2) epi.take_first = (*first_flag != 0);
  const int rows = (int)(B - b0 < R ? B - b0 : R);
  const int nbytes = rows * N, nch = nbytes >> 4;
  // row scalars: lane r < rows owns row b0 + r (coalesced)
  const bool rl = lane < rows;
  const int64_t rb = b0 + (rl ? lane : 0);
  const int64_t a_raw = rl ? action[rb] : 0;
  int64_t iv = 0, fv = 0;
  if (rl) {
    iv = epi.i_in[rb];
    if (!epi.take_first) fv = epi.first_in[rb];
  }
  const uint4* src = reinterpret_cast<const uint4*>(mask_in + b0 * N);
  uint4 m[CPL];
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int j = lane + 64 * u;
    m[u] = j < nch ? src[j] : make_uint4(0u, 0u, 0u, 0u);
  }
  // tail dwords of a partial last wave (nbytes % 16 != 0)
  const int ntail = (nbytes & 15) >> 2;
  const uint32_t* srcw = reinterpret_cast<const uint32_t*>(mask_in + b0 * N) + 4 * nch;
  uint32_t tw = lane < ntail ? srcw[lane] : 0u;
  const bool bad = rl && (a_raw < 0 || a_raw >= N);
  if (bad) set_status(status, CO_ST_INDEX_RANGE);
  const int a32 = bad ? -1 : (int)a_raw;  // the row's action (-1: clears nothing)
  uint64_t B0[CPL], B1[CPL];
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int j = lane + 64 * u;
    const int o = 16 * j;                       // the chunk's first byte (wave-relative)
    const int r0 = o / N, r1 = (o + 15) / N;    // its rows (r1 <= r0 + 1 for N >= 16)
    const int a0 = __shfl(a32, r0 < 64 ? r0 : 63, 64), a1 = __shfl(a32, r1 < 64 ? r1 : 63, 64);
    const int p0 = a0 < 0 ? -1 : r0 * N + a0 - o, p1 = a1 < 0 ? -1 : r1 * N + a1 - o;
    uint32_t w[4] = {m[u].x, m[u].y, m[u].z, m[u].w};
    const int split = r1 == r0 ? 16 : r1 * N - o;  // first byte of row r1 in the chunk
    bool f0 = false, f1 = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t x = w[q];
      if ((unsigned)(p0 - 4 * q) < 4u) x &= ~(0xffu << (8 * (p0 - 4 * q)));
      if ((unsigned)(p1 - 4 * q) < 4u) x &= ~(0xffu << (8 * (p1 - 4 * q)));
      w[q] = x;
      const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
      // bytes 4q + e (high bit of byte e of nz) before / at-or-after the row split
      const int lo = split - 4 * q;  // bytes e < lo belong to row r0
      const uint32_t below = lo <= 0 ? 0u : (lo >= 4 ? 0xffffffffu : (1u << (8 * lo)) - 1u);
      f0 |= (nz & below) != 0u;
      f1 |= (nz & ~below) != 0u;
    }
    m[u] = make_uint4(w[0], w[1], w[2], w[3]);
    const bool live = j < nch;
    B0[u] = __ballot(live && f0);
    B1[u] = __ballot(live && f1 && r1 != r0);
  }
  uint4* dst = reinterpret_cast<uint4*>(mask_out + b0 * N);
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int j = lane + 64 * u;
    if (j < nch) dst[j] = m[u];
  }
  // the tail dwords: row of byte 4*(4*nch + lane) and its action
  bool tail_nz = false;
  int tail_row = 0;
  if (ntail) {
    const int o = 16 * nch + 4 * lane;
    tail_row = o / N;
    const int at = __shfl(a32, tail_row < 64 ? tail_row : 63, 64);
    const int pt = at < 0 ? -1 : tail_row * N + at - o;
    if ((unsigned)pt < 4u) tw &= ~(0xffu << (8 * pt));
    tail_nz = lane < ntail && tw != 0u;
    if (lane < ntail) reinterpret_cast<uint32_t*>(mask_out + b0 * N)[4 * nch + lane] = tw;
  }
  const uint64_t BT = __ballot(tail_nz);
  if (!rl) return;
  // row lane r: its chunks jlo..jhi (and tail dwords past the last whole chunk)
  const int r = lane;
  const int first_b = r * N, last_b = r * N + N - 1;
  const int jlo = first_b >> 4, jhi = last_b >> 4;
  bool left = false;
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    // chunk j = 64u + bit: f1 part for jlo when it starts in row r - 1, else f0 parts
    const int lo = jlo - 64 * u, hi = (jhi < nch - 1 ? jhi : nch - 1) - 64 * u;
    const int lo0 = ((jlo << 4) < first_b ? jlo + 1 : jlo) - 64 * u;
    auto range = [](int a, int b) -> uint64_t {  // bits a..b of a 64-bit word (clamped)
      a = a < 0 ? 0 : a;
      b = b > 63 ? 63 : b;
      if (a > b) return 0ull;
      const uint64_t hi_m = b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
      return hi_m & ~((1ull << a) - 1ull);
    };
    left |= (B0[u] & range(lo0, hi)) != 0ull;
    if ((jlo << 4) < first_b) left |= (B1[u] & range(lo, lo)) != 0ull;
  }
  if (ntail) {  // tail dwords t: byte offset 16*nch + 4t, row (16*nch + 4t) / N
    const int t_lo = (first_b - 16 * nch) >> 2, t_hi = (last_b - 16 * nch) >> 2;
    for (int t = t_lo < 0 ? 0 : t_lo; t <= t_hi && t < ntail; ++t) left |= (BT >> t) & 1ull;
  }
  epi.store(rb, a_raw, left ? 1 : 0, TspRowEpilogue::Row{iv, fv});
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void tsp_reward_kernel(int64_t B, int N, int T,
                                                                const float2* locs, int64_t LB,
                                                                const int64_t* actions,
                                                                int64_t sb, int64_t st, int check,
                                                                float* reward, int32_t* status) {
  extern __shared__ uint32_t s_bits[];
  const int w = threadIdx.x >> 6, lane = lane_id();
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
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
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
  // flat step: R rows per wave as 16-byte chunks (N % 4 == 0, 16 <= N, R*N % 16 == 0,
  // 16-byte aligned masks, at most 4 chunks per lane)
  constexpr int FR = CO_TSP_FLAT_ROWS;
  if (FR > 0 && (N & 3) == 0 && N >= 16 && (FR * N) % 16 == 0 && (FR * N + 1023) / 1024 <= 4 &&
      ((reinterpret_cast<uintptr_t>(mask_in) | reinterpret_cast<uintptr_t>(mask_out)) & 15) == 0) {
    const int cpl = (int)((FR * N / 16 + 63) / 64);
    const int64_t waves = (B + FR - 1) / FR;
    const dim3 grid((unsigned)((waves + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
#define CO_TSF(C)                                                                              \
  hipLaunchKernelGGL((tsp_step_flat_kernel<FR, C>), grid, dim3(256), 0, s, B, (int)N, action,   \
                     mask_in, mask_out, epi, first_mode, first_flag, status)
    if (cpl <= 1) CO_TSF(1);
    else if (cpl == 2) CO_TSF(2);
    else if (cpl == 3) CO_TSF(3);
    else CO_TSF(4);
#undef CO_TSF
    return launch_status();
  }
  if (CO_TSP_STEP_GROUP && (N & 3) == 0 && (N >> 2) <= 64 * CO_TSP_WPL &&
      ((reinterpret_cast<uintptr_t>(mask_in) | reinterpret_cast<uintptr_t>(mask_out)) & 3) == 0) {
    const int W = (int)(N >> 2), WG = (W + CO_TSP_WPL - 1) / CO_TSP_WPL;
    const int G = WG <= 2 ? 2 : WG <= 4 ? 4 : WG <= 8 ? 8 : WG <= 16 ? 16 : WG <= 32 ? 32 : 64;
    const int64_t waves = (B * G + 63) / 64;
    const dim3 grid(grid_for(waves, 4, (int64_t)1 << 30));  // a wave per row group
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
  const unsigned grid = (unsigned)((B + kTileRows - 1) / kTileRows);
  hipLaunchKernelGGL(tsp_step_kernel, dim3(grid), dim3(kTileThreads), 0, (hipStream_t)stream, B,
                     (int)N, action, mask_in, mask_out, epi, first_mode, first_flag, status, vec);
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
