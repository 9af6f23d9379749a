// CVRP env kernels for gfx950: reset (+mask), fused step + get_action_mask,
// stand-alone mask, episode reward with the validity/capacity check, and the
// nearest-feasible bench policy.
//
// Step layout: 16-B-aligned buffers take the row-tile kernel (cvrp_step_tile_kernel,
// below); otherwise one wavefront per instance (grid-stride), lanes over the N+1
// columns.  Capacity test `demand + used > capacity` (strict, f32, no contraction);
// visited-sum and any-feasible-customer are row reductions.  The capacity arithmetic
// follows cvrp/env.py:83-85 exactly: used = (used + d) * float(a != 0).
#include "co_common.hpp"
#include "co_tile.hpp"

using namespace co;

#if CO_CVRP_CUT || CO_CVRP_RCUT
// timing-diagnostic builds (tools/build_variants.sh) cut work out of the step / reward
// kernels: their results and status bits are wrong by design.  The marker makes
// _native.load() warn loudly for any library built this way.
extern "C" __attribute__((visibility("default"))) const int co_variant_timing_cut = 1;
#endif

namespace {

// Writes visited_out (optional update at column `a`), the action mask and returns
// the visited sum for the row.  `a` < 0 means no visited update (reset / mask).
__device__ __forceinline__ int cvrp_row(int N, const float* dem, float used, float cap,
                                        const uint8_t* vis_in, uint8_t* vis_out, int64_t a,
                                        int64_t cur, uint8_t* mask) {
  const int lane = lane_id();
  int vsum = 0;
  bool any_feas = false;
  for (int c = lane; c <= N; c += 64) {
    uint8_t v = vis_in[c];
    if (c == a) v = 1;
    if (vis_out) vis_out[c] = v;
    vsum += v;
    if (c >= 1) {
      const bool exceeds = dem[c - 1] + used > cap;
      const bool masked = (v != 0) || exceeds;
      mask[c] = !masked;
      any_feas |= !masked;
    }
  }
  vsum = wave_sum(vsum);
  const bool anyf = __any(any_feas);
  if (lane == 0) mask[0] = !((cur == 0) && anyf);
  return vsum;
}

__global__ __launch_bounds__(256) void cvrp_reset_kernel(int64_t B, int N, const float2* depot,
                                                         const float2* locs_in,
                                                         const float* demand, float vcap,
                                                         float2* locs_out, int64_t* cur,
                                                         float* used, float* vcap_out,
                                                         uint8_t* visited, uint8_t* mask) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    float2* lo = locs_out + b * (N + 1);
    const float2* li = locs_in + b * (int64_t)N;
    for (int c = lane; c <= N; c += 64) lo[c] = (c == 0) ? depot[b] : li[c - 1];
    uint8_t* vrow = visited + b * (N + 1);
    for (int c = lane; c <= N; c += 64) vrow[c] = 0;
    if (lane == 0) {
      cur[b] = 0;
      used[b] = 0.f;
      vcap_out[b] = vcap;
    }
    // mask from the fresh state: visited == 0, used == 0, current == 0
    const float* dem = demand + b * (int64_t)N;
    uint8_t* mrow = mask + b * (N + 1);
    bool any_feas = false;
    for (int c = lane + 1; c <= N; c += 64) {
      const bool masked = dem[c - 1] + 0.f > vcap;
      mrow[c] = !masked;
      any_feas |= !masked;
    }
    const bool anyf = __any(any_feas);
    if (lane == 0) mrow[0] = !anyf;
  }
}

__global__ __launch_bounds__(256) void cvrp_step_kernel(
    int64_t B, int N, const int64_t* action, const float* demand, const float* used_in,
    float* used_out, const float* vcap, const uint8_t* vis_in, uint8_t* vis_out, int64_t* cur_out,
    uint8_t* done, uint8_t* reward, uint8_t* mask, int32_t* status,
    int32_t* not_done) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  int left = 0;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const int64_t a = action[b];
    const bool bad = a < 0 || a > N;
    if (bad && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    const float* dem = demand + b * (int64_t)N;
    int64_t di = a - 1;
    di = di < 0 ? 0 : (di > N - 1 ? N - 1 : di);
    const float d = dem[di];
    const float u = (used_in[b] + d) * ((a != 0) ? 1.0f : 0.0f);
    const float cap = vcap[b];
    const int vsum = cvrp_row(N, dem, u, cap, vis_in + b * (N + 1), vis_out + b * (N + 1),
                              bad ? -1 : a, a, mask + b * (N + 1));
    if (lane == 0) {
      used_out[b] = u;
      if (cur_out) cur_out[b] = a;
      done[b] = vsum == N + 1;
      left += vsum != N + 1;
      reward[b] = 0;
    }
  }
  if (not_done && lane == 0 && left) atomicAdd(not_done, left);
}

// ---------------------------------------------------------------------------
// Tile step: one 256-thread workgroup owns R consecutive rows (R a multiple of 16, so
// the [R, N+1] byte tiles of visited / action_mask start 16-B aligned).  The visited
// tile streams through registers in 16-B chunks (at most kCvrpCpt per thread, kept in
// registers across the barrier), the [R, N] demand tile is staged in LDS by float4
// loads, and the two row reductions of the step (visited sum for `done`, "any feasible
// customer" for the depot column) are per-chunk partials in LDS summed per row.  The
// depot byte of each row is patched into its chunk after the barrier, so every byte of
// the mask tile is written once by a 16-B store.  `not_done` (optional) receives one
// atomicAdd per workgroup: the number of its rows that are not done.
#ifndef CO_CVRP_QUAD
#define CO_CVRP_QUAD 1  // co_cvrp_step takes the row-group kernel (below) when it can
#endif
#ifndef CO_CVRP_Q
#define CO_CVRP_Q 1  // row groups per wave in the row-group kernel
#endif
#ifndef CO_CVRP_G
#define CO_CVRP_G 16  // lanes per row in the row-group kernel
#endif
#ifndef CO_CVRP_ROWS
#define CO_CVRP_ROWS 64
#endif
#ifndef CO_CVRP_CPT
#define CO_CVRP_CPT 2
#endif
constexpr int kCvrpCpt = CO_CVRP_CPT;
constexpr int kCvrpMaxRows = CO_CVRP_ROWS;

template <int THREADS>
__global__ __launch_bounds__(THREADS) void cvrp_step_tile_kernel(
    int64_t B, int N, int R, const int64_t* __restrict__ action, const float* __restrict__ demand,
    const float* __restrict__ used_in, float* __restrict__ used_out,
    const float* __restrict__ vcap, const uint8_t* vis_in, uint8_t* vis_out,
    int64_t* __restrict__ cur_out, uint8_t* __restrict__ done, uint8_t* __restrict__ reward,
    uint8_t* __restrict__ mask, int32_t* status, int32_t* not_done) {
  extern __shared__ float s_dem_raw[];  // 4 pad floats, then [R, N]
  float* const s_dem = s_dem_raw + 4;
  __shared__ int s_act[kCvrpMaxRows];
  __shared__ float s_u[kCvrpMaxRows], s_cap[kCvrpMaxRows];
  __shared__ int s_cnt[kCvrpMaxRows], s_feas[kCvrpMaxRows];
  __shared__ int s_part[2 * kCvrpCpt * THREADS];  // per chunk: (sum, any) of its <= 2 rows
  const int tid = threadIdx.x;
  const int NC = N + 1;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int rows = (int)((B - row0) < R ? (B - row0) : R);
  const int nbytes = rows * NC;
  const int nchunks = (nbytes + 15) >> 4;
  const uint8_t* vsrc = vis_in + row0 * NC;

  // every global load of the tile is issued before the first barrier
  int64_t a_raw = 0;
  float uin = 0.f, cap = 0.f;
  if (tid < rows) {
    a_raw = action[row0 + tid];
    uin = used_in[row0 + tid];
    cap = vcap[row0 + tid];
  }
  uint4 v[kCvrpCpt];
#pragma unroll
  for (int k = 0; k < kCvrpCpt; ++k) {
    const int c = tid + k * THREADS;
    if (c < nchunks) v[k] = tile_load(vsrc, c << 4, nbytes, true);
  }
  // demand tile -> LDS by LDS-DMA; the helper's vmcnt(0) + barrier also covers the loads above
#if CO_CVRP_CUT & 1  // timing diagnostic only (tools/diag_cvrp_step.py): no demand tile
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
#else
  stage_bytes_lds(reinterpret_cast<const unsigned char*>(demand + row0 * N), rows * N * 4,
                  reinterpret_cast<unsigned char*>(s_dem));
#endif
  if (tid < rows) {  // cvrp/env.py:79-85
    const bool bad = a_raw < 0 || a_raw > N;
    if (bad) set_status(status, CO_ST_INDEX_RANGE);
    s_act[tid] = bad ? -1 : (int)a_raw;
    s_cap[tid] = cap;
    int64_t di = a_raw - 1;
    di = di < 0 ? 0 : (di > N - 1 ? N - 1 : di);
    s_u[tid] = (uin + s_dem[tid * N + di]) * ((a_raw != 0) ? 1.0f : 0.0f);
  }
  __syncthreads();

  // Each chunk spans at most two rows (NC >= 17): r0 from byte 0, r1 from byte `split`.
  // No branches per byte (selects and word-wide byte arithmetic); each chunk leaves (sum, any-feasible) of both row
  // parts in LDS and one thread per row adds its ~NC/16 parts after the barrier.
  uint4 m[kCvrpCpt];
  uint8_t* vdst = vis_out + row0 * NC;
#pragma unroll
  for (int k = 0; k < kCvrpCpt; ++k) {
    const int ch = tid + k * THREADS;
    if (ch >= nchunks) continue;
    const int off = ch << 4;
    const int r0 = off / NC, c0 = off - r0 * NC;
    const int split = NC - c0;  // bytes of row r0 in this chunk
    const int r1 = r0 + 1;
    const bool has1 = split < 16 && r1 < rows;
    const int act0 = s_act[r0], act1 = has1 ? s_act[r1] : -1;
    const float u0 = s_u[r0], cp0 = s_cap[r0];
    const float u1 = has1 ? s_u[r1] : 0.f, cp1 = has1 ? s_cap[r1] : 0.f;
    const int dbase = off - r0 - 1;  // s_dem index of byte j: dbase + j (row r0), one less (r1)
    uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#if CO_CVRP_CUT & 2  // timing diagnostic only: no per-byte update
    s_part[2 * ch] = 0;
    s_part[2 * ch + 1] = 0;
    tile_store(vdst, off, nbytes, true, v[k]);
    m[k] = v[k];
    continue;
#endif
    // all 16 demand reads issued before any use (a short-circuit `||` would put each
    // behind a branch and an lgkmcnt(0) wait)
    // 17 consecutive floats from one base (static offsets, no per-read address math): byte
    // j of r0 takes D[j + 1], of r1 D[j]; the first tile's base is -2 (pad floats, unused)
    float D[17], dm[16];
    const float* dp = s_dem + dbase - 1;
#pragma unroll
    for (int t = 0; t < 17; ++t) D[t] = dp[t];
#pragma unroll
    for (int j = 0; j < 16; ++j) dm[j] = j >= split ? D[j] : D[j + 1];
    // Per byte only the capacity test (f32 add + compare, as the reference) sets a flag bit;
    // the rest is word-wide (SWAR) on the chunk's four u32 words: r0 / r1 byte masks from
    // `split`, the action byte of each row set to 1, the nonzero test, byte sums by
    // v_sad_u8, the customer mask and its any-feasible tests.
    const int ja0 = (act0 >= c0 && act0 - c0 < split) ? act0 - c0 : -1;  // byte of r0's action
    const int ja1 = (act1 >= 0 && split + act1 < 16) ? split + act1 : -1;
    int cnt0 = 0, cnt1 = 0;
    uint32_t f0 = 0u, f1 = 0u, um_w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lo = split - 4 * q;  // bytes of this word that belong to r0
      const uint32_t m0 = lo >= 4 ? 0xffffffffu : lo <= 0 ? 0u : (1u << (8 * lo)) - 1u;
      uint32_t x = w[q];
      if ((ja0 >> 2) == q) x = (x & ~(0xffu << (8 * (ja0 & 3)))) | (1u << (8 * (ja0 & 3)));
      if ((ja1 >> 2) == q) x = (x & ~(0xffu << (8 * (ja1 & 3)))) | (1u << (8 * (ja1 & 3)));
      w[q] = x;
      uint32_t over = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * q + e;
        const bool sec = j >= split;
        over |= (dm[j] + (sec ? u1 : u0) > (sec ? cp1 : cp0)) ? (0x80u << (8 * e)) : 0u;
      }
      const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
      uint32_t mk = (~(nz | over) & 0x80808080u) >> 7;
      // depot bytes (column 0: byte 0 when r0 starts here, byte `split` for r1) are left 0
      // here and patched after the row sums; they take no part in any-feasible
      if (q == 0 && c0 == 0) mk &= ~0xffu;
      if ((split >> 2) == q && split < 16) mk &= ~(0xffu << (8 * (split & 3)));
      cnt0 = __builtin_amdgcn_sad_u8(x & m0, 0u, cnt0);
      cnt1 = __builtin_amdgcn_sad_u8(x & ~m0, 0u, cnt1);
      f0 |= mk & m0;
      f1 |= mk & ~m0;
      um_w[q] = mk;
    }
    const int feas0 = f0 != 0u, feas1 = f1 != 0u;
    s_part[2 * ch] = cnt0 | (feas0 << 16);
    s_part[2 * ch + 1] = cnt1 | (feas1 << 16);
    tile_store(vdst, off, nbytes, true, make_uint4(w[0], w[1], w[2], w[3]));
    m[k] = make_uint4(um_w[0], um_w[1], um_w[2], um_w[3]);
  }
  __syncthreads();
  if (tid < rows) {  // row sums over the row's chunk parts
    int cnt = 0, feas = 0;
    const int ch_lo = (tid * NC) >> 4, ch_hi = ((tid + 1) * NC - 1) >> 4;
    for (int ch = ch_lo; ch <= ch_hi; ++ch) {
      const int pv = s_part[2 * ch + (((ch << 4) / NC) == tid ? 0 : 1)];
      cnt += pv & 0xffff;
      feas |= pv >> 16;
    }
    s_cnt[tid] = cnt;
    s_feas[tid] = feas;
  }
  __syncthreads();
  // depot column of the rows starting in each chunk (cvrp/env.py:146-148), patched with
  // static byte positions only (a dynamic byte index would spill the chunk to scratch)
  uint8_t* mdst = mask + row0 * NC;
#pragma unroll
  for (int k = 0; k < kCvrpCpt; ++k) {
    const int ch = tid + k * THREADS;
    if (ch >= nchunks) continue;
    const int off = ch << 4;
    const int r0 = off / NC, c0 = off - r0 * NC;
    const int split = NC - c0;
    const int r1 = r0 + 1;
    const int pos0 = c0 == 0 ? 0 : -1;
    const int pos1 = (split < 16 && r1 < rows) ? split : -1;
    const uint32_t d0 = !((s_act[r0] == 0) && s_feas[r0]);
    const uint32_t d1 = pos1 >= 0 ? (uint32_t) !((s_act[r1] == 0) && s_feas[r1]) : 0u;
    uint32_t w[4] = {m[k].x, m[k].y, m[k].z, m[k].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = q * 4 + e;
        const uint32_t keep = ~(0xffu << (8 * e));
        if (j == pos0) w[q] = (w[q] & keep) | (d0 << (8 * e));
        if (j == pos1) w[q] = (w[q] & keep) | (d1 << (8 * e));
      }
    }
    tile_store(mdst, off, nbytes, true, make_uint4(w[0], w[1], w[2], w[3]));
  }
  if (tid < rows) {
    const int64_t b = row0 + tid;
    used_out[b] = s_u[tid];
    if (cur_out) cur_out[b] = a_raw;
    const bool dn = s_cnt[tid] == NC;
    done[b] = dn;
    reward[b] = 0;
    if (not_done) {
      const int left = __popcll(__ballot(!dn));
      if (tid == 0 && left) atomicAdd(not_done, left);
    }
  }
}

// Row-group step (cvrp/env.py:73-149, the env step the tile kernel above also
// implements): 16 lanes per row, 4 rows per wave, Q groups of 4 consecutive rows ("quads")
// per wave whose loads are all issued before the first quad is computed (the compiler's
// counted vmcnt lets quad i's work overlap quads i+1.. still in flight).  The visited /
// action_mask rows (N+1 bytes, not 4-byte aligned) are read and written in place as the
// aligned dwords that cover the row: lane sl owns dwords k = sl + 16j of it, byte e of
// dword k is column 4k + e - s (s: the row's first byte within its first dword).  The
// demand of those 4 columns is one 4-byte-aligned float4 load (demand[4k - s - 1 ...]).
// Row-uniform values (action, used / vehicle capacity) are group-uniform; the selected
// demand (the action's column) comes from the lane that holds it by a 16-lane OR
// reduction, so no load depends on another.  Per dword only the f32 capacity test
// `demand + used > capacity` runs per byte; the action byte, the nonzero test, the byte
// sums (v_sad_u8) and the customer mask are word-wide; the row sums (done, the depot
// column) are 16-lane DPP / ballot operations.  Interior dwords are stored whole, the
// row's first and last dword (shared with the neighbouring rows) as its own bytes.  No
// LDS, no workgroup barrier on the data path; `not_done` (optional): one atomic per
// workgroup.
typedef float f4_a4 __attribute__((ext_vector_type(4), aligned(4)));

template <int G, int U, int Q, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void cvrp_step_rows_kernel(
    int64_t B, int N, const int64_t* __restrict__ action, const float* __restrict__ demand,
    const float* __restrict__ used_in, float* __restrict__ used_out,
    const float* __restrict__ vcap, const uint8_t* vis_in, uint8_t* vis_out,
    int64_t* __restrict__ cur_out, uint8_t* __restrict__ done, uint8_t* __restrict__ reward,
    uint8_t* __restrict__ mask, int32_t* status, int32_t* not_done) {
  __shared__ int s_left[WAVES];
  constexpr int RW = 64 / G;  // rows per wave
  const int lane = lane_id(), w = wave_in_block(), sl = lane % G, grp = lane / G;
  const int NC = N + 1;
  const int64_t wrow0 = ((int64_t)blockIdx.x * WAVES + w) * (RW * Q);
  int left = 0;
  if (wrow0 < B) {
    // ---- every load of the wave's Q quads (rows past B re-read row B-1: not stored)
    int64_t A[Q];
    float UI[Q], CP[Q];
    uint32_t V[Q][U];
    f4_a4 D[Q][U];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t b0 = wrow0 + RW * q + grp;
      const int64_t b = b0 < B ? b0 : B - 1;
      A[q] = action[b];
      UI[q] = used_in[b];
      CP[q] = vcap[b];
      const int64_t byte0 = b * NC;
      const int s = (int)(byte0 & 3);
      const int ndw = (s + NC + 3) >> 2;
      const uint32_t* vrow = reinterpret_cast<const uint32_t*>(vis_in + (byte0 - s));
      const float* drow = demand + b * N;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int k0 = sl + G * j;
        const int k = k0 < ndw ? k0 : 0;
        const int cb = 4 * k - s;
        if (b == B - 1 && k == ndw - 1 && ((byte0 + NC) & 3)) {  // the buffer's last bytes
          uint32_t x = 0u;
#pragma unroll
          for (int e = 0; e < 3; ++e)
            if (e < ((byte0 + NC) & 3)) x |= (uint32_t)vis_in[byte0 - s + 4 * k + e] << (8 * e);
          V[q][j] = x;
        } else {
          V[q][j] = vrow[k];
        }
        if ((b == 0 && cb < 1) || (b == B - 1 && cb + 2 > N - 1)) {
          // the buffer's first / last row: out-of-row elements clamped (they belong to no
          // customer byte of this row)
          f4_a4 d;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ix = cb - 1 + e;
            d[e] = drow[ix < 0 ? 0 : (ix > N - 1 ? N - 1 : ix)];
          }
          D[q][j] = d;
        } else {
          D[q][j] = *reinterpret_cast<const f4_a4*>(drow + (cb - 1));
        }
      }
    }
    // ---- per quad: cvrp/env.py:79-92 and get_action_mask (:137-149)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t b = wrow0 + RW * q + grp;
      const bool valid = b < B;
      const int64_t bb = valid ? b : B - 1;
      const int64_t a_raw = A[q];
      const bool bad = a_raw < 0 || a_raw > N;
      if (valid && bad && sl == 0) set_status(status, CO_ST_INDEX_RANGE);
      const int64_t byte0 = bb * NC;
      const int s = (int)(byte0 & 3);
      const int ndw = (s + NC + 3) >> 2;
      // the selected demand demand[clamp(a - 1, 0, N - 1)] from the lane holding it
      const int csel = (int)(a_raw - 1 < 0 ? 0 : (a_raw - 1 > N - 1 ? N - 1 : a_raw - 1)) + 1;
      uint32_t selb = 0u;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int k = sl + G * j;
        const int es = csel - (4 * k - s);
        if (k < ndw && es >= 0 && es < 4) {
          const f4_a4 d = D[q][j];
          selb = __float_as_uint(es == 0 ? d[0] : es == 1 ? d[1] : es == 2 ? d[2] : d[3]);
        }
      }
      selb = grp_reduce<G>(selb, [](uint32_t x, uint32_t y) { return x | y; });
      const float u = (UI[q] + __uint_as_float(selb)) * ((a_raw != 0) ? 1.0f : 0.0f);
      const float cap = CP[q];
      const int a = bad ? -1 : (int)a_raw;
      uint32_t m[U];
      uint32_t cnt = 0u;
      bool feas = false;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int k = sl + G * j;
        const bool live = valid && k < ndw;
        const int cb = live ? 4 * k - s : 0;  // column of byte 0 (dead slots: dword 0's)
        // the row's own bytes [lo, hi) of this dword; the depot byte (column 0) at -cb
        const int lo = cb < 0 ? -cb : 0;
        const int hi = NC - cb < 4 ? NC - cb : 4;
        const uint32_t own = !live ? 0u
                             : ((hi >= 4 ? 0xffffffffu : (1u << (8 * hi)) - 1u) &
                                ~((1u << (8 * lo)) - 1u));
        const uint32_t cust = cb <= 0 ? own & ~(0xffu << (8 * lo)) : own;  // depot excluded
        uint32_t x = V[q][j];
        const int ea = a - cb;  // the action's byte, if in this dword
        if (a >= 0 && ea >= 0 && ea < 4) x = (x & ~(0xffu << (8 * ea))) | (1u << (8 * ea));
        V[q][j] = x;
        const f4_a4 d = D[q][j];
        const uint32_t over = ((d[0] + u > cap) ? 0x80u : 0u) | ((d[1] + u > cap) ? 0x8000u : 0u) |
                              ((d[2] + u > cap) ? 0x800000u : 0u) |
                              ((d[3] + u > cap) ? 0x80000000u : 0u);
        const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
        const uint32_t mk = ((~(nz | over) & 0x80808080u) >> 7) & cust;
        cnt = __builtin_amdgcn_sad_u8(x & own, 0u, cnt);
        feas |= mk != 0u;
        m[j] = mk;
      }
      // row sums over the group (cvrp/env.py:92 done; :146-148 the depot column)
      cnt = grp_reduce<G>(cnt, [](uint32_t x, uint32_t y) { return x + y; });
      const uint64_t gm = G == 64 ? ~0ull : ((1ull << G) - 1ull);
      const bool anyf = ((__ballot(feas) >> (G * grp)) & gm) != 0ull;
      const uint32_t dep = !((a_raw == 0) && anyf);
      uint8_t* vdst = vis_out + byte0;
      uint8_t* mdst = mask + byte0;
      // Stores as whole dwords: the dword a row shares with the previous row of its quad
      // (its first, when the row does not start 4-aligned) is written by this row's lane 0
      // with the previous row's bytes merged in (one lane shuffle of each word); the
      // previous row skips it.  A quad of 4 rows starts and ends 4-aligned (4 (N+1) bytes
      // from a 4-aligned start), so no dword is shared between waves -- only the buffer's
      // last row, when B % 4 != 0, stores its trailing bytes one by one.
      uint32_t mm[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int cb = 4 * (sl + G * j) - s;
        mm[j] = cb <= 0 ? m[j] | (dep << (8 * -cb)) : m[j];
      }
      const int jl = (ndw - 1) / G;  // the slot of the row's last dword (group-uniform)
      uint32_t lastv = 0u, lastm = 0u;
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j == jl) {
          lastv = V[q][j];
          lastm = mm[j];
        }
      const int sp = (int)((byte0 - NC) & 3);  // the previous row's first-byte offset
      const int src = grp > 0 ? (grp - 1) * G + ((((sp + NC + 3) >> 2) - 1) % G) : lane;
      const uint32_t prev_v = __shfl(lastv, src, 64), prev_m = __shfl(lastm, src, 64);
      const bool tail_shared = ((byte0 + NC) & 3) != 0;  // the last dword holds row b + 1's bytes
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int k = sl + G * j;
        if (!valid || k >= ndw) continue;
        uint32_t vv = V[q][j], mv = mm[j];
        if (k == 0 && s > 0) {  // shared with the previous row of the quad: merged
          const uint32_t ownb = ~((1u << (8 * s)) - 1u);
          vv = (vv & ownb) | (prev_v & ~ownb);
          mv = (mv & ownb) | (prev_m & ~ownb);
        }
        if (k == ndw - 1 && tail_shared) {
          if (b + 1 < B) continue;  // the next row's lane 0 writes it
          const int cb = 4 * k - s;  // the buffer's last row: its own bytes only
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e < NC - cb) {
              vdst[cb + e] = (uint8_t)(vv >> (8 * e));
              mdst[cb + e] = (uint8_t)(mv >> (8 * e));
            }
          continue;
        }
        reinterpret_cast<uint32_t*>(vdst - s)[k] = vv;
        reinterpret_cast<uint32_t*>(mdst - s)[k] = mv;
      }
      if (valid) {  // the row scalars, spread over the group's lanes
        if (sl == 0) used_out[b] = u;
        if (sl == 1 && cur_out) cur_out[b] = a_raw;
        if (sl == 2) done[b] = (int)cnt == NC;
        if (sl == 3) reward[b] = 0;
      }
      left += valid && sl == 0 && (int)cnt != NC;
    }
  }
  if (not_done) {  // one atomic per workgroup (the counter of rows not done)
    const int wl = (int)wave_sum((uint32_t)left);
    if (lane == 0) s_left[w] = wl;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int q = 0; q < WAVES; ++q) t += s_left[q];
      if (t) atomicAdd(not_done, t);
    }
  }
}

// Nearest-feasible policy, G lanes per instance: node c = 1 + sl + k*G (coalesced float2
// and mask-byte loads across the group, all KM of a lane issued before any use),
// Euclidean distance as torch (f32, no contraction), group argmin with the lowest index
// on ties, depot when no customer is feasible.  KM = 0: runtime loop for large N.  Loop
// counts are wave-uniform (the DPP reductions need every lane).
template <int G, int KM>
__global__ __launch_bounds__(256) void cvrp_nearest_group_kernel(int64_t B, int N,
                                                                 const float2* __restrict__ locs,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const int64_t* __restrict__ cur,
                                                                 int64_t* __restrict__ out) {
  const int lane = lane_id(), sl = lane % G;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const int K = (N + G - 1) / G;
  for (int64_t base = wid * (64 / G); base < B; base += nwaves * (64 / G)) {
    const int64_t b = base + lane / G;
    const bool valid = b < B;
    const int64_t r = valid ? b : 0;
    const float2* lrow = locs + r * (int64_t)(N + 1);
    const uint8_t* mrow = mask + r * (int64_t)(N + 1);
    int64_t c0 = cur[r];
    float best = __builtin_inff();
    int bi = 0x7fffffff;
    if (KM > 0) {
      // unconditional loads at clamped columns and select-based updates: a predicated
      // load would be sunk by the compiler behind the mask test and its vmcnt(0) wait
      float2 q[KM > 0 ? KM : 1];
      uint8_t mk[KM > 0 ? KM : 1];
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int c = 1 + sl + k * G;
        const int cc = c <= N ? c : N;
        mk[k] = mrow[cc];
        q[k] = lrow[cc];
      }
      c0 = (c0 < 0 || c0 > N) ? 0 : c0;
      const float2 p = lrow[c0];
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int c = 1 + sl + k * G;
        const float d = edge_len(p.x, p.y, q[k].x, q[k].y);
        const bool take = (k < K) & (c <= N) & (mk[k] != 0) & (d < best);
        best = take ? d : best;
        bi = take ? c : bi;
      }
    } else {
      c0 = (c0 < 0 || c0 > N) ? 0 : c0;
      const float2 p = lrow[c0];
      for (int k = 0; k < K; ++k) {
        const int c = 1 + sl + k * G;
        if (valid && c <= N && mrow[c]) {
          const float2 q = lrow[c];
          const float d = edge_len(p.x, p.y, q.x, q.y);
          if (d < best) { best = d; bi = c; }
        }
      }
    }
    grp_argmin_split<G>(best, bi);
    if (valid && sl == 0) out[b] = bi == 0x7fffffff ? 0 : bi;
  }
}

// The nearest-feasible bench policy fused with the step (co_cvrp_nearest_step: the
// results of co_cvrp_nearest_action + co_cvrp_step in one launch).  A 256-thread
// workgroup owns a tile of 16 rows, G = 16 lanes per row; lane sl owns nodes
// c = sl + k*16 (k < KM).  The tile's visited and mask bytes (16 x (N+1), a multiple of 16
// bytes, so the tile starts 16-B aligned) move between HBM and LDS as 16-B chunks; the
// lanes' coordinates and demands are loaded straight into registers (coalesced across
// the group), all before the first use.  The current node's coordinates and the chosen
// node's demand come from their owner lanes by shuffle; the policy is the group argmin of
// the torch-exact Euclidean distance over feasible customers (lowest index on ties, depot
// when none); the step then updates visited / capacity and recomputes the mask in
// registers (cvrp/env.py:73-105,137-149).  One not-done atomic per workgroup.
constexpr int kCnsRows = 16;
template <int KM>
__global__ __launch_bounds__(256) void cvrp_nearest_step_kernel(
    int64_t B, int N, const float2* __restrict__ locs, const float* __restrict__ demand,
    const float* __restrict__ used_in, float* __restrict__ used_out,
    const float* __restrict__ vcap, const uint8_t* vis_in, uint8_t* vis_out,
    const uint8_t* mask_in, const int64_t* __restrict__ cur_in, int64_t* __restrict__ action_out,
    int64_t* __restrict__ cur_out, uint8_t* __restrict__ done, uint8_t* __restrict__ reward,
    uint8_t* mask_out, bool vec, int32_t* not_done) {
  constexpr int G = 16;
  __shared__ __attribute__((aligned(16))) uint8_t s_vis[kCnsRows * 16 * KM];
  __shared__ __attribute__((aligned(16))) uint8_t s_mk[kCnsRows * 16 * KM];
  __shared__ int s_left[4];
  const int tid = threadIdx.x, lane = tid & 63, sl = tid % G, row = tid / G;
  const int NC = N + 1;
  for (int64_t tile = blockIdx.x; tile * kCnsRows < B; tile += gridDim.x) {
    const int64_t row0 = tile * kCnsRows;
    const int rows = (int)((B - row0) < kCnsRows ? (B - row0) : kCnsRows);
    const int nbytes = rows * NC, nchunks = (nbytes + 15) >> 4;
    const bool valid = row < rows;
    const int64_t r = row0 + (valid ? row : 0);
    // every global load before the barrier: the byte tiles (16-B chunks), the lane's
    // coordinates and demands at clamped columns, the row scalars
    uint4 cv = make_uint4(0, 0, 0, 0), cm = cv;
    if (tid < nchunks) {
      cv = tile_load(vis_in + row0 * NC, tid << 4, nbytes, vec);
      cm = tile_load(mask_in + row0 * NC, tid << 4, nbytes, vec);
    }
    const float2* lrow = locs + r * NC;
    const float* drow = demand + r * (int64_t)N;
    float2 q[KM];
    float dm[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int c = sl + k * G;
      const int cc = c <= N ? c : N;
      q[k] = lrow[cc];
      dm[k] = drow[cc >= 1 ? cc - 1 : 0];
    }
    int64_t c0 = cur_in[r];
    const float u_in = used_in[r], cap = vcap[r];
    if (tid < nchunks) {
      *reinterpret_cast<uint4*>(s_vis + (tid << 4)) = cv;
      *reinterpret_cast<uint4*>(s_mk + (tid << 4)) = cm;
    }
    __syncthreads();
    uint8_t mk[KM], vs[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int c = sl + k * G;
      const int o = row * NC + (c <= N ? c : N);
      mk[k] = s_mk[o];
      vs[k] = s_vis[o];
    }
    c0 = (c0 < 0 || c0 > N) ? 0 : c0;
    float2 pc = q[0];
#pragma unroll
    for (int k = 1; k < KM; ++k) pc = (k == (int)(c0 / G)) ? q[k] : pc;
    const int g0 = lane - sl;
    const float px = __shfl(pc.x, g0 + (int)(c0 % G), 64);
    const float py = __shfl(pc.y, g0 + (int)(c0 % G), 64);
    // the policy (co_cvrp_nearest_action)
    float best = __builtin_inff();
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int c = sl + k * G;
      const float d = edge_len(px, py, q[k].x, q[k].y);
      const bool take = (c >= 1) & (c <= N) & (mk[k] != 0) & (d < best);
      best = take ? d : best;
      bi = take ? c : bi;
    }
    grp_argmin_split<G>(best, bi);
    const int a = bi == 0x7fffffff ? 0 : bi;
    // the step (cvrp/env.py:79-85): d = demand[clamp(a - 1, 0, N - 1)], from its owner lane
    const int nd = a >= 1 ? a : 1;
    float dsel = dm[0];
#pragma unroll
    for (int k = 1; k < KM; ++k) dsel = (k == nd / G) ? dm[k] : dsel;
    dsel = __shfl(dsel, g0 + nd % G, 64);
    const float u = (u_in + dsel) * ((a != 0) ? 1.0f : 0.0f);
    int vsum = 0, anyf = 0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int c = sl + k * G;
      if (c <= N) {
        const uint8_t v = (uint8_t)(vs[k] | (c == a));
        vs[k] = v;
        vsum += v;
        if (c >= 1) {  // cvrp/env.py:140-144: visited | demand + used > capacity (strict)
          const bool masked = (v != 0) || (dm[k] + u > cap);
          mk[k] = !masked;
          anyf |= !masked;
        }
      }
    }
    vsum = (int)grp_reduce<G>((uint32_t)vsum, [](uint32_t x, uint32_t y) { return x + y; });
    anyf = grp_max_int<G>(anyf);
    if (sl == 0) mk[0] = !((a == 0) && anyf);  // node 0 is lane 0's k = 0
    if (valid) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int c = sl + k * G;
        if (c <= N) {
          s_vis[row * NC + c] = vs[k];
          s_mk[row * NC + c] = mk[k];
        }
      }
    }
    const bool dn = vsum == N + 1;
    if (not_done) {
      const int left = __popcll(__ballot(valid && sl == 0 && !dn));
      if (lane == 0) s_left[tid >> 6] = left;
    }
    __syncthreads();
    if (tid < nchunks) {
      tile_store(vis_out + row0 * NC, tid << 4, nbytes, vec,
                 *reinterpret_cast<const uint4*>(s_vis + (tid << 4)));
      tile_store(mask_out + row0 * NC, tid << 4, nbytes, vec,
                 *reinterpret_cast<const uint4*>(s_mk + (tid << 4)));
    }
    if (valid && sl == 0) {
      action_out[r] = a;
      used_out[r] = u;
      cur_out[r] = a;
      done[r] = dn;
      reward[r] = 0;
    }
    if (not_done && tid == 0) {
      const int left = s_left[0] + s_left[1] + s_left[2] + s_left[3];
      if (left) atomicAdd(not_done, left);
    }
    __syncthreads();  // the LDS tiles are reused by the next tile
  }
}

__global__ __launch_bounds__(256) void cvrp_mask_kernel(int64_t B, int N, const float* demand,
                                                        const float* used, const float* vcap,
                                                        const uint8_t* visited,
                                                        const int64_t* cur, uint8_t* mask) {
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    cvrp_row(N, demand + b * (int64_t)N, used[b], vcap[b], visited + b * (N + 1), nullptr, -1,
             cur[b], mask + b * (N + 1));
  }
}

// Reward: ordered = [depot] + locs[actions] (T+1 points, closed tour).
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void cvrp_reward_kernel(
    int64_t B, int N, int T, const float2* locs, const int64_t* actions, int64_t sb, int64_t st,
    const float* demand, const float* vcap, int check, float* reward, int32_t* status) {
  extern __shared__ uint32_t s_mem[];
  const int w = wave_in_block(), lane = lane_id();
  const int words = (N + 32) >> 5;  // bits for values 0..N
  uint32_t* bits = s_mem + w * (words + 4 * T);
  float* dseq = reinterpret_cast<float*>(bits + words);
  int* starts = reinterpret_cast<int*>(dseq + T);  // route (segment) start steps
  float* sval = dseq + 2 * T;                       // [2][T] route start values (ping-pong)
  for (int64_t b = (int64_t)blockIdx.x * WAVES + w; b < B; b += (int64_t)gridDim.x * WAVES) {
    const int64_t* arow = actions + b * sb;
    const float2* lrow = locs + b * (int64_t)(N + 1);
    if (check) {
      for (int k = lane; k < words; k += 64) bits[k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const float cap = check ? vcap[b] : 0.f;
    double acc = 0.0;
    bool bad = false, range = false, start_here = false;
    int nonzero = 0, nseg = 0;
    const int M = T + 1;
    // lane m loads action m and its coordinates once; the edge's start node comes from
    // lane m-1 (shuffle) or, for lane 0, from the previous block's lane 63 (depot at m = 0)
    int a_carry = 0;
    float px_carry = lrow[0].x, py_carry = lrow[0].y;
    // kPre 64-step pieces at a time: their action loads issued together, then their
    // coordinate / demand gathers together (r05: one piece per iteration waited for two
    // dependent round trips per 64 steps -- 8 for T = 199)
    constexpr int kPre = 4;
    for (int base0 = 0; base0 < M; base0 += 64 * kPre) {
    int64_t a_pre[kPre];
    float2 q_pre[kPre];
    float d_pre[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int m = base0 + 64 * u + lane;
      a_pre[u] = (m < T) ? arow[(int64_t)m * st] : 0;  // m == T: back to the depot
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int m = base0 + 64 * u + lane;
      const int a32 = a_pre[u] >= 0 && a_pre[u] <= N ? (int)a_pre[u] : 0;
      q_pre[u] = lrow[m < M ? a32 : 0];
      d_pre[u] = check ? demand[b * (int64_t)N + (a32 > 0 ? a32 - 1 : 0)] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {  // wave-uniform trip count (ballot below)
      const int base = base0 + 64 * u;
      if (base >= M) break;
      const int m = base + lane;
      const int64_t a_to = a_pre[u];
      const bool ok_to = a_to >= 0 && a_to <= N;
      const int a32 = ok_to ? (int)a_to : -1;
      const float2 q = q_pre[u];
      int a_from = __shfl_up(a32, 1, 64);
      float px = __shfl_up(q.x, 1, 64), py = __shfl_up(q.y, 1, 64);
      if (lane == 0) {
        a_from = a_carry;
        px = px_carry;
        py = py_carry;
      }
      a_carry = __shfl(a32, 63, 64);
      px_carry = __shfl(q.x, 63, 64);
      py_carry = __shfl(q.y, 63, 64);
      if (m < M) {
        if (check && m < T && a_from == 0) start_here = true;  // step 0 or right after a depot
        if (a_from < 0 || !ok_to) {
          range = true;
        } else {
          acc += (double)edge_len(px, py, q.x, q.y);
        }
        if (check && m < T) {
          const int64_t a = a_to;  // = actions[m]
          if (!ok_to) {
            bad = true;
            dseq[m] = 0.f;
          } else {
            if (a != 0) {
              ++nonzero;
              const uint32_t bit = 1u << (a & 31);
              if (atomicOr(&bits[a >> 5], bit) & bit) bad = true;
            }
            dseq[m] = (a == 0) ? -cap : d_pre[u];
          }
        }
      }
      if (check) {  // route starts, in step order
        const uint64_t bal = __ballot(start_here);
        if (start_here)
          starts[nseg + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = m;
        nseg += __popcll(bal);
        start_here = false;
      }
    }
    }
    acc = wave_sum(acc);
    if (lane == 0) reward[b] = -(float)acc;
    if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    if (check) {
      nonzero = wave_sum(nonzero);
      const bool invalid = __any(bad) || nonzero != N;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (invalid) {
        if (lane == 0) set_status(status, CO_ST_INVALID_TOUR);
      } else {
        // cvrp/env.py:181-190: used = max(used + d_t, 0), over if !(used <= cap + 1e-5), a
        // sequential f32 scan.  Split at the routes (step 0 / a depot's next step through
        // the next depot): route k starts from the value route k-1 ends with, exactly 0
        // unless that route ended in (cap, cap + 1e-5] (f32 sums of demands often land a
        // hair above cap).  Each lane scans its routes -- the reference's f32 operations in
        // its order -- from the current start values; a route whose end differs from its
        // successor's start value updates it and the routes are scanned again, until no
        // start changes (one repeat per chain of residual routes).  Every pass's values are
        // <= the sequential ones (f32 add and max are monotone), so an overflow seen in any
        // pass is one the sequential scan sees, and the last pass is the sequential scan.
        const float lim = cap + 1e-5f;
        bool over = false;
        float* cur_v = sval;
        float* nxt_v = sval + T;
        for (int k = lane; k < nseg; k += 64) cur_v[k] = nxt_v[k] = 0.f;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#if !CO_CVRP_RCUT
        // an overflow is final (stop); a NaN demand overflows; at most nseg passes
        for (int pass = 0, again = 1; again && pass < nseg; ++pass) {
          bool changed = false;
          for (int k = lane; k < nseg; k += 64) {
            const int t0 = starts[k], t1 = k + 1 < nseg ? starts[k + 1] : T;
            float used = cur_v[k];
            // 8 steps per block, their LDS reads issued together; steps past the route add
            // +0.f (used >= 0 stays bit-identical up to the sign of a zero, which no
            // comparison sees)
            for (int t = t0; t < t1; t += 8) {
              float d[8];
#pragma unroll
              for (int i = 0; i < 8; ++i) d[i] = t + i < t1 ? dseq[t + i] : 0.f;
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                used += d[i];
                if (used < 0.f) used = 0.f;
                if (!(used <= lim)) over = true;
              }
            }
            if (k + 1 < nseg) {
              nxt_v[k + 1] = used;
              changed |= used != cur_v[k + 1];
            }
          }
          again = __any(changed) && !__any(over);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
          float* tmp = cur_v;
          cur_v = nxt_v;
          nxt_v = tmp;
        }
#endif
        over = __any(over);
        if (over && lane == 0) set_status(status, CO_ST_OVER_CAPACITY);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Reward + validity over step-major actions ([T, B] rows, what the stepwise episode
// records; any strides work): 64 consecutive instances per workgroup, lane = instance,
// so each action load of a wave is one coalesced 512-B piece of a row that no other
// workgroup touches.  The tile's [64, N+1] coordinates (and, with `check`, its [64, N]
// demand rows) are staged once into LDS by LDS-DMA.
// * Walker waves take U-step batches of action rows round-robin (walker p: batches p,
//   p + P, ...; a batch's first edge starts from the action before it, loaded with the
//   batch), double-buffered, and sum the edges (f32 per batch, f64 across batches); they
//   also flag out-of-range indices.  Round-robin keeps the walkers together on a short
//   window of steps that the scanner follows, so its re-reads of the same action lines
//   are L2 hits (contiguous per-walker ranges left most lines to be fetched twice).
// * With `check`, wave 0 is the scanner: it walks the whole episode in step order with
//   a two-stage pipeline (batch k+1's action rows in flight -- L2 hits after the walkers
//   -- while batch k is processed): marks the node in the instance's LDS visited words
//   (no-return ds_or; the permutation test is "N nonzero steps and N distinct bits"),
//   takes d_t from the LDS demand row (cvrp/env.py:177-178: -capacity at the depot) and
//   runs the reference's sequential f32 capacity scan (cvrp/env.py:180-190) in its exact
//   operation order.  Its serial chain overlaps the walkers instead of following them.
#ifndef CO_CVRPR_U
#define CO_CVRPR_U 4
#endif
#ifndef CO_CVRPR_Q
#define CO_CVRPR_Q 8
#endif
#ifndef CO_CVRPR_SU
#define CO_CVRPR_SU 8
#endif
struct CvrpRewardTile {  // LDS carve-up of cvrp_reward_tile_kernel (host + device)
  int NC, VW;
  size_t xy, dem, len, vis, ncap, total;
  __host__ __device__ CvrpRewardTile(int N, int Q, int check) {
    NC = N + 1;
    VW = ((N + 32) >> 5) | 1;  // visited words per instance (odd stride)
    const size_t dbytes = check ? (((size_t)64 * N * 4) + 15) & ~(size_t)15 : 0;
    const size_t lbytes = (size_t)Q * 64 * 8;
    size_t o = 0;
    xy = o;   o += (((size_t)64 * NC * 8) + 15) & ~(size_t)15;
    dem = len = o;  // the partial sums reuse the demand rows after the episode
    o += dbytes > lbytes ? dbytes : lbytes;
    vis = o;  o += check ? (size_t)64 * VW * 4 : 0;
    ncap = o; o += check ? 64 * 4 : 0;  // -vehicle_capacity per instance (depot's term)
    total = o;
  }
};

template <int Q>
__global__ __launch_bounds__(64 * Q) void cvrp_reward_tile_kernel(
    int64_t B, int N, int T, const float2* __restrict__ locs, const int64_t* __restrict__ acts,
    int64_t sb, int64_t st, const float* __restrict__ demand, const float* __restrict__ vcap,
    int check, float* __restrict__ reward, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const CvrpRewardTile L(N, Q, check);
  const int NC = N + 1;
  const float2* s_xy = reinterpret_cast<const float2*>(smem + L.xy);
  uint32_t* s_vis = reinterpret_cast<uint32_t*>(smem + L.vis);
  double* s_len = reinterpret_cast<double*>(smem + L.len);
  __shared__ float2 s_last[64];  // the point after step T-1 (closing edge)
  __shared__ int s_lok[64], s_range[64], s_cnt[64], s_over[64];
  const int lane = threadIdx.x & 63, q = wave_in_block();
  const int64_t row0 = (int64_t)blockIdx.x * 64;
  const int rows = (int)((B - row0) < 64 ? (B - row0) : 64);
  const bool live = lane < rows;
  const int64_t b = live ? row0 + lane : row0;  // dead lanes mirror lane 0's loads
  const int64_t* ap = acts + b * sb;             // this lane's column (row t at ap[t * st])
#ifdef CO_CVRPR_TIMING  // diagnostic: phase clocks of each workgroup into reward[row0 + i]
  __shared__ unsigned long long s_tm[8];
  const unsigned long long tm0 = __builtin_readcyclecounter();
  if (threadIdx.x < 8) s_tm[threadIdx.x] = 0;
#endif
  // roles; each issues its first action rows before the tiles are staged (the staging
  // helper's vmcnt(0) + barrier then covers them too)
  const bool scanner = check && q == 0;
  constexpr int SU = CO_CVRPR_SU, U = CO_CVRPR_U;
  const uint32_t* ap32 = reinterpret_cast<const uint32_t*>(ap);  // low dwords
  const int64_t st2 = st * 2;
  uint32_t a0[SU], a1[SU], a2[SU];
  auto sload = [&](uint32_t (&dst)[SU], int t0) {  // scanner rows, clamped into [0, T)
#pragma unroll
    for (int u = 0; u < SU; ++u) dst[u] = ap32[(int64_t)(t0 + u < T ? t0 + u : T - 1) * st2];
  };
  const int P = check ? Q - 1 : Q;  // walker waves
  const int p = check ? q - 1 : q;
  const int nbt = (T + U - 1) / U;  // U-step batches, walker p takes p, p + P, ...
  int64_t bufA[U], bufB[U], prevA = 0, prevB = 0;
  auto wload = [&](int64_t (&dst)[U], int64_t& prev, int j) {  // batch j (+ the step before)
    const int t0 = j * U;
    prev = t0 > 0 ? ap[(int64_t)(t0 - 1) * st] : 0;  // step 0 starts from the depot
#pragma unroll
    for (int u = 0; u < U; ++u) dst[u] = ap[(int64_t)(t0 + u < T ? t0 + u : T - 1) * st];
  };
  if (scanner) {
    sload(a0, 0);
    sload(a1, SU);
  } else if (p < nbt) {
    wload(bufA, prevA, p);
  }
  if (check)
    for (int k = threadIdx.x; k < 64 * L.VW; k += 64 * Q) s_vis[k] = 0u;
  if (threadIdx.x < 64) s_range[threadIdx.x] = s_cnt[threadIdx.x] = 0;
  if (check) {  // demand rows by LDS-DMA (walker waves), in flight with the coordinates
    const unsigned char* dsrc = reinterpret_cast<const unsigned char*>(demand + row0 * N);
    const int dbytes = rows * N * 4, d16 = dbytes & ~15;
    for (int base = (q - 1) * 1024; q > 0 && base < d16; base += (Q - 1) * 1024)
      if (base + lane * 16 < d16)
        __builtin_amdgcn_global_load_lds((const void*)(dsrc + base + lane * 16),
                                         (lds_void*)(smem + L.dem + base), 16, 0, CO_STAGE_AUX);
    for (int k = d16 + (int)threadIdx.x; k < dbytes; k += 64 * Q) smem[L.dem + k] = dsrc[k];
  }
  stage_bytes_lds(reinterpret_cast<const unsigned char*>(locs + row0 * NC), rows * NC * 8,
                  smem + L.xy);  // ends with vmcnt(0) + a barrier
  const float2* xy = s_xy + (size_t)lane * NC;
#ifdef CO_CVRPR_TIMING
  if (threadIdx.x == 0) s_tm[1] = __builtin_readcyclecounter() - tm0;
#endif
  double len = 0.0;
  if (scanner) {
    // ---- scanner (cvrp/env.py:177-190 in step order).  Only the low dword of each
    // action is read: an index outside [0, N] makes the tour invalid (the walkers flag
    // it), which overrides the capacity result, so it is only clamped here.  Node a's
    // demand term is one LDS read without a branch: a == 0 reads the lane's
    // -capacity slot instead of the demand row (cvrp/env.py:177).
    const unsigned dem_base = (unsigned)(L.dem + (size_t)lane * N * 4) - 4u;  // node a at +4a
    const unsigned cap_off = (unsigned)(L.ncap + lane * 4);
    const float cap = vcap[b];
    *reinterpret_cast<float*>(smem + cap_off) = -cap;
    const float lim = cap + 1e-5f;
    float used = 0.f;
    bool over = false;
    // cvrp/env.py:183-190 per step: used += d; used[used < 0] = 0; assert used <= cap +
    // 1e-5.  As max(used + d, 0) the chain is two dependent VALU ops; max differs from
    // the reference only for a NaN sum (the reference keeps NaN, which fails the assert),
    // so a NaN sum is flagged as an overflow directly -- an overflow is final.  Steps
    // past T (the last batch's padding) add +0.
    auto scan = [&](const uint32_t (&src)[SU], int t0) {
      float dv[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const uint32_t a = src[u] < (uint32_t)N ? src[u] : (uint32_t)N;
        dv[u] = *reinterpret_cast<const float*>(smem + (a == 0 ? cap_off : dem_base + a * 4u));
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const float t = used + (t0 + u < T ? dv[u] : 0.f);
        used = fmaxf(t, 0.f);
        over |= !(used <= lim) | (t != t);
      }
    };
    // three-deep batch pipeline: batches k+1 and k+2 in flight while k is scanned
    const int nb = (T + SU - 1) / SU;
    int k = 0;
    for (; k + 2 < nb; k += 3) {
      sload(a2, (k + 2) * SU);
      scan(a0, k * SU);
      sload(a0, (k + 3) * SU);
      scan(a1, (k + 1) * SU);
      sload(a1, (k + 4) * SU);
      scan(a2, (k + 2) * SU);
    }
    if (k < nb) scan(a0, k * SU);
    if (k + 1 < nb) scan(a1, (k + 1) * SU);
    s_over[lane] = over;
#ifdef CO_CVRPR_TIMING
    if (lane == 0) s_tm[2] = __builtin_readcyclecounter() - tm0;
#endif
  } else {
    // ---- walkers: edges (+ visited words) over round-robin U-step batches
    bool range = false;
    int nonzero = 0;
    uint32_t* vw = s_vis + lane * L.VW;
    auto run = [&](const int64_t (&src)[U], int64_t prev, int j) {
      const int t0 = j * U;
      const int cnt = T - t0 < U ? T - t0 : U;  // wave-uniform
      bool pok = prev >= 0 && prev <= N;  // the point before the batch
      float2 pt = xy[pok ? (int)prev : 0];
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < cnt) {
          const bool ok = src[u] >= 0 && src[u] <= N;
          const int a = ok ? (int)src[u] : 0;
          const float2 qq = xy[a];
          if (check) {  // no-return ds_or; node 0 (depot / out of range) is not counted
            __hip_atomic_fetch_or(&vw[a >> 5], 1u << (a & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            nonzero += a != 0;
          }
          if (pok && ok) {
            const float dx = qq.x - pt.x, dy = qq.y - pt.y;
            acc += sqrtf(dx * dx + dy * dy);
          }
          range |= !ok;
          pt = qq;
          pok = ok;
        }
      }
      len += (double)acc;
      if (t0 + cnt == T) {  // owner of the last step: the closing edge starts here
        s_last[lane] = pt;
        s_lok[lane] = pok;
      }
    };
    int j = p;
    for (; j + P < nbt; j += 2 * P) {
      wload(bufB, prevB, j + P);
      run(bufA, prevA, j);
      if (j + 2 * P < nbt) wload(bufA, prevA, j + 2 * P);
      run(bufB, prevB, j + P);
    }
    if (j < nbt) run(bufA, prevA, j);
    if (range) s_range[lane] = 1;
    if (check && nonzero) atomicAdd(&s_cnt[lane], nonzero);
#ifdef CO_CVRPR_TIMING
    if (lane == 0) atomicMax(&s_tm[3], __builtin_readcyclecounter() - tm0);
#endif
  }
  const float2 dep = xy[0];
  __syncthreads();  // episode walked: the demand rows are free for the partial sums
  s_len[q * 64 + lane] = len;  // the scanner's entry is 0
  __syncthreads();
  if (q == 0) {
    const bool rng = live && s_range[lane];
    if (live) {
      double tot = 0.0;
#pragma unroll
      for (int w = 0; w < Q; ++w) tot += s_len[w * 64 + lane];
      if (s_lok[lane]) tot += (double)edge_len(s_last[lane].x, s_last[lane].y, dep.x, dep.y);
      reward[b] = -(float)tot;
    }
    // status bits are batch-wide: one atomic per bit per workgroup
    if (__any(rng) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    if (check) {  // a permutation of 1..N among the steps: N nonzero steps, N distinct bits
      const uint32_t* vw = s_vis + lane * L.VW;
      int bits = -(int)(vw[0] & 1u);  // node 0 (the depot) is not a customer
      for (int w = 0; w < L.VW; ++w) bits += __popc(vw[w]);
      const bool invalid = live && (rng || s_cnt[lane] != N || bits != N);
      const bool ovr = live && !invalid && s_over[lane];
      if (__any(invalid) && lane == 0) set_status(status, CO_ST_INVALID_TOUR);
      if (__any(ovr) && lane == 0) set_status(status, CO_ST_OVER_CAPACITY);
    }
#ifdef CO_CVRPR_TIMING
    if (lane == 0) s_tm[4] = __builtin_readcyclecounter() - tm0;
    if (lane < 5 && lane < rows) reward[row0 + lane] = (float)s_tm[lane];
#endif
  }
}

}  // namespace

extern "C" int co_cvrp_reset(int64_t B, int64_t N, const float* depot, const float* locs_in,
                             const float* demand, float vcap, float* locs_out, int64_t* cur,
                             float* used, float* vcap_out, uint8_t* visited, uint8_t* mask,
                             void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!depot || !locs_in || !demand || !locs_out || !cur || !used || !vcap_out || !visited ||
      !mask)
    return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(depot) | reinterpret_cast<uintptr_t>(locs_in) |
       reinterpret_cast<uintptr_t>(locs_out)) & 7)
    return CO_E_ALIGN;
  hipLaunchKernelGGL(cvrp_reset_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, reinterpret_cast<const float2*>(depot),
                     reinterpret_cast<const float2*>(locs_in), demand, vcap,
                     reinterpret_cast<float2*>(locs_out), cur, used, vcap_out, visited, mask);
  return launch_status();
}

extern "C" int co_cvrp_step(int64_t B, int64_t N, const int64_t* action, const float* demand,
                            const float* used_in, float* used_out, const float* vcap,
                            const uint8_t* vis_in, uint8_t* vis_out, int64_t* cur_out,
                            uint8_t* done, uint8_t* reward, uint8_t* mask, int32_t* status,
                            int32_t* not_done, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !demand || !used_in || !used_out || !vcap || !vis_in || !vis_out || !done ||
      !reward || !mask)
    return CO_E_INVAL;
  // 256-thread tiles of R = min(64, 8192 / (N+1)) & ~15 rows (single-wave 16-row tiles
  // measured slower at N = 100: 16.3 vs 12.2 us per step at B = 32,768)
  const int64_t NC = N + 1;
  const bool aligned = ((reinterpret_cast<uintptr_t>(vis_in) | reinterpret_cast<uintptr_t>(vis_out) |
                         reinterpret_cast<uintptr_t>(mask) | reinterpret_cast<uintptr_t>(demand)) &
                        15) == 0;
  // row-group kernel: 4-byte-aligned byte rows and demand
  const bool rows_ok =
      N >= 3 && N <= 252 &&
      ((reinterpret_cast<uintptr_t>(vis_in) | reinterpret_cast<uintptr_t>(vis_out) |
        reinterpret_cast<uintptr_t>(mask) | reinterpret_cast<uintptr_t>(demand)) & 3) == 0;
  constexpr int G = CO_CVRP_G, Q = CO_CVRP_Q;
  // dwords per lane: ceil(ceil((N+4)/4) / G), at most 4
  const int kpl = (int)((NC + 6) / 4 + G - 1) / G;
  if (CO_CVRP_QUAD && rows_ok && kpl <= 4) {
    // 16 waves per workgroup when the not-done counter is wanted (fewer atomics), else 4
    const int waves = not_done ? 16 : 4;
    const int64_t rows_per_wg = (int64_t)(64 / G) * Q * waves;
    const int64_t wgs = (B + rows_per_wg - 1) / rows_per_wg;
    const unsigned grid = cover_grid(wgs, 1, 64 * waves);
    if (grid == 0) return CO_E_INVAL;
    hipStream_t s = (hipStream_t)stream;
#define CO_CQ(K, W)                                                                         \
  hipLaunchKernelGGL((cvrp_step_rows_kernel<G, K, Q, W>), dim3(grid), dim3(64 * W), 0, s, B,  \
                     (int)N, action, demand, used_in, used_out, vcap, vis_in, vis_out, cur_out, \
                     done, reward, mask, status, not_done)
#define CO_CQK(W)                 \
  if (kpl == 1) CO_CQ(1, W);      \
  else if (kpl == 2) CO_CQ(2, W); \
  else if (kpl == 3) CO_CQ(3, W); \
  else CO_CQ(4, W);
    if (waves == 16) {
      CO_CQK(16)
    } else {
      CO_CQK(4)
    }
#undef CO_CQK
#undef CO_CQ
    return launch_status();
  }
  int R = (int)((256 * kCvrpCpt * 16) / NC);
  R = (R > kCvrpMaxRows ? kCvrpMaxRows : R) & ~15;
  if (N >= 16 && aligned && R >= 16 && (size_t)R * N * sizeof(float) + 16 <= 64 * 1024) {
    const unsigned grid = cover_grid(B, R);
    if (grid == 0) return CO_E_INVAL;
    hipLaunchKernelGGL(cvrp_step_tile_kernel<256>, dim3(grid), dim3(256),
                       (size_t)R * N * sizeof(float) + 16, (hipStream_t)stream, B, (int)N, R, action,
                       demand, used_in, used_out, vcap, vis_in, vis_out, cur_out, done, reward,
                       mask, status, not_done);
    return launch_status();
  }
  hipLaunchKernelGGL(cvrp_step_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, action, demand, used_in, used_out, vcap,
                     vis_in, vis_out, cur_out, done, reward, mask, status, not_done);
  return launch_status();
}

extern "C" int co_cvrp_action_mask(int64_t B, int64_t N, const float* demand, const float* used,
                                   const float* vcap, const uint8_t* visited, const int64_t* cur,
                                   uint8_t* mask, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!demand || !used || !vcap || !visited || !cur || !mask) return CO_E_INVAL;
  hipLaunchKernelGGL(cvrp_mask_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, demand, used, vcap, visited, cur, mask);
  return launch_status();
}

extern "C" int co_cvrp_reward(int64_t B, int64_t N, int64_t T, const float* locs,
                              const int64_t* actions, int64_t sb, int64_t st,
                              const float* demand, const float* vcap, int check, float* reward,
                              int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || T <= 0 || T > (1 << 20)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !actions || !reward) return CO_E_INVAL;
  if (check && (!demand || !vcap || !status)) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  // step-major actions (or a row-major episode too long for the wave-per-instance
  // kernel's LDS sequence) and a 16-B aligned coordinate tensor: the tile kernel
  constexpr int kQ = CO_CVRPR_Q;
  const size_t per_wave = check ? (size_t)((N + 32) / 32 + 4 * T) * 4 : 0;
  const bool step_major = sb == 1 && st == B;
  const size_t tile_lds = CvrpRewardTile((int)N, kQ, check).total;
  if ((step_major || per_wave > 64 * 1024) &&
      ((reinterpret_cast<uintptr_t>(locs) | (check ? reinterpret_cast<uintptr_t>(demand) : 0)) &
       15) == 0 &&
      tile_lds <= 80 * 1024) {
    hipLaunchKernelGGL(cvrp_reward_tile_kernel<kQ>, dim3((unsigned)((B + 63) / 64)),
                       dim3(64 * kQ), tile_lds, (hipStream_t)stream, B, (int)N, (int)T,
                       reinterpret_cast<const float2*>(locs), actions, sb, st, demand, vcap,
                       check, reward, status);
    return launch_status();
  }
  // row-major actions: one wave per instance, lanes over steps (coalesced rows)
  int waves = 4;
  while (waves > 1 && per_wave * waves > 64 * 1024) waves >>= 1;
  if (per_wave > 64 * 1024) return CO_E_INVAL;
  const size_t shmem = per_wave * waves;
  const dim3 grid(grid_for(B, waves, 256 * 32));
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  switch (waves) {
    case 4:
      hipLaunchKernelGGL(cvrp_reward_kernel<4>, grid, dim3(256), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
    case 2:
      hipLaunchKernelGGL(cvrp_reward_kernel<2>, grid, dim3(128), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
    default:
      hipLaunchKernelGGL(cvrp_reward_kernel<1>, grid, dim3(64), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
  }
  return launch_status();
}

extern "C" int co_cvrp_nearest_action(int64_t B, int64_t N, const float* locs,
                                      const uint8_t* mask, const int64_t* cur, int64_t* out,
                                      void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !mask || !cur || !out) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  const hipStream_t s = (hipStream_t)stream;
#define CO_CNG(GG, KK)                                                                  \
  hipLaunchKernelGGL((cvrp_nearest_group_kernel<GG, KK>),                             \
                     dim3(grid_for(B, 4 * (64 / GG), 256 * 32)), dim3(256), 0, s, B, (int)N, l2, \
                     mask, cur, out)
  if (N <= 64) CO_CNG(8, 8);
  else if (N <= 160) CO_CNG(16, 10);
  else if (N <= 320) CO_CNG(32, 10);
  else CO_CNG(64, 0);
#undef CO_CNG
  return launch_status();
}

extern "C" int co_cvrp_nearest_step(int64_t B, int64_t N, const float* locs, const float* demand,
                                    const float* used_in, float* used_out, const float* vcap,
                                    const uint8_t* vis_in, uint8_t* vis_out,
                                    const uint8_t* mask_in, const int64_t* cur_in,
                                    int64_t* action_out, int64_t* cur_out, uint8_t* done,
                                    uint8_t* reward, uint8_t* mask_out, int32_t* status,
                                    int32_t* not_done, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !demand || !used_in || !used_out || !vcap || !vis_in || !vis_out || !mask_in ||
      !cur_in || !action_out || !cur_out || !done || !reward || !mask_out)
    return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  if (N + 1 > 16 * 8) {  // the two launches it fuses
    int rc = co_cvrp_nearest_action(B, N, locs, mask_in, cur_in, action_out, stream);
    if (rc != CO_OK) return rc;
    return co_cvrp_step(B, N, action_out, demand, used_in, used_out, vcap, vis_in, vis_out,
                        cur_out, done, reward, mask_out, status, not_done, stream);
  }
  // 16-B chunk access when every byte tile starts 16-B aligned (16 x (N+1) bytes per tile)
  const bool vec = ((reinterpret_cast<uintptr_t>(vis_in) | reinterpret_cast<uintptr_t>(vis_out) |
                     reinterpret_cast<uintptr_t>(mask_in) |
                     reinterpret_cast<uintptr_t>(mask_out)) & 15) == 0;
  const int64_t tiles = (B + kCnsRows - 1) / kCnsRows;
  const dim3 grid((unsigned)(tiles < 65536 ? tiles : 65536));
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  hipStream_t s = (hipStream_t)stream;
#define CO_CNS(KM)                                                                            \
  hipLaunchKernelGGL((cvrp_nearest_step_kernel<KM>), grid, dim3(256), 0, s, B, (int)N, l2,     \
                     demand, used_in, used_out, vcap, vis_in, vis_out, mask_in, cur_in,        \
                     action_out, cur_out, done, reward, mask_out, vec, not_done)
  const int km = (int)((N + 1 + 15) / 16);
  if (km <= 2) CO_CNS(2);
  else if (km <= 4) CO_CNS(4);
  else if (km <= 7) CO_CNS(7);
  else CO_CNS(8);
#undef CO_CNS
  return launch_status();
}
