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
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
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
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
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
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
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

__global__ __launch_bounds__(256) void cvrp_mask_kernel(int64_t B, int N, const float* demand,
                                                        const float* used, const float* vcap,
                                                        const uint8_t* visited,
                                                        const int64_t* cur, uint8_t* mask) {
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
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
  const int w = threadIdx.x >> 6, lane = lane_id();
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
    for (int base = 0; base < M; base += 64) {  // wave-uniform trip count (ballot below)
      const int m = base + lane;
      const int64_t a_to = (m < T) ? arow[(int64_t)m * st] : 0;  // m == T: back to the depot
      const bool ok_to = a_to >= 0 && a_to <= N;
      const int a32 = ok_to ? (int)a_to : -1;
      const float2 q = lrow[ok_to && m < M ? a32 : 0];
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
            dseq[m] = (a == 0) ? -cap : demand[b * (int64_t)N + a - 1];
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
  int R = (int)((256 * kCvrpCpt * 16) / NC);
  R = (R > kCvrpMaxRows ? kCvrpMaxRows : R) & ~15;
  if (N >= 16 && aligned && R >= 16 && (size_t)R * N * sizeof(float) + 16 <= 64 * 1024) {
    const unsigned grid = (unsigned)((B + R - 1) / R);
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
  const size_t per_wave = check ? (size_t)((N + 32) / 32 + 4 * T) * 4 : 0;
  // step-major actions ([T, B] rows): 16 consecutive instances per workgroup, so each
  // 128-B line of an action row is consumed on one CU (4 per workgroup spread a line over
  // 4 XCDs' L2s: 160 MB read per launch at B = 32,768, T = 112, vs ~70 MB algorithmic)
  int waves = (sb == 1 && st == B) ? 16 : 4;
  while (waves > 1 && per_wave * waves > 64 * 1024) waves >>= 1;
  if (per_wave > 64 * 1024) return CO_E_INVAL;
  const size_t shmem = per_wave * waves;
  const dim3 grid(grid_for(B, waves, 256 * 32));
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  switch (waves) {
    case 16:
      hipLaunchKernelGGL(cvrp_reward_kernel<16>, grid, dim3(1024), shmem, (hipStream_t)stream,
                         B, (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
    case 8:
      hipLaunchKernelGGL(cvrp_reward_kernel<8>, grid, dim3(512), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
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
