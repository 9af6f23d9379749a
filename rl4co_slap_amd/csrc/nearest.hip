// Fused nearest-policy episodes for gfx950: the whole env-only rollout
// (rl4co/utils/decoding.py:88-109) of TSP (tsp/env.py:67-173) and CVRP
// (cvrp/env.py:73-190) with the nearest-node bench policy of SURVEY.md 8d in-kernel.
//
// Layout: a G-lane group per instance, 64/G instances per wavefront.  Lane `sl` of
// the group keeps nodes c = sl + G*k (k < EPL) in VGPRs for the whole episode:
// coordinates, CVRP demand, and a visited bit per node.  One policy step is EPL
// squared distances per lane (one sqrt), a DPP / permlane-swap argmin over the group and
// three lane broadcasts (x, y, demand of the chosen node); nothing is read from
// memory after the first load and the only per-step store is the step-major action.
// The oracle's policy (oracle/envs.py tsp_nearest_action / cvrp_nearest_action):
// argmin over feasible nodes of f32 sqrt(dx*dx + dy*dy), ties -> lowest index.
#include "co_common.hpp"

using namespace co;

namespace {

constexpr int kNoNode = 0x7fffffff;

#ifndef CO_NEAREST_LDS
#define CO_NEAREST_LDS 1  // 0: the register engines (coordinates in VGPRs, a visited bit mask)
#endif

#ifndef CO_NEAREST_LDS_G
#define CO_NEAREST_LDS_G 4  // TSP N <= 104: lanes per instance (4 x 26 slots, or 8 x 14)
#endif
#ifndef CO_NEAREST_CVRP_G
#define CO_NEAREST_CVRP_G 8  // CVRP N + 1 <= 112: lanes per instance (4 x 28 or 8 x 14 slots)
#endif

#ifndef CO_NEAREST_G8
#define CO_NEAREST_G8 0  // 1: 8 lanes x 13 slots per instance for N (+1) <= 104 (payload by shuffle)
#endif

// a constant materialised in a scalar register at its use (an empty asm with an "s"
// operand): hoisted out of the step loop, the loop's constants otherwise hold VGPRs for
// the whole kernel, and the CVRP episode needs <= 64 of them for 8 waves per SIMD
__device__ __forceinline__ uint32_t su(uint32_t c) {
  asm volatile("" : "+s"(c));
  return c;
}

// Lane-local nearest candidate: argmin over the candidates (bit k of `cand`) of the f32
// distance sqrt(dx*dx + dy*dy), ties -> lowest node index, exactly as torch.argmin over
// the oracle's distances.  The scan compares squared distances (the same IEEE products
// and sum) and takes one correctly rounded sqrt, of the minimum.  A larger squared
// distance can round to the same sqrt only within a relative 2^-22; a lower-index
// candidate inside that window is resolved with its own sqrt in a branch that is almost
// never taken.  Returns (+inf, kNoNode) when there is no candidate.
template <int G, int EPL>
__device__ __forceinline__ void lane_nearest(float cx, float cy, const float (&px)[EPL],
                                             const float (&py)[EPL], uint32_t cand, int sl,
                                             float& best, int& bi) {
  float sq[EPL];
  float smin = __builtin_inff(), sbef = __builtin_inff();
  int kmin = -1;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const float dx = px[k] - cx, dy = py[k] - cy;
    sq[k] = dx * dx + dy * dy;
    const bool take = ((cand >> k) & 1u) && sq[k] < smin;
    sbef = take ? smin : sbef;  // running min of the candidates before the new best
    smin = take ? sq[k] : smin;
    kmin = take ? k : kmin;
  }
  best = kmin >= 0 ? sqrtf(smin) : __builtin_inff();
  bi = kmin >= 0 ? sl + G * kmin : kNoNode;
  const float win = smin * (1.0f + 0x1p-20f);
  // sbef = min over the candidates with k < kmin: one compare instead of an EPL-wide test
  if (kmin >= 0 && sbef <= win) {  // rare: an earlier node whose distance rounds to the same sqrt
    int kk = kmin;
#pragma unroll
    for (int k = EPL - 1; k >= 0; --k)
      if (((cand >> k) & 1u) && k < kmin && sq[k] <= win && sqrtf(sq[k]) == best) kk = k;
    bi = sl + G * kk;
  }
}

// The group's nearest candidate, exactly as lane_nearest + grp_argmin_split, with the
// common case on squared distances only: each lane scans its candidates once (the first
// index of its smallest squared distance, strict <, and sbef = the smallest before it),
// the group min of the squared distances is one integer DPP min per stage (non-negative
// f32 order as their bit patterns), and the winner is the lowest node index holding it.
// The f32 sqrt can merge squared distances within a relative 2^-22: when some candidate
// other than the winner lies within 2^-20 of the minimum at a lower index, or before its
// lane's best (rare), the wave redoes the step with the per-lane correctly rounded sqrt
// (lane_nearest, grp_argmin_split).  Returns the winning node (kNoNode: no candidate)
// and its squared distance m (+inf: none); every lane of the wave must take part.
template <int G, int EPL>
__device__ __forceinline__ int grp_nearest(float cx, float cy, const float (&px)[EPL],
                                           const float (&py)[EPL], uint32_t cand, int sl,
                                           float& m) {
  const float inf = __uint_as_float(su(0x7f800000u));
  float smin = inf, sbef = inf;
  int kmin = -1;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const float dx = px[k] - cx, dy = py[k] - cy;
    const float sq = dx * dx + dy * dy;
    const bool take = ((cand >> k) & 1u) && sq < smin;
    sbef = take ? smin : sbef;
    smin = take ? sq : smin;
    kmin = take ? k : kmin;
  }
  const uint32_t mb = grp_reduce<G>(__float_as_uint(smin), [](uint32_t a, uint32_t b) {
    return a < b ? a : b;
  });
  const int none = (int)su((uint32_t)kNoNode);
  const int my = kmin >= 0 ? sl + G * kmin : none;
  int w = grp_min_int<G>(__float_as_uint(smin) == mb ? my : none);
  m = __uint_as_float(mb);
  const float win = m * (1.0f + 0x1p-20f);
  const bool near = mb < su(0x7f800000u) && ((smin <= win && my < w) || sbef <= win);
  if (__builtin_expect(__any(near), 0)) {  // a tie of the rounded distances: exact path
    float best;
    int bi;
    lane_nearest<G, EPL>(cx, cy, px, py, cand, sl, best, bi);
    grp_argmin_split<G>(best, bi);
    w = bi;  // m stays: the winner's distance rounds to sqrtf(m)
  }
  return w;
}

// grp_nearest that also hands every lane of the group the winner's coordinates (and, DEM,
// its demand): each lane keeps the payload of its own best candidate during the scan (one
// select per value and candidate) and the owner's is read by one lane shuffle -- no LDS
// row per instance (the G = 8 engines: 13 slots per lane, whose LDS rows would cap the
// occupancy).  The rare exact path selects the owner's payload by slot.
template <int G, int EPL, bool DEM>
__device__ __forceinline__ int grp_nearest_x(float cx, float cy, const float (&px)[EPL],
                                             const float (&py)[EPL], const float (&dm)[EPL],
                                             uint32_t cand, int sl, int gbase, float& m,
                                             float& wx, float& wy, float& wd) {
  const float inf = __uint_as_float(su(0x7f800000u));
  float smin = inf, sbef = inf, bx = 0.f, by = 0.f, bd = 0.f;
  int kmin = -1;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const float dx = px[k] - cx, dy = py[k] - cy;
    const float sq = dx * dx + dy * dy;
    const bool take = ((cand >> k) & 1u) && sq < smin;
    sbef = take ? smin : sbef;
    smin = take ? sq : smin;
    kmin = take ? k : kmin;
    bx = take ? px[k] : bx;
    by = take ? py[k] : by;
    if (DEM) bd = take ? dm[k] : bd;
  }
  const uint32_t mb = grp_reduce<G>(__float_as_uint(smin), [](uint32_t a, uint32_t b) {
    return a < b ? a : b;
  });
  const int none = (int)su((uint32_t)kNoNode);
  const int my = kmin >= 0 ? sl + G * kmin : none;
  int w = grp_min_int<G>(__float_as_uint(smin) == mb ? my : none);
  m = __uint_as_float(mb);
  const float win = m * (1.0f + 0x1p-20f);
  const bool near = mb < su(0x7f800000u) && ((smin <= win && my < w) || sbef <= win);
  if (__builtin_expect(__any(near), 0)) {  // a tie of the rounded distances: exact path
    float best;
    int bi;
    lane_nearest<G, EPL>(cx, cy, px, py, cand, sl, best, bi);
    grp_argmin_split<G>(best, bi);
    w = bi;
    const int slot = (w == kNoNode ? 0 : w) / G;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      bx = k == slot ? px[k] : bx;
      by = k == slot ? py[k] : by;
      if (DEM) bd = k == slot ? dm[k] : bd;
    }
  }
  const int src = gbase + (w == none ? 0 : w % G);
  wx = __shfl(bx, src, 64);
  wy = __shfl(by, src, 64);
  if (DEM) wd = __shfl(bd, src, 64);
  return w;
}

// The group's value from lane `owner` (`v` of the other lanes is ignored): an OR over the
// group of the owner's bits, DPP only.
template <int G>
__device__ __forceinline__ float grp_from(float v, bool mine) {
  return __uint_as_float(grp_reduce<G>(mine ? __float_as_uint(v) : 0u,
                                       [](uint32_t a, uint32_t b) { return a | b; }));
}

// TSP: step 0 takes node 0, steps 1..N-1 the nearest unvisited node.  One group of G
// lanes per instance, 64/G per wave, one wave's instances per 64/G rows of the grid (no
// grid-stride loop: nothing is hoisted across instances, so the kernel stays within 64
// VGPRs -- 8 waves per SIMD); the group's coordinate row in LDS (8 B per node) gives the
// chosen node's coordinates as one broadcast read.
template <int G, int EPL, bool TR>
__global__ __launch_bounds__(256) void tsp_nearest_episode_kernel(
    int64_t B, int N, const float2* __restrict__ locs, int64_t* __restrict__ acts_out,
    uint8_t* __restrict__ mask_out, int64_t* __restrict__ first_out,
    int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out) {
  constexpr int IPW = 64 / G;
  __shared__ float2 s_xy[TR ? 1 : 256 * EPL];  // TR: the payload comes by lane shuffle
  const int lane = lane_id(), sl = lane % G;
  float2* xyg = s_xy + (TR ? 0 : (threadIdx.x / G) * (G * EPL));
  const int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * IPW;
  if (base >= B) return;  // wave-uniform
  const int64_t b = base + lane / G;
  const bool valid = b < B;
  const int64_t bb = valid ? b : B - 1;  // a dead group mirrors the last instance
  const float2* lrow = locs + bb * N;
  float px[EPL], py[EPL], nod[EPL];
  uint32_t vis = 0;  // bit k: node sl + G*k visited (or past N)
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
    const float2 q = c < N ? lrow[c] : make_float2(0.f, 0.f);
    px[k] = q.x;
    py[k] = q.y;
    if (!TR) xyg[c] = q;
    if (c >= N) vis |= 1u << k;
  }
  // the row is written and read by lanes of this wave only: a wave-level fence
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (sl == 0) vis |= 1u;  // step 0: node 0
  const float x0 = px[0], y0 = py[0];  // node 0 is lane 0's slot 0: broadcast it
  float cx = __shfl(x0, lane - sl, 64), cy = __shfl(y0, lane - sl, 64);
  const float fx = cx, fy = cy;
  if (valid && sl == 0) acts_out[bb] = 0;
  double len = 0.0;
  int cur = 0;
  for (int t = 1; t < N; ++t) {
    float m;
    int a;  // t < N: an unvisited node is left
    if (TR) {
      float wd;
      a = grp_nearest_x<G, EPL, false>(cx, cy, px, py, nod, ~vis, sl, lane - sl, m, cx, cy, wd);
    } else {
      a = grp_nearest<G, EPL>(cx, cy, px, py, ~vis, sl, m);
      const float2 q = xyg[a];
      cx = q.x;
      cy = q.y;
    }
    if (sl == a % G) vis |= 1u << (a / G);
    len += (double)__builtin_sqrtf(m);
    cur = a;
    if (valid && sl == 0) acts_out[(int64_t)t * B + bb] = a;
  }
  len += (double)edge_len(cx, cy, fx, fy);
  if (!valid) return;
  uint8_t* mrow = mask_out + bb * N;
  for (int c = sl; c < N; c += G) mrow[c] = 0;  // every node visited
  if (sl == 0) {
    first_out[bb] = 0;
    cur_out[bb] = cur;
    i_out[bb] = N;
    done_out[bb] = 1;
    step_reward_out[bb] = 0;
    reward_out[bb] = -(float)len;
  }
}

// CVRP: nodes 0..N (0 = depot).  Each step the nearest customer that is unvisited and
// fits (!(demand + used > capacity), cvrp/env.py:140), else the depot; the env
// transition of cvrp/env.py:73-105 on group-uniform scalars: used = (used + d) *
// (a != 0), done = every node visited (visited.sum == N + 1, so the depot must have
// been entered once).  A finished instance stops; co_cvrp_rollout's pad pass then
// applies the reference's remaining depot steps up to the batch-wide episode length.
// Coordinates and demand in VGPRs; the chosen node's coordinates from the group's LDS
// row (8 B per node: with 4 KB of LDS per wave, 8 waves fit per SIMD), its demand from
// the owner lane's register by a group OR.
template <int G, int EPL, bool TR>
__global__ __launch_bounds__(256) void cvrp_nearest_episode_kernel(
    int64_t B, int N, const float2* __restrict__ depot, const float2* __restrict__ locs_in,
    const float* __restrict__ demand, float vcap, int max_steps, int64_t* __restrict__ acts_out,
    float2* __restrict__ locs_out, int64_t* __restrict__ cur_out, float* __restrict__ used_out,
    float* __restrict__ vcap_out, uint8_t* __restrict__ visited_out,
    uint8_t* __restrict__ mask_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out,
    int32_t* __restrict__ len_out, int32_t* __restrict__ tmax, int32_t* status) {
  constexpr int IPW = 64 / G;
  __shared__ float2 s_xy[TR ? 1 : 256 * EPL];  // TR: the payload comes by lane shuffle
  const int lane = lane_id(), sl = lane % G, gbase = lane - sl;
  float2* xyg = s_xy + (TR ? 0 : (threadIdx.x / G) * (G * EPL));
  const int M = N + 1;
  const int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * IPW;
  if (base >= B) return;  // wave-uniform
  const int64_t b = base + lane / G;
  const bool valid = b < B;
  const int bb = (int)(valid ? b : B - 1);  // a dead group mirrors the last instance
  const float2* lrow = locs_in + (int64_t)bb * N;
  const float* drow = demand + (int64_t)bb * N;
  const float2 dep = depot[bb];
  float px[EPL], py[EPL], dm[EPL];
  uint32_t vis = 0;  // bit k: node sl + G*k visited (or past N)
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
    float2 q = make_float2(0.f, 0.f);
    float d = 0.f;
    if (c == 0) {
      q = dep;
    } else if (c <= N) {
      q = lrow[c - 1];
      d = drow[c - 1];
    }
    px[k] = q.x;
    py[k] = q.y;
    dm[k] = d;
    if (!TR) xyg[c] = q;
    if (c > N) vis |= 1u << k;
    if (valid && locs_out && c <= N) locs_out[(int64_t)bb * M + c] = q;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float cx = dep.x, cy = dep.y, used = 0.f;
  // packed group-uniform counters (register pressure: 8 waves per SIMD need <= 64 VGPRs):
  // st = customers visited (bits 0-15) | steps taken (bits 16-30) | depot entered (bit 31)
  uint32_t st = 0;
  int cur = 0;
  bool done = false;
  double dist = 0.0;
  for (int t = 0; t < max_steps; ++t) {
    if (__ballot(!done) == 0) break;  // wave-uniform: the group reductions need every lane
    uint32_t cand = 0;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const int c = sl + G * k;
      const bool feas = c >= 1 && !((vis >> k) & 1u) && !(dm[k] + used > vcap);
      cand |= (uint32_t)feas << k;
    }
    float m, ad;
    int a;
    float2 q;
    if (TR) {
      float wx, wy;
      const int bi = grp_nearest_x<G, EPL, true>(cx, cy, px, py, dm, cand, sl, gbase, m, wx, wy,
                                                 ad);
      a = bi == kNoNode ? 0 : bi;
      q = a == 0 ? dep : make_float2(wx, wy);
    } else {
      const int bi = grp_nearest<G, EPL>(cx, cy, px, py, cand, sl, m);
      a = bi == kNoNode ? 0 : bi;
      const int slot = a / G;
      float dsel = 0.f;  // the owner lane's demand of node a
#pragma unroll
      for (int k = 0; k < EPL; ++k) dsel = k == slot ? dm[k] : dsel;
      ad = grp_from<G>(dsel, sl == a % G);
      q = xyg[a];
    }
    if (done) continue;
    if (sl == a % G) vis |= 1u << (a / G);
    const float dx = q.x - cx, dy = q.y - cy;  // = m for a customer (same operations)
    dist += (double)__builtin_sqrtf(dx * dx + dy * dy);
    used = a != 0 ? (used + ad) * 1.0f : 0.0f;  // cvrp/env.py:83-85
    st = ((st & 0x8000ffffu) + (a != 0 ? 1u : 0u)) | ((uint32_t)(t + 1) << 16) |
         (a == 0 ? 0x80000000u : 0u);
    cur = a;
    cx = q.x;
    cy = q.y;
    if (valid && sl == 0) acts_out[(int64_t)t * B + bb] = a;
    done = (st & 0x8000ffffu) == (0x80000000u | (uint32_t)N);
  }
  const int len = (int)((st >> 16) & 0x7fffu);
  dist += (double)edge_len(cx, cy, dep.x, dep.y);  // closing edge to the depot
  // final state rows: visited and get_action_mask (cvrp/env.py:137-149)
  bool any_feas = false;
  uint8_t* vrow = visited_out + (int64_t)bb * M;
  uint8_t* mrow = mask_out + (int64_t)bb * M;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = sl + G * k;
    const bool v = (vis >> k) & 1u;
    const bool feas = c >= 1 && c <= N && !v && !(dm[k] + used > vcap);
    any_feas |= feas;
    if (valid && c <= N) {
      vrow[c] = v;
      if (c >= 1) mrow[c] = feas;
    }
  }
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
  const bool anyf = (__ballot(any_feas) & gmask) != 0;
  if (valid && sl == 0) {
    mrow[0] = !((cur == 0) && anyf);
    cur_out[bb] = cur;
    used_out[bb] = used;
    vcap_out[bb] = vcap;
    done_out[bb] = done;
    step_reward_out[bb] = 0;
    reward_out[bb] = -(float)dist;
    len_out[bb] = len;
    if (!done) set_status(status, CO_ST_TRUNCATED);
    atomicMax(tmax, len);
  }
}

// The reference keeps stepping finished instances until every instance is done
// (constructive/base.py:230): their action is the depot (no customer fits), which
// sets current_node = 0 and used_capacity = 0 and leaves visited / the mask as they
// are.  Pads actions [len_b, T) with 0 and applies that state.
__global__ __launch_bounds__(256) void cvrp_pad_kernel(int64_t B, const int32_t* __restrict__ len,
                                                       const int32_t* __restrict__ tmax,
                                                       int64_t* __restrict__ acts_out,
                                                       int64_t* __restrict__ cur_out,
                                                       float* __restrict__ used_out) {
  const int T = *tmax;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const int L = len[b];
    for (int t = L; t < T; ++t) acts_out[(int64_t)t * B + b] = 0;
    if (L < T) {
      cur_out[b] = 0;
      used_out[b] = 0.f;
    }
  }
}

inline unsigned group_grid(int64_t B, int G) {  // a wave per 64/G instances, covering B
  return cover_grid((B * G + 63) / 64, 4);
}

// ---------------------------------------------------------------------------------------
// LDS-row episodes (the default engines).  The per-step cost of the register engines above
// is the per-candidate VALU work: two subtractions, two products, a sum, the visited /
// capacity bit test and four selects per node.  Here each lane keeps its slots' y (and CVRP
// demand) in registers as pairs, and the instance's x row lives in LDS, slot pairs
// (x_k, x_k+1) of its G lanes adjacent; a visited node (and every padding slot, and the CVRP
// depot) has x = NaN, so its distance is NaN and it can never be the minimum -- visiting is
// one LDS store instead of a per-candidate test.  Per pair of candidates: one 8-byte LDS
// read, five packed f32 operations (v_pk_add / v_pk_mul: the same IEEE operations, two
// slots at a time), and per candidate a key = the squared distance's bits with the low KB
// bits replaced by the slot (one v_and_or) folded into the lane's two smallest keys
// (v_med3_u32 + v_min_u32, two independent chains).  The group merges (min, second min)
// pairs over DPP, and the winner is exact without a sqrt per candidate:
//   keys compare as (truncated squared distance, node); with T = the squared distance's
//   bits with the low BB bits cleared (a relative error below 2^(BB-23)), if the second
//   smallest key's T exceeds the winner's T by a factor 1 + 2^(BB-20), every other
//   candidate's squared distance is above the winner's by more than a factor
//   1 + 2^(BB-21), so its correctly rounded sqrt is strictly larger: the winner is the
//   unique argmin of the rounded distances.  Otherwise (a near tie, a winner below 2^-100
//   where the relative bound does not hold, or an infinite distance) the wave redoes the
//   step with the correctly rounded sqrt per candidate and the lowest-index tie break
//   (lds_exact) -- about once per 10^4 instance-steps on uniform coordinates.
// Nothing is read from global memory inside the step loop: the winner's x comes from the
// LDS row (before its visit mark), its y from the owner lane's registers (a select tree
// over the slot's bits, then one lane shuffle), the CVRP demand from a read-only LDS row.
// The kernels are bound by each wave's dependent-instruction latency (4 waves per SIMD:
// every wave of a B = 65,536 episode is resident at once with 4 B of LDS per TSP node), so
// the step's tour-length sqrt is taken one step late, where it overlaps the next scan.
typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int clog2(int v) {
  int b = 0;
  while ((1 << b) < v) ++b;
  return b;
}

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// float index of node c's x in its instance's x row: node c is slot c / G of lane c % G,
// slots in pairs of 8 bytes, a pair's G lanes adjacent
template <int G>
__device__ __forceinline__ int lds_xoff(int c) {
  const unsigned k = (unsigned)c / G, sl = (unsigned)c % G;
  return (int)(((k >> 1) * G + sl) * 2 + (k & 1));
}

// the lane's x slot pairs from its instance's LDS row
template <int G, int EPL>
__device__ __forceinline__ void lds_load_x(const float* __restrict__ rowx, int sl,
                                           v2f (&x2)[EPL / 2]) {
  const float2* r2 = reinterpret_cast<const float2*>(rowx);
#pragma unroll
  for (int p = 0; p < EPL / 2; ++p) {
    const float2 q = r2[p * G + sl];
    x2[p] = (v2f){q.x, q.y};
  }
}

// the lane's two smallest keys (m1 <= m2) over its EPL slots; DEM: a customer whose demand
// does not fit (dm + used > vcap, cvrp/env.py:140) gets the key ~0
template <int G, int EPL, bool DEM>
__device__ __forceinline__ void lds_scan(const v2f (&x2)[EPL / 2], float cx, float cy,
                                         const v2f (&y2)[EPL / 2], const v2f (&dm2)[EPL / 2],
                                         float used, float vcap, uint32_t& m1, uint32_t& m2) {
  constexpr uint32_t KM = (1u << clog2(EPL)) - 1u;
  const v2f cx2 = {cx, cx}, cy2 = {cy, cy};
  const v2f u2 = {used, used};
  uint32_t a1 = 0xffffffffu, a2 = 0xffffffffu, b1 = 0xffffffffu, b2 = 0xffffffffu;
#pragma unroll
  for (int p = 0; p < EPL / 2; ++p) {
    const v2f dx = x2[p] - cx2, dy = y2[p] - cy2;
    const v2f s = dx * dx + dy * dy;  // -ffp-contract=off: two products and a sum
    v2f du = {0.f, 0.f};
    if (DEM) du = dm2[p] + u2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t key = (__float_as_uint(s[h]) & ~KM) | (uint32_t)(2 * p + h);
      if (DEM && du[h] > vcap) key = 0xffffffffu;
      if (p & 1) {  // two independent (min, second min) chains
        b2 = med3u(b1, b2, key);
        b1 = min(b1, key);
      } else {
        a2 = med3u(a1, a2, key);
        a1 = min(a1, key);
      }
    }
  }
  m1 = min(a1, b1);
  m2 = med3u(a1, b1, min(a2, b2));
}

// (smallest, second smallest) over the group's lanes
template <int G>
__device__ __forceinline__ void grp_min2(uint32_t& m1, uint32_t& m2) {
#define CO_MIN2(C)                                             \
  {                                                            \
    const uint32_t t1 = dpp_u<C>(m1), t2 = dpp_u<C>(m2);       \
    m2 = med3u(m1, t1, min(m2, t2));                           \
    m1 = min(m1, t1);                                          \
  }
  if (G >= 2) CO_MIN2(0xB1);
  if (G >= 4) CO_MIN2(0x4E);
  if (G >= 8) CO_MIN2(0x141);
  if (G >= 16) CO_MIN2(0x140);
#undef CO_MIN2
  if (G >= 32) {
    const auto a = __builtin_amdgcn_permlane16_swap(m1, m1, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(m2, m2, false, false);
    m2 = med3u(a[0], a[1], min(b[0], b[1]));
    m1 = min(a[0], a[1]);
  }
  if (G >= 64) {
    const auto a = __builtin_amdgcn_permlane32_swap(m1, m1, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(m2, m2, false, false);
    m2 = med3u(a[0], a[1], min(b[0], b[1]));
    m1 = min(a[0], a[1]);
  }
}

// The rare exact step: per candidate the correctly rounded f32 distance, the group argmin
// with the lowest-index tie break (torch.argmin over the oracle's distances); kNoNode when
// no candidate has a finite distance.  A call taking only scalars and pointers (y and the
// demand re-read from the input rows): passing the register arrays would put them in
// scratch memory, whose per-wave reservation caps the resident waves.
template <int G, int EPL, bool DEM>
__device__ __noinline__ int lds_exact(const float* __restrict__ rowx,
                                      const float2* __restrict__ lrow,
                                      const float* __restrict__ drow, int lo, int hi, int sl,
                                      float cx, float cy, float used, float vcap) {
  float best = __builtin_inff();
  int bi = kNoNode;
#pragma unroll 2
  for (int k = 0; k < EPL; ++k) {
    const int c = k * G + sl;
    const int ci = c < lo ? 0 : (c > hi ? hi - lo : c - lo);  // in range; x is NaN outside
    // NaN for visited / padding / the CVRP depot: never taken
    const float d = edge_len(cx, cy, rowx[lds_xoff<G>(c)], lrow[ci].y);
    const bool fits = !DEM || !(drow[ci] + used > vcap);
    if (fits && d < best) {
      best = d;
      bi = c;
    }
  }
  grp_argmin_split<G>(best, bi);
  return bi;
}

// The group's nearest candidate: the node, or kNoNode when every slot is poisoned (no
// candidate).  Every lane of the wave must take part.
template <int G, int EPL, bool DEM>
__device__ __forceinline__ int lds_nearest(const float* __restrict__ rowx,
                                           const v2f (&x2)[EPL / 2], int sl, float cx, float cy,
                                           const v2f (&y2)[EPL / 2], const v2f (&dm2)[EPL / 2],
                                           float used, float vcap,
                                           const float2* __restrict__ lrow,
                                           const float* __restrict__ drow, int lo, int hi) {
  constexpr uint32_t KM = (1u << clog2(EPL)) - 1u, BM = (1u << clog2(G * EPL)) - 1u;
  constexpr float kWin = 1.0f + (float)(1u << clog2(G * EPL)) * 0x1p-20f;
  uint32_t m1, m2;
  lds_scan<G, EPL, DEM>(x2, cx, cy, y2, dm2, used, vcap, m1, m2);
  // lane keys (T | slot) -> group keys (T | node); slot * G + lane < 2^BB never reaches T
  m1 = (m1 & ~BM) | ((m1 & KM) * G + sl);
  m2 = (m2 & ~BM) | ((m2 & KM) * G + sl);
  grp_min2<G>(m1, m2);
  const uint32_t t1 = m1 & ~BM, t2 = m2 & ~BM;
  const bool none = t1 >= 0x7fc00000u;  // every slot NaN or ~0
  const bool ok = none || (t1 >= 0x0d800000u && t1 < 0x7f800000u &&
                           t2 > __float_as_uint(__uint_as_float(t1) * kWin));
  int w = none ? kNoNode : (int)(m1 & BM);
  if (__builtin_expect(__any(!ok), 0))
    w = lds_exact<G, EPL, DEM>(rowx, lrow, drow, lo, hi, sl, cx, cy, used, vcap);
  return w;
}

// (m & x) | (~m & y), opaque to the optimizer (which would otherwise fold the select tree
// below back into an indexed read and lower that as a compare chain per element)
__device__ __forceinline__ float bfi(uint32_t m, float x, float y) {
  float r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y));
  return r;
}

// slot k's value among the lane's pairs: a select tree over k's bits (one v_bfi per node)
template <int P>
__device__ __forceinline__ float sel_pair(const v2f (&v)[P], unsigned k) {
  float t[P];
  const uint32_t m0 = 0u - (k & 1u);
#pragma unroll
  for (int p = 0; p < P; ++p) t[p] = bfi(m0, v[p][1], v[p][0]);
#pragma unroll
  for (int w = 1, l = 1; w < P; w <<= 1, ++l) {
    const uint32_t m = 0u - ((k >> l) & 1u);
#pragma unroll
    for (int i = 0; i + w < P; i += 2 * w) t[i] = bfi(m, t[i + w], t[i]);
  }
  return t[0];
}

// the winner's y: its owner lane's register, handed to the group by one lane shuffle
template <int G, int EPL>
__device__ __forceinline__ float owner_y(const v2f (&y2)[EPL / 2], int w, int gbase) {
  const float yv = sel_pair<EPL / 2>(y2, (unsigned)w / G);
  return __shfl(yv, gbase + w % G, 64);
}

#ifndef CO_NEAREST_PAY
#define CO_NEAREST_PAY 0  // the winner's y: 0 from the input row, 1 from the owner lane (tree)
#endif

// The tour terms sqrtf(sq_t) (correctly rounded, as torch's) summed in f64, G at a time:
// lane (t mod G) of the group holds step t's squared length until each of the group's G
// lanes holds one, then every lane takes one sqrt -- a sqrt per G steps instead of one per
// step.  The lanes' partial sums are added at the end: a sum of f32 terms in f64 is exact
// while the terms span less than 2^29, so the order does not show in the f32 reward.
template <int G>
struct TermAcc {
  double sum = 0.0;
  float hold = 0.f;
  __device__ __forceinline__ void add(float sq, int t, int sl) {
    const int r = t & (G - 1);  // wave-uniform
    hold = sl == r ? sq : hold;
    if (r == G - 1) {
      sum += (double)__builtin_sqrtf(hold);
      hold = 0.f;
    }
  }
  __device__ __forceinline__ double total() {  // every lane of the wave
    return grp_sum_f64<G>(sum + (double)__builtin_sqrtf(hold));
  }
};

// TSP with the x rows in LDS (see above): one wave per block, 64/G instances per wave.
template <int G, int EPL>
__global__ __launch_bounds__(64) void tsp_nearest_lds_kernel(
    int64_t B, int N, const float2* __restrict__ locs, int64_t* __restrict__ acts_out,
    uint8_t* __restrict__ mask_out, int64_t* __restrict__ first_out,
    int64_t* __restrict__ cur_out, int64_t* __restrict__ i_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out) {
  static_assert(EPL % 2 == 0 && (G & (G - 1)) == 0 && G * EPL <= 1024, "slot pairs");
  constexpr int IPW = 64 / G, SLOTS = G * EPL;
  __shared__ float2 s_x[IPW * SLOTS / 2];
  const int lane = threadIdx.x, sl = lane % G, gi = lane / G, gbase = lane - sl;
  const int64_t base = (int64_t)blockIdx.x * IPW;
  if (base >= B) return;  // block-uniform
  const int64_t b = base + gi;
  const bool valid = b < B;
  const int64_t bb = valid ? b : B - 1;  // a dead group mirrors the last instance
  const float2* lrow = locs + bb * N;
  float* const rowx = reinterpret_cast<float*>(s_x) + gi * SLOTS;
  const float qnan = __builtin_nanf("");
  v2f y2[EPL / 2];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {  // padding slots: x NaN (loads unconditional: no serial waits)
    const int c = k * G + sl;
    const float2 q = lrow[c < N ? c : N - 1];
    rowx[lds_xoff<G>(c)] = c < N ? q.x : qnan;
    y2[k >> 1][k & 1] = c < N ? q.y : 0.f;
  }
  const v2f nodem[EPL / 2] = {};  // no demand
  const float2 q0 = lrow[0];  // step 0: node 0
  __syncthreads();
  rowx[0] = qnan;
  float cx = q0.x, cy = q0.y;
  if (valid && sl == 0) acts_out[bb] = 0;
  TermAcc<G> len;
  int cur = 0;
  v2f x2[EPL / 2];
  lds_load_x<G, EPL>(rowx, sl, x2);
  for (int t = 1; t < N; ++t) {
    int a = lds_nearest<G, EPL, false>(rowx, x2, sl, cx, cy, y2, nodem, 0.f, 0.f, lrow,
                                       nullptr, 0, N - 1);
    a = a == kNoNode ? 0 : a;  // only when every remaining distance is infinite
    float* px = rowx + lds_xoff<G>(a);
#if CO_NEAREST_PAY
    const float wx = *px, wy = owner_y<G, EPL>(y2, a, gbase);
#else
    const float2 wq = lrow[a];
    const float wx = wq.x, wy = wq.y;
#endif
    *px = qnan;  // visited
    lds_load_x<G, EPL>(rowx, sl, x2);  // the next step's x pairs
    const float dx = wx - cx, dy = wy - cy;
    len.add(dx * dx + dy * dy, t, sl);
    cx = wx;
    cy = wy;
    cur = a;
    if (valid && sl == 0) acts_out[(int64_t)t * B + bb] = a;
  }
  const float ex = q0.x - cx, ey = q0.y - cy;  // the closing edge
  len.add(ex * ex + ey * ey, N, sl);
  const double tour = len.total();
  if (!valid) return;
  uint8_t* mrow = mask_out + bb * N;
  for (int c = sl; c < N; c += G) mrow[c] = 0;  // every node visited
  if (sl == 0) {
    first_out[bb] = 0;
    cur_out[bb] = cur;
    i_out[bb] = N;
    done_out[bb] = 1;
    step_reward_out[bb] = 0;
    reward_out[bb] = -(float)tour;
  }
}

// CVRP with the x rows in LDS (the depot's x NaN: never a candidate), y and demand per slot
// in registers (the capacity test, packed), the demand also in a read-only LDS row (the
// chosen customer's).  The transition, finishing and final rows are those of
// cvrp_nearest_episode_kernel; a customer is visited iff its LDS x is NaN (NaN input
// coordinates would read as visited).
template <int G, int EPL>
__global__ __launch_bounds__(64) void cvrp_nearest_lds_kernel(
    int64_t B, int N, const float2* __restrict__ depot, const float2* __restrict__ locs_in,
    const float* __restrict__ demand, float vcap, int max_steps, int64_t* __restrict__ acts_out,
    float2* __restrict__ locs_out, int64_t* __restrict__ cur_out, float* __restrict__ used_out,
    float* __restrict__ vcap_out, uint8_t* __restrict__ visited_out,
    uint8_t* __restrict__ mask_out, uint8_t* __restrict__ done_out,
    uint8_t* __restrict__ step_reward_out, float* __restrict__ reward_out,
    int32_t* __restrict__ len_out, int32_t* __restrict__ tmax, int32_t* status) {
  static_assert(EPL % 2 == 0 && (G & (G - 1)) == 0 && G * EPL <= 1024, "slot pairs");
  constexpr int IPW = 64 / G, SLOTS = G * EPL;
  __shared__ float2 s_x[IPW * SLOTS / 2];
  __shared__ float s_dem[IPW * SLOTS];
  const int lane = threadIdx.x, sl = lane % G, gi = lane / G, gbase = lane - sl;
  const int M = N + 1;
  const int64_t base = (int64_t)blockIdx.x * IPW;
  if (base >= B) return;  // block-uniform
  const int64_t b = base + gi;
  const bool valid = b < B;
  const int64_t bb = valid ? b : B - 1;  // a dead group mirrors the last instance
  const float2* lrow = locs_in + bb * N;  // customer c >= 1 is lrow[c - 1]
  const float* drow = demand + bb * N;
  float* const rowx = reinterpret_cast<float*>(s_x) + gi * SLOTS;
  float* const rowd = s_dem + gi * SLOTS;  // node-indexed
  const float qnan = __builtin_nanf("");
  const float2 dep = depot[bb];
  v2f y2[EPL / 2], dm2[EPL / 2];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {  // loads unconditional (clamped): no serial waits
    const int c = k * G + sl;
    const int ci = c < 1 ? 0 : (c <= N ? c - 1 : N - 1);
    const float2 lq = lrow[ci];
    const float ld = drow[ci];
    const float2 q = c == 0 ? dep : (c <= N ? lq : make_float2(qnan, 0.f));
    const float d = (c >= 1 && c <= N) ? ld : 0.f;
    if (valid && locs_out && c <= N) locs_out[bb * M + c] = q;
    rowx[lds_xoff<G>(c)] = c == 0 ? qnan : q.x;  // the depot is never a nearest candidate
    rowd[c] = d;
    y2[k >> 1][k & 1] = q.y;
    dm2[k >> 1][k & 1] = d;
  }
  __syncthreads();
  float cx = dep.x, cy = dep.y, used = 0.f;
  // st = customers visited (bits 0-15) | steps taken (bits 16-30) | depot entered (bit 31)
  uint32_t st = 0;
  int cur = 0;
  bool done = false;
  TermAcc<G> dist;
  v2f x2[EPL / 2];
  lds_load_x<G, EPL>(rowx, sl, x2);
  int t = 0;
  for (; t < max_steps; ++t) {
    if (__ballot(!done) == 0) break;  // wave-uniform: the group reductions need every lane
    const int w = lds_nearest<G, EPL, true>(rowx, x2, sl, cx, cy, y2, dm2, used, vcap, lrow,
                                            drow, 1, N);
    const int a = w == kNoNode ? 0 : w;
    float* px = rowx + lds_xoff<G>(a);
#if CO_NEAREST_PAY
    const float wx = *px, wy = owner_y<G, EPL>(y2, a, gbase), wd = rowd[a];
#else
    const int ai = a == 0 ? 0 : a - 1;
    const float2 wq = lrow[ai];
    const float wx = wq.x, wy = wq.y, wd = drow[ai];
#endif
    if (!done && a != 0) *px = qnan;  // visited
    lds_load_x<G, EPL>(rowx, sl, x2);  // the next step's x pairs
    const float2 q = a == 0 ? dep : make_float2(wx, wy);
    const float dx = q.x - cx, dy = q.y - cy;
    dist.add(done ? 0.f : dx * dx + dy * dy, t, sl);
    if (done) continue;
    used = a != 0 ? (used + wd) * 1.0f : 0.0f;  // cvrp/env.py:83-85
    st = ((st & 0x8000ffffu) + (a != 0 ? 1u : 0u)) | ((uint32_t)(t + 1) << 16) |
         (a == 0 ? 0x80000000u : 0u);
    cur = a;
    cx = q.x;
    cy = q.y;
    if (valid && sl == 0) acts_out[(int64_t)t * B + bb] = a;
    done = (st & 0x8000ffffu) == (0x80000000u | (uint32_t)N);
  }
  const int len = (int)((st >> 16) & 0x7fffu);
  const float ex = dep.x - cx, ey = dep.y - cy;  // the closing edge to the depot
  dist.add(ex * ex + ey * ey, t, sl);
  const double tour = dist.total();
  // final state rows: visited and get_action_mask (cvrp/env.py:137-149)
  bool any_feas = false;
  uint8_t* vrow = visited_out + bb * M;
  uint8_t* mrow = mask_out + bb * M;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const int c = k * G + sl;
    const bool v = c == 0 ? (st >> 31) != 0 : __builtin_isnan(rowx[lds_xoff<G>(c)]);
    const bool feas = c >= 1 && c <= N && !v && !(dm2[k >> 1][k & 1] + used > vcap);
    any_feas |= feas;
    if (valid && c <= N) {
      vrow[c] = v;
      if (c >= 1) mrow[c] = feas;
    }
  }
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
  const bool anyf = (__ballot(any_feas) & gmask) != 0;
  if (valid && sl == 0) {
    mrow[0] = !((cur == 0) && anyf);
    cur_out[bb] = cur;
    used_out[bb] = used;
    vcap_out[bb] = vcap;
    done_out[bb] = done;
    step_reward_out[bb] = 0;
    reward_out[bb] = -(float)tour;
    len_out[bb] = len;
    if (!done) set_status(status, CO_ST_TRUNCATED);
    atomicMax(tmax, len);
  }
}

inline unsigned lds_grid(int64_t B, int G) {  // a one-wave block per 64/G instances
  return cover_grid(B, 64 / G, 64);
}

}  // namespace

// Called by co_tsp_rollout for the nearest policy (acts_in == NULL).
int co_internal_tsp_nearest_rollout(int64_t B, int64_t N, const float* locs, int64_t* acts_out,
                                    uint8_t* mask_out, int64_t* first_out, int64_t* cur_out,
                                    int64_t* i_out, uint8_t* done_out, uint8_t* step_reward_out,
                                    float* reward_out, void* stream) {
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  hipStream_t s = (hipStream_t)stream;
  if (group_grid(B, 64) == 0) return CO_E_INVAL;
#define CO_TSPN(G, EPL)                                                                        \
  hipLaunchKernelGGL((tsp_nearest_episode_kernel<G, EPL, (G <= 8 && EPL > 8)>),                \
                     dim3(group_grid(B, G)), dim3(256),                                         \
                     0, s, B, (int)N, l2, acts_out, mask_out, first_out, cur_out, i_out,       \
                     done_out, step_reward_out, reward_out)
#define CO_TSPL(G, EPL)                                                                        \
  hipLaunchKernelGGL((tsp_nearest_lds_kernel<G, EPL>), dim3(lds_grid(B, G)), dim3(64), 0, s, B,  \
                     (int)N, l2, acts_out, mask_out, first_out, cur_out, i_out, done_out,        \
                     step_reward_out, reward_out)
  if (CO_NEAREST_LDS) {
    if (N <= 32) CO_TSPL(4, 8);
    else if (N <= 64) CO_TSPL(4, 16);
    else if (N <= 104 && CO_NEAREST_LDS_G == 4) CO_TSPL(4, 26);
    else if (N <= 112) CO_TSPL(8, 14);
    else if (N <= 128) CO_TSPL(8, 16);
    else if (N <= 256) CO_TSPL(8, 32);
    else if (N <= 512) CO_TSPL(16, 32);
    else CO_TSPL(32, 32);
    return launch_status();
  }
#undef CO_TSPL
  if (N <= 32) CO_TSPN(4, 8);
  else if (N <= 64) CO_TSPN(8, 8);
  else if (CO_NEAREST_G8 && N <= 104) CO_TSPN(8, 13);
  else if (N <= 112) CO_TSPN(16, 7);
  else if (N <= 128) CO_TSPN(16, 8);
  else if (N <= 256) CO_TSPN(32, 8);
  else if (N <= 512) CO_TSPN(64, 8);
  else CO_TSPN(64, 16);
#undef CO_TSPN
  return launch_status();
}

extern "C" int co_cvrp_rollout(int64_t B, int64_t N, const float* depot, const float* locs,
                               const float* demand, float vcap, int64_t max_steps,
                               int64_t* acts_out, float* locs_out, int64_t* cur_out,
                               float* used_out, float* vcap_out, uint8_t* visited_out,
                               uint8_t* mask_out, uint8_t* done_out, uint8_t* step_reward_out,
                               float* reward_out, int32_t* len_out, int32_t* steps_out,
                               int32_t* status, void* stream) {
  // the episode's step count is packed into 15 bits in the kernel; instance indices are int
  if (B < 0 || B > 0x7fffffff || N <= 0 || N > 1023 || max_steps <= 0 || max_steps > 0x7fff)
    return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!depot || !locs || !demand || !acts_out || !cur_out || !used_out || !vcap_out ||
      !visited_out || !mask_out || !done_out || !step_reward_out || !reward_out || !len_out ||
      !steps_out || !status)
    return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(depot) | reinterpret_cast<uintptr_t>(locs) |
       reinterpret_cast<uintptr_t>(locs_out)) & 7)
    return CO_E_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  if (group_grid(B, 64) == 0) return CO_E_INVAL;
  if (zero_i32(steps_out, s) != hipSuccess) return launch_status();
  const float2* d2 = reinterpret_cast<const float2*>(depot);
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  float2* lo = reinterpret_cast<float2*>(locs_out);
#define CO_CVRPN(G, EPL)                                                                       \
  hipLaunchKernelGGL((cvrp_nearest_episode_kernel<G, EPL, (G <= 8 && EPL > 8)>),               \
                     dim3(group_grid(B, G)), dim3(256),                                         \
                     0, s, B, (int)N, d2, l2, demand, vcap, (int)max_steps, acts_out, lo,      \
                     cur_out, used_out, vcap_out, visited_out, mask_out, done_out,             \
                     step_reward_out, reward_out, len_out, steps_out, status)
  const int64_t M = N + 1;
#define CO_CVRPL(G, EPL)                                                                       \
  hipLaunchKernelGGL((cvrp_nearest_lds_kernel<G, EPL>), dim3(lds_grid(B, G)), dim3(64), 0, s, B, \
                     (int)N, d2, l2, demand, vcap, (int)max_steps, acts_out, lo, cur_out,        \
                     used_out, vcap_out, visited_out, mask_out, done_out, step_reward_out,       \
                     reward_out, len_out, steps_out, status)
  if (CO_NEAREST_LDS) {
    if (M <= 32) CO_CVRPL(4, 8);
    else if (M <= 64) CO_CVRPL(4, 16);
    else if (M <= 112) CO_CVRPL(CO_NEAREST_CVRP_G, 112 / CO_NEAREST_CVRP_G);
    else if (M <= 128) CO_CVRPL(8, 16);
    else if (M <= 256) CO_CVRPL(8, 32);
    else if (M <= 512) CO_CVRPL(16, 32);
    else CO_CVRPL(32, 32);
  } else if (M <= 32) CO_CVRPN(4, 8);
  else if (M <= 64) CO_CVRPN(8, 8);
  else if (CO_NEAREST_G8 && M <= 104) CO_CVRPN(8, 13);
  else if (M <= 112) CO_CVRPN(16, 7);
  else if (M <= 128) CO_CVRPN(16, 8);
  else if (M <= 256) CO_CVRPN(32, 8);
  else if (M <= 512) CO_CVRPN(64, 8);
  else CO_CVRPN(64, 16);
#undef CO_CVRPN
#undef CO_CVRPL
  hipLaunchKernelGGL(cvrp_pad_kernel, dim3(grid_for(B, 256, 2048)), dim3(256), 0, s, B, len_out,
                     steps_out, acts_out, cur_out, used_out);
  return launch_status();
}
