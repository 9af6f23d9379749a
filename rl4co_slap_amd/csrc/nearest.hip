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
  if (M <= 32) CO_CVRPN(4, 8);
  else if (M <= 64) CO_CVRPN(8, 8);
  else if (CO_NEAREST_G8 && M <= 104) CO_CVRPN(8, 13);
  else if (M <= 112) CO_CVRPN(16, 7);
  else if (M <= 128) CO_CVRPN(16, 8);
  else if (M <= 256) CO_CVRPN(32, 8);
  else if (M <= 512) CO_CVRPN(64, 8);
  else CO_CVRPN(64, 16);
#undef CO_CVRPN
  hipLaunchKernelGGL(cvrp_pad_kernel, dim3(grid_for(B, 256, 2048)), dim3(256), 0, s, B, len_out,
                     steps_out, acts_out, cur_out, used_out);
  return launch_status();
}
