// Fused nearest-policy episodes for gfx950: the whole env-only rollout
// (rl4co/utils/decoding.py:88-109) of TSP (tsp/env.py:67-173) and CVRP
// (cvrp/env.py:73-190) with the nearest-node bench policy of SURVEY.md 8d in-kernel.
// The oracle's policy (oracle/envs.py tsp_nearest_action / cvrp_nearest_action):
// argmin over feasible nodes of f32 sqrt(dx*dx + dy*dy), ties -> lowest index.
//
// Layout: a G-lane group per instance, 64/G instances per one-wave workgroup.  Lane `sl`
// of the group owns nodes c = sl + G*k (k < EPL): their y (and CVRP demand) in VGPRs, their
// x in the instance's LDS row, where a visit writes NaN (see "LDS-row episodes" below).
// Measured and dropped: coordinates and a visited bit mask in VGPRs
// (r04/r05 register engines, 0.31 / 0.28 ms), (x, y) rows in LDS (a second, one-third
// occupied round of waves at B = 65,536), the winner's y from its owner lane's registers by
// a select tree (+30 VALU per step, slower than the L2 read it replaces) and a speculative
// read of every lane's best candidate (its DPP hand-off costs more than the latency saved).
#include "co_common.hpp"

using namespace co;

namespace {

constexpr int kNoNode = 0x7fffffff;

#ifndef CO_NEAREST_LDS_G
#define CO_NEAREST_LDS_G 4  // TSP N <= 104: lanes per instance (4 x 26 slots, or 8 x 14)
#endif
#ifndef CO_NEAREST_CVRP_G
#define CO_NEAREST_CVRP_G 8  // CVRP N + 1 <= 112: lanes per instance (4 x 28 or 8 x 14 slots)
#endif

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

// ---------------------------------------------------------------------------------------
// LDS-row episodes.  The per-step cost of a register-resident engine (round 4: coordinates
// and a visited bit mask in VGPRs) is the per-candidate VALU work: two subtractions, two
// products, a sum, the visited / capacity bit test and four selects per node.  Here each
// lane keeps its slots' y (and CVRP demand) in registers as pairs, and the instance's x row
// lives in LDS in node order; a visited node (and every padding slot, and the CVRP depot)
// has x = NaN, so its distance is NaN and it can never be the minimum -- visiting is one
// LDS store instead of a per-candidate test.  Per pair of candidates: one ds_read2_b32,
// five packed f32 operations (v_pk_add / v_pk_mul: the same IEEE operations, two slots at
// a time), and per candidate a key = the squared distance's bits with the low BB bits
// replaced by slot * G (one v_and_or; the lane's index is ORed in once) folded into the
// lane's two smallest keys (v_med3_u32 + v_min_u32, two independent chains).  The group
// merges (min, second min)
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
// The winner's coordinates (and CVRP demand) are one read of the input row, an L2 / MALL hit
// whose latency the other resident waves cover: with 4 B of LDS per node and the y slots in
// VGPRs, every wave of a B = 65,536 TSP-100 episode is resident at once (4 per SIMD).  The
// kernels are VALU-issue bound: measured (tools/valu_rates.py) a wave64 VALU instruction
// takes about 5 SIMD cycles at 4 waves per SIMD (v_pk_* f32 about 5.4, for two slots), and
// time grows by one wave-episode of issue per added wave per SIMD (tools/nearest_scaling.py),
// so the lever is instructions per instance-step: the packed scan, a sqrt per G steps
// (TermAcc) and no per-step global wait besides the winner's read.
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

// The instance's x row is in node order (node c = slot c / G of lane c % G): a visit and the
// winner's read address node c directly, and a lane's slot pair (2p, 2p+1) is one
// ds_read2_b32 (dword offsets 2pG and (2p+1)G from the lane's base) into a register pair.
template <int G, int EPL>
__device__ __forceinline__ void lds_load_x(const float* __restrict__ rowx, int sl,
                                           v2f (&x2)[EPL / 2]) {
  const float* r = rowx + sl;
#pragma unroll
  for (int p = 0; p < EPL / 2; ++p) x2[p] = (v2f){r[2 * p * G], r[(2 * p + 1) * G]};
}

// the lane's two smallest keys (m1 <= m2) over its EPL slots, key = the squared distance's
// bits with the low BB bits replaced by slot * G (the node index less the lane, which the
// caller ORs in); DEM: a customer whose demand does not fit (dm + used > vcap,
// cvrp/env.py:140) gets the key ~0
template <int G, int EPL, bool DEM>
__device__ __forceinline__ void lds_scan(const v2f (&x2)[EPL / 2], float cx, float cy,
                                         const v2f (&y2)[EPL / 2], const v2f (&dm2)[EPL / 2],
                                         float used, float vcap, uint32_t& m1, uint32_t& m2) {
  constexpr uint32_t BM = (1u << clog2(G * EPL)) - 1u;
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
      uint32_t key = (__float_as_uint(s[h]) & ~BM) | (uint32_t)((2 * p + h) * G);
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
    const float d = edge_len(cx, cy, rowx[c], lrow[ci].y);
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
  constexpr uint32_t BM = (1u << clog2(G * EPL)) - 1u;
  constexpr float kWin = 1.0f + (float)(1u << clog2(G * EPL)) * 0x1p-20f;
  uint32_t m1, m2;
  lds_scan<G, EPL, DEM>(x2, cx, cy, y2, dm2, used, vcap, m1, m2);
  m1 |= (uint32_t)sl;  // lane keys (T | slot * G) -> group keys (T | node)
  m2 |= (uint32_t)sl;
  grp_min2<G>(m1, m2);
  const uint32_t t1 = m1 & ~BM, t2 = m2 & ~BM;
  // one bitwise test (no short-circuit branches): every slot poisoned (NaN or ~0), or a
  // normal finite winner whose next key is outside the ratio window
  const bool none = t1 >= 0x7fc00000u;
  const bool ok = none | ((t1 - 0x0d800000u < 0x7f800000u - 0x0d800000u) &
                          (t2 > __float_as_uint(__uint_as_float(t1) * kWin)));
  int w = none ? kNoNode : (int)(m1 & BM);
  if (__builtin_expect(__any(!ok), 0))
    w = lds_exact<G, EPL, DEM>(rowx, lrow, drow, lo, hi, sl, cx, cy, used, vcap);
  return w;
}

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
    if (r == G - 1) {  // a real branch: the compiler would if-convert it (a sqrt every step)
      asm volatile("");
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
    rowx[c] = c < N ? q.x : qnan;
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
    float* px = rowx + a;
    const float2 wq = lrow[a];  // an L2 read: the winner's y is in its owner lane's VGPRs
    const float wx = wq.x, wy = wq.y;
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

// CVRP: nodes 0..N (0 = depot).  Each step the nearest customer that is unvisited and fits
// (!(demand + used > capacity), cvrp/env.py:140), else the depot; the env transition of
// cvrp/env.py:73-105 on group-uniform scalars: used = (used + d) * (a != 0), done = every
// node visited (visited.sum == N + 1, so the depot must have been entered once).  A
// finished instance stops; co_cvrp_rollout's pad pass then applies the reference's
// remaining depot steps up to the batch-wide episode length.  x rows in LDS (the depot's x
// NaN: never a candidate), y and demand per slot in VGPRs (the capacity test, packed); a
// customer is visited iff its LDS x is NaN (NaN input coordinates would read as visited).
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
    rowx[c] = c == 0 ? qnan : q.x;  // the depot is never a nearest candidate
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
    float* px = rowx + a;
    const int ai = a == 0 ? 0 : a - 1;
    const float2 wq = lrow[ai];  // L2 reads
    const float wx = wq.x, wy = wq.y, wd = drow[ai];
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
    const bool v = c == 0 ? (st >> 31) != 0 : __builtin_isnan(rowx[c]);
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
  if (lds_grid(B, 4) == 0) return CO_E_INVAL;
#define CO_TSPL(G, EPL)                                                                        \
  hipLaunchKernelGGL((tsp_nearest_lds_kernel<G, EPL>), dim3(lds_grid(B, G)), dim3(64), 0, s, B,  \
                     (int)N, l2, acts_out, mask_out, first_out, cur_out, i_out, done_out,        \
                     step_reward_out, reward_out)
  if (N <= 32) CO_TSPL(4, 8);
  else if (N <= 64) CO_TSPL(4, 16);
  else if (N <= 104 && CO_NEAREST_LDS_G == 4) CO_TSPL(4, 26);
  else if (N <= 112) CO_TSPL(8, 14);
  else if (N <= 128) CO_TSPL(8, 16);
  else if (N <= 256) CO_TSPL(8, 32);
  else if (N <= 512) CO_TSPL(16, 32);
  else CO_TSPL(32, 32);
#undef CO_TSPL
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
  if (lds_grid(B, 4) == 0) return CO_E_INVAL;
  if (zero_i32(steps_out, s) != hipSuccess) return launch_status();
  const float2* d2 = reinterpret_cast<const float2*>(depot);
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  float2* lo = reinterpret_cast<float2*>(locs_out);
  const int64_t M = N + 1;
#define CO_CVRPL(G, EPL)                                                                       \
  hipLaunchKernelGGL((cvrp_nearest_lds_kernel<G, EPL>), dim3(lds_grid(B, G)), dim3(64), 0, s, B, \
                     (int)N, d2, l2, demand, vcap, (int)max_steps, acts_out, lo, cur_out,        \
                     used_out, vcap_out, visited_out, mask_out, done_out, step_reward_out,       \
                     reward_out, len_out, steps_out, status)
  if (M <= 32) CO_CVRPL(4, 8);
  else if (M <= 64) CO_CVRPL(4, 16);
  else if (M <= 112) CO_CVRPL(CO_NEAREST_CVRP_G, 112 / CO_NEAREST_CVRP_G);
  else if (M <= 128) CO_CVRPL(8, 16);
  else if (M <= 256) CO_CVRPL(8, 32);
  else if (M <= 512) CO_CVRPL(16, 32);
  else CO_CVRPL(32, 32);
#undef CO_CVRPL
  hipLaunchKernelGGL(cvrp_pad_kernel, dim3(grid_for(B, 256, 2048)), dim3(256), 0, s, B, len_out,
                     steps_out, acts_out, cur_out, used_out);
  return launch_status();
}
