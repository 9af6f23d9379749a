// SLAP (storage location assignment) env kernels for gfx950: reset, step
// (assignment write + location mask) and the per-order pick-tour reward.
//
// Step: the 64-instance byte tile of co_tile.hpp for the [B, L] mask (no row
// count needed: done = i == P-1, slap/env.py:57); the assignment row is copied
// only when the output is a fresh buffer (the reference clones, env.py:50), and
// the single element [b, product] is written afterwards by the row's thread.
//
// Reward: one wavefront per instance.  Lane s owns pick slot s = (order o, pick k)
// of the O*K picklist, gathers product -> location -> (x, y) into LDS; lane o then
// sums its order's closed-tour edges in pick order and lane 0 accumulates the
// orders in order (slap/env.py:136-142 adds them one by one in f32).
#include "co_common.hpp"
#include "co_tile.hpp"

using namespace co;

#ifndef CO_SLAP_GROUP_STEP
#define CO_SLAP_GROUP_STEP 1  // co_slap_step on the 16-lane group kernel when it can
#endif

namespace {

__global__ __launch_bounds__(256) void slap_reset_kernel(int64_t B, int64_t L, int64_t P,
                                                         uint8_t* mask, float* to_choose,
                                                         int64_t* it, float* reward,
                                                         float* ratio, uint8_t* done,
                                                         uint8_t* terminated) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // 16-byte units where the buffers allow it (the launcher checks alignment)
  const bool vm = (reinterpret_cast<uintptr_t>(mask) & 15) == 0;
  const int64_t nm = B * L, nm16 = vm ? nm >> 4 : 0;
  for (int64_t k = t0; k < nm16; k += stride) {  // mask[b, l] = l != 0 (depot masked)
    union {
      uint4 v;
      uint8_t c[16];
    } u;
    int64_t col = (k << 4) % L;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      u.c[j] = col != 0;
      if (++col == L) col = 0;
    }
    reinterpret_cast<uint4*>(mask)[k] = u.v;
  }
  for (int64_t k = (nm16 << 4) + t0; k < nm; k += stride) mask[k] = (k % L) != 0;
  for (int64_t k = t0; k < B * P; k += stride) to_choose[k] = (float)(k % P);
  if (ratio) {
    const bool vr = (reinterpret_cast<uintptr_t>(ratio) & 15) == 0;
    const int64_t nr4 = vr ? nm >> 2 : 0;
    for (int64_t k = t0; k < nr4; k += stride)
      reinterpret_cast<float4*>(ratio)[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t k = (nr4 << 2) + t0; k < nm; k += stride) ratio[k] = 0.f;
  }
  for (int64_t b = t0; b < B; b += stride) {
    it[b] = 0;
    reward[b] = 0.f;
    if (done) done[b] = 0;
    if (terminated) terminated[b] = 0;
  }
}

struct SlapRowEpilogue {
  int P;
  const float* to_choose;
  int64_t tc_stride;
  int32_t* assign_out;
  const int64_t* i_in;
  int64_t* i_out;
  uint8_t* done;
  uint8_t* reward;
  int32_t* status;
  struct Row {
    int64_t i;
    float product;
  };
  // to_choose NULL: every row's product is tc_stride (the untouched arange at that step)
  __device__ Row load(int64_t b) const {
    return {i_in[b], to_choose ? to_choose[b * tc_stride] : (float)tc_stride};
  }
  __device__ void store(int64_t b, int64_t action, int, const Row& r) const {
    int64_t p = (int64_t)(int)r.product;  // .to(torch.int), env.py:52
    if (p < 0) p += P;
    if (p < 0 || p >= P) {
      set_status(status, CO_ST_INDEX_RANGE);
    } else {
      assign_out[b * P + p] = (int32_t)action;  // .to(torch.int), env.py:53-54
    }
    done[b] = r.i == (int64_t)(P - 1);
    i_out[b] = r.i + 1;
    reward[b] = 0;
  }
};

__global__ __launch_bounds__(256) void slap_step_kernel(int64_t B, int L, const int64_t* action,
                                                        const uint8_t* mask_in, uint8_t* mask_out,
                                                        const int32_t* assign_in,
                                                        SlapRowEpilogue epi, int vec) {
  // Out-of-place assignment: copy the tile's [rows, P] int32 block first.
  if (assign_in != epi.assign_out) {
    const int64_t row0 = (int64_t)blockIdx.x * kTileRows;
    const int rows = (int)((B - row0) < kTileRows ? (B - row0) : kTileRows);
    const int64_t n = (int64_t)rows * epi.P;
    const int32_t* s = assign_in + row0 * epi.P;
    int32_t* d = epi.assign_out + row0 * epi.P;
    for (int64_t k = threadIdx.x; k < n; k += kTileThreads) d[k] = s[k];
    // the epilogue's element write must follow every thread's copy of the block
    __syncthreads();
  }
  mask_clear_tile<false, true>(B, L, action, mask_in, mask_out, epi.status, vec != 0, epi);
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void slap_reward_kernel(
    int64_t B, int L, int P, int O, int K, const int32_t* assignment, const int64_t* picklist,
    const float2* locs, float* reward, int32_t* status) {
  // LDS per wave: the instance's locations [L] and assignment [P] (staged by lane loads
  // issued together with the picklist loads: one memory latency per instance instead of
  // the picklist -> assignment -> location chain), then the pick points [S] and the
  // per-order lengths [O].
  extern __shared__ float s_rew[];
  const int w = wave_in_block(), lane = lane_id();
  const int S = O * K;
  float2* lxy = reinterpret_cast<float2*>(s_rew) + (size_t)w * (L + S + O + (P + 1) / 2);
  float2* pts = lxy + L;
  float* olen = reinterpret_cast<float*>(pts + S);
  int32_t* asg = reinterpret_cast<int32_t*>(olen + O);
  for (int64_t b = (int64_t)blockIdx.x * WAVES + w; b < B; b += (int64_t)gridDim.x * WAVES) {
    const int64_t* prow = picklist + b * (int64_t)S;
    const int32_t* arow = assignment + b * (int64_t)P;
    const float2* lrow = locs + b * (int64_t)L;
    constexpr int PU = 4;  // picks per lane kept in registers (S <= 256); more: a loop
    constexpr int LU = 4;  // locations per lane (L <= 256); more: a loop
    int64_t pk[PU];
    float2 lv[LU];
    int32_t av = 0;
    // every load of the instance issued before any LDS store (one memory latency):
    // unconditional clamped addresses, the out-of-row values are never stored
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int sidx = lane + 64 * u;
      pk[u] = prow[sidx < S ? sidx : S - 1];
    }
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const int c = lane + 64 * u;
      lv[u] = lrow[c < L ? c : L - 1];
    }
    av = arow[lane < P ? lane : P - 1];
#pragma unroll
    for (int u = 0; u < LU; ++u)
      if (lane + 64 * u < L) lxy[lane + 64 * u] = lv[u];
    for (int c = lane + 64 * LU; c < L; c += 64) lxy[c] = lrow[c];
    if (lane < P) asg[lane] = av;
    for (int c = lane + 64; c < P; c += 64) asg[c] = arow[c];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    bool range = false;
    for (int s0 = 0; s0 < S; s0 += 64 * PU) {
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int s = s0 + lane + 64 * u;
        if (s < S) {
          int64_t p = s0 == 0 ? pk[u] : prow[s];
          if (p < 0) p += P;  // python indexing of assignment[b, picklist] (slap/env.py:139)
          int64_t loc = 0;
          if (p < 0 || p >= P) {
            range = true;
          } else {
            loc = asg[p];
            if (loc < 0) loc += L;  // the -1 of an unassigned product wraps (locs[b, -1])
            if (loc < 0 || loc >= L) {
              range = true;
              loc = 0;
            }
          }
          pts[s] = lxy[loc];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // per-order closed tour (lane o), edges summed in pick order; the orders then added one
    // by one in f32 (slap/env.py:136-142) from the lanes' registers (v_readlane: no LDS
    // round trip in the serial part)
    float total = 0.f;
    for (int o0 = 0; o0 < O; o0 += 64) {
      const int o = o0 + lane;
      float len = 0.f;
      if (o < O) {
        const float2* op = pts + o * K;
        for (int k = 0; k < K; ++k) {
          const float2 p = op[k], q = op[(k + 1 == K) ? 0 : k + 1];
          len += edge_len(p.x, p.y, q.x, q.y);
        }
      }
      const int cnt = O - o0 < 64 ? O - o0 : 64;
      for (int j = 0; j < cnt; ++j)
        total += -__int_as_float(__builtin_amdgcn_readlane(__float_as_int(len), j));
    }
    if (lane == 0) reward[b] = total;
    if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// SLAPEnv._get_reward (slap/env.py:131-143), G lanes per instance, 256/G instances per
// workgroup, no loop: every load of the instance (its L coordinates, P assignment
// entries and O*K picks, LU / PU / SU per lane, coalesced 8G- / 4G-byte row pieces) is
// issued at once; coordinates and assignment land in the group's LDS, then each pick's
// location (python's negative-index wrap of slap/env.py:139 and of the -1 of an
// unassigned product) is looked up, its point stored, each order's closed tour summed
// in pick order (edge_len, as torch's norm) by one lane per order, and the orders added
// one by one in f32 by the group's lane 0 -- the reference's accumulation order.
// LDS per instance: 8L + 4P + 8S + 4O bytes (16-byte rounded).
__host__ __device__ inline int slap_rg_bytes(int L, int P, int S, int O) {
  return (8 * L + ((4 * P + 7) & ~7) + 8 * S + 4 * O + 15) & ~15;
}
template <int G, int LU, int PU, int SU>
__global__ __launch_bounds__(256) void slap_reward_group_kernel(
    int64_t B, int L, int P, int O, int K, const int32_t* __restrict__ assignment,
    const int64_t* __restrict__ picklist, const float2* __restrict__ locs,
    float* __restrict__ reward, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_rg[];
  const int S = O * K;
  const int sl = threadIdx.x % G, gib = threadIdx.x / G;
  const int64_t b = (int64_t)blockIdx.x * (256 / G) + gib;
  const bool valid = b < B;
  const int64_t rb = valid ? b : B - 1;  // dead groups mirror the last instance
  unsigned char* base = s_rg + (size_t)gib * slap_rg_bytes(L, P, S, O);
  float2* xy = reinterpret_cast<float2*>(base);
  int32_t* asg = reinterpret_cast<int32_t*>(xy + L);
  float2* pts = reinterpret_cast<float2*>(base + 8 * L + ((4 * P + 7) & ~7));
  float* olen = reinterpret_cast<float*>(pts + S);
  const float2* lrow = locs + rb * (int64_t)L;
  const int32_t* arow = assignment + rb * (int64_t)P;
  const int64_t* prow = picklist + rb * (int64_t)S;
  float2 lv[LU];
  int32_t av[PU];
  int64_t pk[SU];
#pragma unroll
  for (int u = 0; u < LU; ++u) {
    const int c = sl + G * u;
    lv[u] = lrow[c < L ? c : L - 1];
  }
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int c = sl + G * u;
    av[u] = arow[c < P ? c : P - 1];
  }
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int c = sl + G * u;
    pk[u] = prow[c < S ? c : S - 1];
  }
#pragma unroll
  for (int u = 0; u < LU; ++u)
    if (sl + G * u < L) xy[sl + G * u] = lv[u];
#pragma unroll
  for (int u = 0; u < PU; ++u)
    if (sl + G * u < P) asg[sl + G * u] = av[u];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  bool range = false;
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int sidx = sl + G * u;
    if (sidx < S) {
      int64_t pp = pk[u];
      if (pp < 0) pp += P;
      int64_t loc = 0;
      if (pp < 0 || pp >= P) {
        range = true;
      } else {
        loc = asg[pp];
        if (loc < 0) loc += L;
        if (loc < 0 || loc >= L) {
          range = true;
          loc = 0;
        }
      }
      pts[sidx] = xy[loc];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int o = sl; o < O; o += G) {  // one lane per order: its closed tour in pick order
    const float2* op = pts + o * K;
    float len = 0.f;
    for (int k = 0; k < K; ++k) {
      const float2 p0 = op[k], p1 = op[k + 1 == K ? 0 : k + 1];
      len += edge_len(p0.x, p0.y, p1.x, p1.y);
    }
    olen[o] = len;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool bad = (__ballot(range && valid) != 0ull);
  if (valid && sl == 0) {
    float total = 0.f;  // orders added one by one (slap/env.py:135-142)
    for (int o = 0; o < O; ++o) total += -olen[o];
    reward[b] = total;
  }
  if (bad && threadIdx.x % 64 == 0) set_status(status, CO_ST_INDEX_RANGE);
}

// The reward for instances too large for the LDS staging of slap_reward_kernel (huge
// L / order counts): one wave per instance, lane o walks order o's picks reading the
// assignment and coordinates straight from global memory (L2), the orders added in order
// from the lanes' registers.  Same results as the staged kernels.
__global__ __launch_bounds__(256) void slap_reward_global_kernel(
    int64_t B, int L, int P, int O, int K, const int32_t* __restrict__ assignment,
    const int64_t* __restrict__ picklist, const float2* __restrict__ locs,
    float* __restrict__ reward, int32_t* status) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const int64_t* prow = picklist + b * (int64_t)O * K;
    const int32_t* arow = assignment + b * (int64_t)P;
    const float2* lrow = locs + b * (int64_t)L;
    bool range = false;
    auto point = [&](int64_t pp) {
      if (pp < 0) pp += P;
      int64_t loc = 0;
      if (pp < 0 || pp >= P) {
        range = true;
      } else {
        loc = arow[pp];
        if (loc < 0) loc += L;
        if (loc < 0 || loc >= L) {
          range = true;
          loc = 0;
        }
      }
      return lrow[loc];
    };
    float total = 0.f;
    for (int o0 = 0; o0 < O; o0 += 64) {
      const int o = o0 + lane;
      float len = 0.f;
      if (o < O) {
        const float2 first = point(prow[(int64_t)o * K]);
        float2 p0 = first;
        for (int k = 1; k <= K; ++k) {
          const float2 p1 = k == K ? first : point(prow[(int64_t)o * K + k]);
          len += edge_len(p0.x, p0.y, p1.x, p1.y);
          p0 = p1;
        }
      }
      const int cnt = O - o0 < 64 ? O - o0 : 64;
      for (int j = 0; j < cnt; ++j)
        total += -__int_as_float(__builtin_amdgcn_readlane(__float_as_int(len), j));
    }
    if (lane == 0) reward[b] = total;
    if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
  }
}

#ifndef CO_SLAP_RGROUP
#define CO_SLAP_RGROUP 1
#endif

__global__ __launch_bounds__(256) void slap_closest_kernel(int64_t B, int L, const float* dist,
                                                           const uint8_t* mask, int64_t* out) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_in_block(); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const float* drow = dist + b * (int64_t)L;
    const uint8_t* mrow = mask + b * (int64_t)L;
    float best = __builtin_inff();
    int bi = 0x7fffffff;
    for (int c = lane; c < L; c += 64) {
      const float dv = drow[c];  // unconditional: a load behind the mask test is serialised
      const float d = mrow[c] ? dv : __builtin_inff();
      if (d < best || (d == best && c < bi)) { best = d; bi = c; }
    }
    wave_argmin(best, bi);
    if (lane == 0) out[b] = bi;
  }
}

// Closest-free bench policy fused with the env step (one launch per stepwise step; the
// same results as co_slap_closest_free_action + co_slap_step with an in-place
// assignment).  16 lanes per instance, 16 instances per 256-thread workgroup; lane sl
// owns 4-location units u = sl + 16 k (k < KU): one float4 of depot distances and one
// u32 of mask bytes each, so a group's loads are 256-B coalesced row pieces.  The
// masked argmin (inf where not free, ties -> lowest index: torch.argmin) is a float
// group min then an index group min (grp_argmin_split); the owner lane's unit is
// written back with the chosen byte cleared, every other unit unchanged; lane 0
// applies the step's row epilogue (slap/env.py:38-93).
// CLOSEST = false: the env step alone (co_slap_step) on the same group layout, the action
// given (action_in; negative values index from the end as python indexing, out-of-range
// ones set CO_ST_INDEX_RANGE and clear nothing, as the tile kernel).
template <int KU, bool CLOSEST>
__global__ __launch_bounds__(256) void slap_closest_step_kernel(
    int64_t B, int L, int P, const float* __restrict__ dist, const uint8_t* __restrict__ mask_in,
    uint8_t* __restrict__ mask_out, const int64_t* __restrict__ action_in,
    int64_t* __restrict__ action_out,
    const float* __restrict__ to_choose, int64_t tc_stride, const int32_t* assign_in,
    int32_t* assign, const int64_t* __restrict__ i_in, int64_t* __restrict__ i_out, uint8_t* __restrict__ done,
    uint8_t* __restrict__ reward, int32_t* status) {
  constexpr int G = 16;
  const int sl = threadIdx.x & (G - 1);
  const int64_t b = (int64_t)blockIdx.x * (256 / G) + (threadIdx.x / G);
  const bool live = b < B;
  const int64_t bb = live ? b : B - 1;  // dead groups mirror the last row (wave-uniform DPP)
  const int U = L >> 2;                  // units per row (L % 4 == 0)
  const float4* drow = reinterpret_cast<const float4*>(dist + bb * (int64_t)L);
  const uint32_t* mrow = reinterpret_cast<const uint32_t*>(mask_in + bb * (int64_t)L);
  float4 dv[KU];
  uint32_t mv[KU];
#pragma unroll
  for (int k = 0; k < KU; ++k) {  // all loads first, unconditional within the row
    const int u = sl + G * k;
    const int uc = u < U ? u : U - 1;
    if constexpr (CLOSEST) dv[k] = drow[uc];
    mv[k] = mrow[uc];
  }
  int64_t it = 0;
  if (sl == 0) it = i_in[bb];
  // every lane (one broadcast line); to_choose NULL: the uniform product tc_stride
  const float prod = to_choose ? to_choose[bb * tc_stride] : (float)tc_stride;
  int bi = 0x7fffffff;
  int64_t a_raw = 0;
  if constexpr (CLOSEST) {
    float best = __builtin_inff();
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      const int u = sl + G * k;
      if (u < U) {
        const float d4[4] = {dv[k].x, dv[k].y, dv[k].z, dv[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = ((mv[k] >> (8 * j)) & 0xffu) ? d4[j] : __builtin_inff();
          if (d < best) {  // ascending index within the lane: strict < keeps the lowest
            best = d;
            bi = 4 * u + j;
          }
        }
        if (bi == 0x7fffffff) bi = 4 * u;  // a lane whose candidates are all masked
      }
    }
    grp_argmin_split<G>(best, bi);
    a_raw = bi;
  } else {
    a_raw = action_in[bb];  // group-uniform address (one request)
    int64_t a = a_raw < 0 ? a_raw + L : a_raw;  // slap/env.py:46 (python indexing)
    if (a < 0 || a >= L) {
      if (live && sl == 0) set_status(status, CO_ST_INDEX_RANGE);
      a = -1;
    }
    bi = (int)a;  // -1: no byte cleared
  }
  if (!live) return;
  int64_t p = (int64_t)(int)prod;  // .to(torch.int), slap/env.py:52
  if (p < 0) p += P;
  const bool p_ok = p >= 0 && p < P;
  const int32_t av = (int32_t)a_raw;  // .to(torch.int), slap/env.py:53-54
  if (assign_in != assign)  // out of place: the group writes the row with [p] = action
    for (int c = sl; c < P; c += G) assign[b * P + c] = c == p ? av : assign_in[b * P + c];
  uint32_t* mo = reinterpret_cast<uint32_t*>(mask_out + b * (int64_t)L);
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    const int u = sl + G * k;
    if (u < U) {
      const uint32_t clr = (bi >> 2) == u ? ~(0xffu << (8 * (bi & 3))) : ~0u;
      mo[u] = mv[k] & clr;
    }
  }
  if (sl == 0) {  // slap/env.py:50-62 (the row epilogue of co_slap_step)
    if constexpr (CLOSEST) action_out[b] = bi;
    if (!p_ok)
      set_status(status, CO_ST_INDEX_RANGE);
    else if (assign_in == assign)
      assign[b * P + p] = av;
    done[b] = it == (int64_t)(P - 1);
    i_out[b] = it + 1;
    reward[b] = 0;
  }
}

// K consecutive co_slap_closest_step launches in one (co_slap_closest_steps, round 6): the
// state ping-pongs between A and B (step k reads A for even k, B for odd k, writes the
// other), step k's action goes to row k of action_out, its product to_choose column k
// (the uniform product tc_stride + k without to_choose), the assignment of step 0 out of
// place from assign_in when it differs from assign, then in place; every step stores its
// whole state as its own launch would.  The row's distances and mask units stay in
// registers between steps; the group argmin is the single step's.
#ifndef CO_SLAP_SSORT
#define CO_SLAP_SSORT 1  // the steps kernel pops per-lane sorted candidate keys (0: masked scan)
#endif
// per-lane ascending sort of u64 keys (Batcher odd-even merge; one v_cmp_lt_u64 and four
// selects per comparator), the candidate order of the closest-free steps
__device__ __forceinline__ uint32_t key_sel32(uint64_t m, uint32_t t, uint32_t f) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
__device__ __forceinline__ void key_cswap(uint64_t& a, uint64_t& b) {
  const uint64_t lt = __builtin_amdgcn_ballot_w64(a < b);
  const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b,
                 bhi = (uint32_t)(b >> 32);
  a = ((uint64_t)key_sel32(lt, ahi, bhi) << 32) | key_sel32(lt, alo, blo);
  b = ((uint64_t)key_sel32(lt, bhi, ahi) << 32) | key_sel32(lt, blo, alo);
}
template <int E>
__device__ __forceinline__ void sort_keys_asc(uint64_t (&k)[E]) {
  static_assert((E & (E - 1)) == 0, "E must be a power of two");
#pragma unroll
  for (int p = 1; p < E; p <<= 1)
#pragma unroll
    for (int q = p; q > 0; q >>= 1)
#pragma unroll
      for (int j = q % p; j + q < E; j += 2 * q)
#pragma unroll
        for (int i = 0; i < q; ++i)
          if (i + j + q < E && (i + j) / (2 * p) == (i + j + q) / (2 * p)) key_cswap(k[i + j], k[i + j + q]);
}

template <int KU>
__global__ __launch_bounds__(256) void slap_closest_steps_kernel(
    int64_t B, int L, int P, int K, const float* __restrict__ dist, const float* to_choose,
    int64_t tc_stride, const int32_t* assign_in, int32_t* assign, uint8_t* mask_a,
    int64_t* i_a, uint8_t* mask_b, int64_t* i_b, int64_t* __restrict__ action_out,
    int64_t astride, uint8_t* __restrict__ done, uint8_t* __restrict__ reward, int32_t* status) {
  constexpr int G = 16;
  const int sl = threadIdx.x & (G - 1);
  const int64_t b = (int64_t)blockIdx.x * (256 / G) + (threadIdx.x / G);
  const bool live = b < B;
  const int64_t bb = live ? b : B - 1;  // dead groups mirror the last row (wave-uniform DPP)
  const int U = L >> 2;
  const float4* drow = reinterpret_cast<const float4*>(dist + bb * (int64_t)L);
  const uint32_t* mrow = reinterpret_cast<const uint32_t*>(mask_a + bb * (int64_t)L);
  float4 dv[KU];
  uint32_t mv[KU];
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    const int u = sl + G * k;
    const int uc = u < U ? u : U - 1;
    dv[k] = drow[uc];
    mv[k] = mrow[uc];
  }
  int64_t it = i_a[bb];  // (every lane: one broadcast line)
  bool range = false;
  // per-row pointers formed once (the lane's first mask unit, the row's scalars, the
  // action column advanced by the row stride each step): the step itself does no 64-bit
  // address arithmetic but the product's assignment entry
  uint32_t* const mo_a = reinterpret_cast<uint32_t*>(mask_a + b * (int64_t)L) + sl;
  uint32_t* const mo_b = reinterpret_cast<uint32_t*>(mask_b + b * (int64_t)L) + sl;
  int64_t* const ip_a = i_a + b;
  int64_t* const ip_b = i_b + b;
  int64_t* ap = action_out + b;
  int32_t* const arow = assign + b * P;
  const int32_t* const arow_in = assign_in + b * P;
  const float* tcp = to_choose ? to_choose + bb * tc_stride : nullptr;
#if CO_SLAP_SSORT
  // closest-free = the free locations in increasing (distance, index) order: each lane
  // sorts its candidates once per launch (key: order-preserving u32 of the distance, +inf
  // for a taken location, then the index); a step is a group min over the lanes' heads and
  // a pop by the owner (the head and next key in registers, the rest in LDS) instead of a
  // masked scan of every candidate.  A key not below +inf's is never chosen; with none left
  // the action is 0 and byte 0 is cleared, as the scan's argmin of all-inf does.
  constexpr int EPL = KU == 3 ? 16 : 4 * KU;
  constexpr uint32_t kOrdInf = 0xff800000u;  // ordered key of +inf
  __shared__ uint64_t s_keys[(EPL - 2) * 256];
  uint64_t hk, nk;
  int h = 2;
  {
    uint64_t key[EPL];
#pragma unroll
    for (int k = 0; k < EPL / 4; ++k) {
      const int u = sl + G * k;
      const float d4[4] = {dv[k < KU ? k : 0].x, dv[k < KU ? k : 0].y, dv[k < KU ? k : 0].z,
                           dv[k < KU ? k : 0].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = k < KU && u < U && ((mv[k < KU ? k : 0] >> (8 * j)) & 0xffu);
        // -0.0 keyed as +0.0 (d + 0.0): they tie as in argmin's float compare
        const uint32_t uu = __float_as_uint(ok ? d4[j] + 0.0f : __builtin_inff());
        const uint32_t ord = uu ^ ((uint32_t)((int32_t)uu >> 31) | 0x80000000u);
        key[4 * k + j] = (k < KU && u < U) ? (((uint64_t)ord << 32) | (uint32_t)(4 * u + j)) : ~0ull;
      }
    }
    sort_keys_asc<EPL>(key);
    hk = key[0];
    nk = key[1];
#pragma unroll
    for (int k = 2; k < EPL; ++k) s_keys[(k - 2) * 256 + threadIdx.x] = key[k];
  }
#endif
  // one step: reads the mask units in registers, writes mask row `mo` and i `ip`
  auto step = [&](int t, uint32_t* mo, int64_t* ip) {
    const float prod = tcp ? tcp[t] : (float)(tc_stride + t);
#if CO_SLAP_SSORT
    const uint32_t hh = (uint32_t)(hk >> 32);
    const uint32_t gm = grp_reduce<G>(hh, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
    const uint32_t cand = hh == gm ? (uint32_t)hk : 0xffffffffu;
    const uint32_t gi = grp_reduce<G>(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
    const bool any = gm < kOrdInf;
    const int bi = any ? (int)gi : 0;
    if (any && (uint32_t)hk == gi) {  // the owner's head is the chosen location: pop it
      hk = nk;
      nk = h < EPL ? s_keys[(h - 2) * 256 + threadIdx.x] : ~0ull;
      ++h;
    }
#else
    float best = __builtin_inff();
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      const int u = sl + G * k;
      if (u < U) {
        const float d4[4] = {dv[k].x, dv[k].y, dv[k].z, dv[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = ((mv[k] >> (8 * j)) & 0xffu) ? d4[j] : __builtin_inff();
          if (d < best) {
            best = d;
            bi = 4 * u + j;
          }
        }
        if (bi == 0x7fffffff) bi = 4 * u;
      }
    }
    grp_argmin_split<G>(best, bi);
#endif
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      const int u = sl + G * k;
      const uint32_t clr = (bi >> 2) == u ? ~(0xffu << (8 * (bi & 3))) : ~0u;
      mv[k] &= clr;
    }
    if (live) {
      int p = (int)prod;  // .to(torch.int), slap/env.py:52
      if (p < 0) p += P;
      const bool p_ok = p >= 0 && p < P;
      if (t == 0 && assign_in != assign)  // out of place: the row with [p] = action
        for (int c = sl; c < P; c += G) arow[c] = c == p ? (int32_t)bi : arow_in[c];
#pragma unroll
      for (int k = 0; k < KU; ++k)
        if (sl + G * k < U) mo[G * k] = mv[k];
      if (sl == 0) {
        *ap = bi;
        if (!p_ok)
          range = true;
        else if (t > 0 || assign_in == assign)
          arow[p] = (int32_t)bi;
        done[b] = it == (int64_t)(P - 1);
        *ip = it + 1;
        reward[b] = 0;
      }
    }
    ap += astride;
    it += 1;
  };
  int t = 0;
  for (; t + 1 < K; t += 2) {  // step t reads A and writes B, step t + 1 the reverse
    step(t, mo_b, ip_b);
    step(t + 1, mo_a, ip_a);
  }
  if (t < K) step(t, mo_b, ip_b);
  if (range) set_status(status, CO_ST_INDEX_RANGE);
}

}  // namespace

extern "C" int co_slap_closest_steps(int64_t B, int64_t L, int64_t P, int64_t K,
                                     const float* dist, const float* to_choose, int64_t tc_stride,
                                     const int32_t* assign_in, int32_t* assign, uint8_t* mask_a,
                                     int64_t* i_a, uint8_t* mask_b, int64_t* i_b,
                                     int64_t* action_out, int64_t act_stride, uint8_t* done,
                                     uint8_t* reward, int32_t* status, void* stream) {
  if (B < 0 || L <= 0 || P <= 0 || L > (1 << 30) || K < 0 || K > (1 << 20)) return CO_E_INVAL;
  if (B == 0 || K == 0) return CO_OK;
  if (!dist || !assign_in || !assign || !mask_a || !i_a || !mask_b || !i_b || !action_out ||
      act_stride < B || !done || !reward || !status ||
      (!to_choose && (tc_stride < 0 || tc_stride + K > P)))
    return CO_E_INVAL;
  const bool vec = L % 4 == 0 && L <= 4 * 16 * 4 &&
                   ((reinterpret_cast<uintptr_t>(dist) & 15) |
                    ((reinterpret_cast<uintptr_t>(mask_a) | reinterpret_cast<uintptr_t>(mask_b)) &
                     3)) == 0;
  if (!vec) {  // the K single steps
    for (int64_t t = 0; t < K; ++t) {
      const bool even = (t & 1) == 0;
      const int rc = co_slap_closest_step(
          B, L, P, dist, to_choose ? to_choose + t : nullptr, to_choose ? tc_stride : tc_stride + t,
          t == 0 ? assign_in : assign, assign, even ? mask_a : mask_b, even ? mask_b : mask_a,
          action_out + t * act_stride, even ? i_a : i_b, even ? i_b : i_a, done, reward, status,
          stream);
      if (rc != CO_OK) return rc;
    }
    return CO_OK;
  }
  const dim3 grid(cover_grid(B, 16));
  if (grid.x == 0) return CO_E_INVAL;
  const int units = (int)(L / 4), ku = (units + 15) / 16;
#define CO_SLAP_CSS(KK)                                                                        \
  hipLaunchKernelGGL((slap_closest_steps_kernel<KK>), grid, dim3(256), 0, (hipStream_t)stream, \
                     B, (int)L, (int)P, (int)K, dist, to_choose, tc_stride, assign_in, assign,  \
                     mask_a, i_a, mask_b, i_b, action_out, act_stride, done, reward, status)
  switch (ku) {
    case 1: CO_SLAP_CSS(1); break;
    case 2: CO_SLAP_CSS(2); break;
    case 3: CO_SLAP_CSS(3); break;
    default: CO_SLAP_CSS(4);
  }
#undef CO_SLAP_CSS
  return launch_status();
}

extern "C" int co_slap_reset(int64_t B, int64_t L, int64_t P, uint8_t* mask, float* to_choose,
                             int64_t* it, float* reward, float* ratio, uint8_t* done,
                             uint8_t* terminated, void* stream) {
  if (B < 0 || L <= 0 || P <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!mask || !to_choose || !it || !reward) return CO_E_INVAL;
  hipLaunchKernelGGL(slap_reset_kernel, dim3(grid_for(B * L / 16 + 1, 256)), dim3(256), 0,
                     (hipStream_t)stream, B, L, P, mask, to_choose, it, reward, ratio, done,
                     terminated);
  return launch_status();
}

extern "C" int co_slap_step(int64_t B, int64_t L, int64_t P, const int64_t* action,
                            const float* to_choose, int64_t tc_stride, const int32_t* assign_in,
                            int32_t* assign_out, const uint8_t* mask_in, uint8_t* mask_out,
                            const int64_t* i_in, int64_t* i_out, uint8_t* done, uint8_t* reward,
                            int32_t* status, void* stream) {
  if (B < 0 || L <= 0 || P <= 0 || L > (1 << 30)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !assign_in || !assign_out || !mask_in || !mask_out || !i_in || !i_out || !done ||
      !reward || (!to_choose && (tc_stride < 0 || tc_stride >= P)))
    return CO_E_INVAL;
  // 16 lanes per instance (the closest-step layout without the policy) for L % 4 == 0,
  // L <= 256 and 4-B-aligned mask rows; else the 64-row byte tile
  if (CO_SLAP_GROUP_STEP && L % 4 == 0 && L <= 256 &&
      ((reinterpret_cast<uintptr_t>(mask_in) | reinterpret_cast<uintptr_t>(mask_out)) & 3) == 0) {
    const dim3 grid(cover_grid(B, 16));
    if (grid.x == 0) return CO_E_INVAL;
    const int ku = (int)((L / 4 + 15) / 16);
#define CO_SLAP_GS(K)                                                                         \
  hipLaunchKernelGGL((slap_closest_step_kernel<K, false>), grid, dim3(256), 0,               \
                     (hipStream_t)stream, B, (int)L, (int)P, nullptr, mask_in, mask_out, action, \
                     nullptr, to_choose, tc_stride, assign_in, assign_out, i_in, i_out, done,  \
                     reward, status)
    switch (ku) {
      case 1: CO_SLAP_GS(1); break;
      case 2: CO_SLAP_GS(2); break;
      case 3: CO_SLAP_GS(3); break;
      default: CO_SLAP_GS(4);
    }
#undef CO_SLAP_GS
    return launch_status();
  }
  SlapRowEpilogue epi{(int)P, to_choose, tc_stride, assign_out, i_in, i_out, done, reward,
                      status};
  const unsigned grid = cover_grid(B, kTileRows, kTileThreads);
  if (grid == 0) return CO_E_INVAL;
  hipLaunchKernelGGL(slap_step_kernel, dim3(grid), dim3(kTileThreads), 0, (hipStream_t)stream, B,
                     (int)L, action, mask_in, mask_out, assign_in, epi,
                     tile_vec_ok(mask_in, mask_out));
  return launch_status();
}

extern "C" int co_slap_reward(int64_t B, int64_t L, int64_t P, int64_t O, int64_t K,
                              const int32_t* assignment, const int64_t* picklist,
                              const float* locs, float* reward, int32_t* status, void* stream) {
  if (B < 0 || L <= 0 || P <= 0 || O <= 0 || K <= 0 || O * K > (1 << 16)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!assignment || !picklist || !locs || !reward) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  // lane group per instance (16 lanes, 16 instances per workgroup) when the instance's
  // rows fit the per-lane register slots: L <= 128, P <= 32, S <= 128
  if (CO_SLAP_RGROUP && L <= 16 * 8 && P <= 16 * 2 && O * K <= 16 * 8) {
    const size_t shmem = (size_t)16 * slap_rg_bytes((int)L, (int)P, (int)(O * K), (int)O);
    if (shmem <= 64 * 1024) {
      hipLaunchKernelGGL((slap_reward_group_kernel<16, 8, 2, 8>), dim3((unsigned)((B + 15) / 16)),
                         dim3(256), shmem, (hipStream_t)stream, B, (int)L, (int)P, (int)O,
                         (int)K, assignment, picklist, reinterpret_cast<const float2*>(locs),
                         reward, status);
      return launch_status();
    }
  }
  // per wave, in float2 units: locations L, picks S, order lengths O (as floats, rounded
  // up to float2 with the assignment ints)
  const size_t per_wave = (size_t)(L + O * K + O + (P + 1) / 2) * sizeof(float2);
  if (per_wave > 64 * 1024) {  // beyond the LDS staging: coordinates gathered from L2
    hipLaunchKernelGGL(slap_reward_global_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                       (hipStream_t)stream, B, (int)L, (int)P, (int)O, (int)K, assignment,
                       picklist, reinterpret_cast<const float2*>(locs), reward, status);
    return launch_status();
  }
  int waves = 4;
  while (waves > 1 && per_wave * waves > 64 * 1024) waves >>= 1;
  const dim3 grid(grid_for(B, waves, 256 * 32));
  const size_t shmem = (size_t)waves * per_wave;
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  switch (waves) {
    case 4:
      hipLaunchKernelGGL(slap_reward_kernel<4>, grid, dim3(256), shmem, (hipStream_t)stream, B,
                         (int)L, (int)P, (int)O, (int)K, assignment, picklist, l2, reward, status);
      break;
    case 2:
      hipLaunchKernelGGL(slap_reward_kernel<2>, grid, dim3(128), shmem, (hipStream_t)stream, B,
                         (int)L, (int)P, (int)O, (int)K, assignment, picklist, l2, reward, status);
      break;
    default:
      hipLaunchKernelGGL(slap_reward_kernel<1>, grid, dim3(64), shmem, (hipStream_t)stream, B,
                         (int)L, (int)P, (int)O, (int)K, assignment, picklist, l2, reward, status);
  }
  return launch_status();
}

extern "C" int co_slap_closest_free_action(int64_t B, int64_t L, const float* dist,
                                           const uint8_t* mask, int64_t* out, void* stream) {
  if (B < 0 || L <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!dist || !mask || !out) return CO_E_INVAL;
  hipLaunchKernelGGL(slap_closest_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)L, dist, mask, out);
  return launch_status();
}

extern "C" int co_slap_closest_step(int64_t B, int64_t L, int64_t P, const float* dist,
                                    const float* to_choose, int64_t tc_stride,
                                    const int32_t* assign_in, int32_t* assign,
                                    const uint8_t* mask_in, uint8_t* mask_out, int64_t* action_out,
                                    const int64_t* i_in, int64_t* i_out, uint8_t* done,
                                    uint8_t* reward, int32_t* status, void* stream) {
  if (B < 0 || L <= 0 || P <= 0 || L > (1 << 30)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!dist || !assign_in || !assign || !mask_in || !mask_out || !action_out || !i_in || !i_out ||
      !done || !reward || (!to_choose && (tc_stride < 0 || tc_stride >= P)))
    return CO_E_INVAL;
  const bool vec = L % 4 == 0 && L <= 4 * 16 * 4 &&
                   ((reinterpret_cast<uintptr_t>(dist) & 15) |
                    ((reinterpret_cast<uintptr_t>(mask_in) | reinterpret_cast<uintptr_t>(mask_out)) &
                     3)) == 0;
  if (!vec) {  // the two launches it fuses
    int rc = co_slap_closest_free_action(B, L, dist, mask_in, action_out, stream);
    if (rc != CO_OK) return rc;
    return co_slap_step(B, L, P, action_out, to_choose, tc_stride, assign_in, assign, mask_in,
                        mask_out, i_in, i_out, done, reward, status, stream);
  }
  const dim3 grid(cover_grid(B, 16));
  if (grid.x == 0) return CO_E_INVAL;
  const int units = (int)(L / 4), ku = (units + 15) / 16;
#define CO_SLAP_CS(K)                                                                        \
  hipLaunchKernelGGL((slap_closest_step_kernel<K, true>), grid, dim3(256), 0, (hipStream_t)stream, \
                     B, (int)L, (int)P, dist, mask_in, mask_out, nullptr, action_out, to_choose, tc_stride, \
                     assign_in, assign, i_in, i_out, done, reward, status)
  switch (ku) {
    case 1: CO_SLAP_CS(1); break;
    case 2: CO_SLAP_CS(2); break;
    case 3: CO_SLAP_CS(3); break;
    default: CO_SLAP_CS(4);
  }
#undef CO_SLAP_CS
  return launch_status();
}


// ---------------------------------------------------------------- instance generator
// The deterministic part of SLAPGenerator._generate (slap/generator.py:51-81,137-155) on
// the device: aisle-grid coordinates x = aisle * inter_aisle_dist, y = loc *
// inter_loc_dist (python float products rounded to f32), the Manhattan matrix
// |dx| + |dy| in f32 (one rounding, as torch.sum over the size-2 dim), its depot row, and
// the -1 assignment.  freq and picklist come from the host RNG streams.
namespace {
__device__ __forceinline__ float2 slap_xy(int i, int n_locs, double inter_aisle,
                                          double inter_loc) {
  return make_float2((float)((double)(i / n_locs) * inter_aisle),
                     (float)((double)(i % n_locs) * inter_loc));
}

__global__ __launch_bounds__(256) void slap_gen_rows_kernel(int64_t B, int L, int P, int n_locs,
                                                            double inter_aisle, double inter_loc,
                                                            float2* __restrict__ locs,
                                                            float* __restrict__ depot,
                                                            int32_t* __restrict__ assign) {
  const float2 p0 = slap_xy(0, n_locs, inter_aisle, inter_loc);
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < B * L;
       k += (int64_t)gridDim.x * blockDim.x) {
    const float2 q = slap_xy((int)(k % L), n_locs, inter_aisle, inter_loc);
    locs[k] = q;
    depot[k] = fabsf(p0.x - q.x) + fabsf(p0.y - q.y);
  }
  if (assign)
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < B * P;
         k += (int64_t)gridDim.x * blockDim.x)
      assign[k] = -1;
}

// dist_mat[b, i, j]: every instance has the same grid; 4 consecutive j per thread
// (float4 stores when L % 4 == 0).
__global__ __launch_bounds__(256) void slap_gen_dist_kernel(int64_t B, int L, int n_locs,
                                                            double inter_aisle, double inter_loc,
                                                            float* __restrict__ dist) {
  const int64_t LL = (int64_t)L * L;
  const bool vec = (L & 3) == 0;
  const int64_t units = vec ? B * (LL / 4) : B * LL;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units;
       u += (int64_t)gridDim.x * blockDim.x) {
    if (vec) {
      const int64_t e = u * 4, r = e % LL;
      const int i = (int)(r / L), j = (int)(r % L);
      const float2 p = slap_xy(i, n_locs, inter_aisle, inter_loc);
      float d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 o = slap_xy(j + q, n_locs, inter_aisle, inter_loc);
        d[q] = fabsf(p.x - o.x) + fabsf(p.y - o.y);
      }
      *reinterpret_cast<float4*>(dist + e) = make_float4(d[0], d[1], d[2], d[3]);
    } else {
      const int64_t r = u % LL;
      const float2 p = slap_xy((int)(r / L), n_locs, inter_aisle, inter_loc);
      const float2 o = slap_xy((int)(r % L), n_locs, inter_aisle, inter_loc);
      dist[u] = fabsf(p.x - o.x) + fabsf(p.y - o.y);
    }
  }
}
}  // namespace

extern "C" int co_slap_generate(int64_t B, int64_t n_aisles, int64_t n_locs,
                                double inter_aisle_dist, double inter_loc_dist,
                                int64_t n_products, float* locs, float* depot_loc_dist,
                                float* dist_mat, int32_t* assignment, void* stream) {
  if (B < 0 || n_aisles <= 0 || n_locs <= 0 || n_products < 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !depot_loc_dist) return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(locs) & 7) || (reinterpret_cast<uintptr_t>(dist_mat) & 15))
    return CO_E_ALIGN;
  const int L = (int)(n_aisles * n_locs);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(slap_gen_rows_kernel, dim3(grid_for(B * L, 256, 8192)), dim3(256), 0, s, B,
                     L, (int)n_products, (int)n_locs, inter_aisle_dist, inter_loc_dist,
                     reinterpret_cast<float2*>(locs), depot_loc_dist, assignment);
  if (dist_mat)
    hipLaunchKernelGGL(slap_gen_dist_kernel, dim3(grid_for(B * L * L / 4 + 1, 256, 16384)),
                       dim3(256), 0, s, B, L, (int)n_locs, inter_aisle_dist, inter_loc_dist,
                       dist_mat);
  return launch_status();
}
