// co_slap_decode_step / co_cvrp_decode_step: the decode step (rl4co/utils/decoding.py:
// 141-191, 327-399, 489-499) fused with the env transition of the selected action, so a
// ConstructivePolicy loop over SLAPEnv / CVRPEnv is one launch per step (as
// co_tsp_decode_step is for TSP):
//   * SLAP (slap/env.py:38-93): assignment[b, to_choose[b, 0]] = action (the row copied
//     when the output is a fresh buffer: the reference clones), action_mask minus the
//     action, done = (i == P-1), i + 1, reward = 0;
//   * CVRP (cvrp/env.py:73-149): used = (used + demand[clamp(a-1)]) * (a != 0), visited[a]
//     = 1, done = sum(visited) == N+1, reward = 0, and get_action_mask recomputed from the
//     new state (the strict `demand + used > capacity` test, the depot rule).
// The row engines are decode_common.hpp's (GreedyRow for greedy, certified by default;
// DecodeRow for sampling / evaluate), with the same lane ownership: lane sl of an RL-lane
// group owns the row's EPL consecutive columns c0 = sl*EPL .. c0+EPL-1.  The env's own
// per-column data (SLAP: nothing; CVRP: the visited bytes and demand[c-1] of those
// columns) is loaded by the same lanes in the same 4-column chunks, issued together with
// the logits, so the transition needs no second memory round trip: the selected
// column's demand comes from its owner lane by one shuffle, the row sums (visited count,
// "any customer feasible") are group reductions.  Outputs are the two-launch path's
// (co_decode_step + co_slap_step / co_cvrp_step) bit for bit, RNG use included.
#include "decode_common.hpp"

namespace {

// ------------------------------------------------------------------ SLAP transition
struct SlapEpi {
  int P;
  const float* to_choose;
  int64_t tc_stride;
  const int32_t* assign_in;
  int32_t* assign_out;
  uint8_t* mask_out;
  const int64_t* i_in;
  int64_t* i_out;
  uint8_t* done;
  uint8_t* reward;
};

// The row's SLAP scalars and (out of place) the assignment row, loaded with the logits.
template <int RL>
struct SlapRow {
  static constexpr int AU = 2;  // assignment entries per lane held in registers (P <= 2*RL)
  int64_t it = 0;
  float prod = 0.f;
  int32_t av[AU];

  __device__ __forceinline__ void load(const SlapEpi& e, bool valid, int64_t r, int sl) {
    if (valid) prod = e.to_choose[r * e.tc_stride];  // one address per group: a broadcast
    if (valid && sl == 0) it = e.i_in[r];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int c = sl + RL * u;
      av[u] = (valid && e.assign_in != e.assign_out && c < e.P) ? e.assign_in[r * e.P + c] : 0;
    }
  }

  // slap/env.py:50-62 for action a_raw (python indexing already applied to the mask by
  // the caller); `sl == 0` writes the row scalars.  Returns false when the product index
  // is out of range (the reference's advanced-index write raises).
  __device__ __forceinline__ bool store(const SlapEpi& e, int64_t r, int sl, int64_t a_raw) const {
    int64_t p = (int64_t)(int)prod;  // .to(torch.int), slap/env.py:52
    if (p < 0) p += e.P;
    const bool p_ok = p >= 0 && p < e.P;
    const int32_t av_new = (int32_t)a_raw;  // .to(torch.int), slap/env.py:53-54
    if (e.assign_in != e.assign_out) {      // the clone with [p] = action
#pragma unroll
      for (int u = 0; u < AU; ++u) {
        const int c = sl + RL * u;
        if (c < e.P) e.assign_out[r * e.P + c] = c == p ? av_new : av[u];
      }
      for (int c = sl + RL * AU; c < e.P; c += RL)
        e.assign_out[r * e.P + c] = c == p ? av_new : e.assign_in[r * e.P + c];
    } else if (sl == 0 && p_ok) {
      e.assign_out[r * e.P + p] = av_new;
    }
    if (sl == 0) {
      e.done[r] = it == (int64_t)(e.P - 1);  // slap/env.py:57
      e.i_out[r] = it + 1;
      e.reward[r] = 0;
    }
    return p_ok;
  }
};

// Greedy (GreedyRow; certified / exact / fast per OPT) decode + SLAP step.
template <int RL, int EPL, int VW, int OPT>
__global__ __launch_bounds__(256) void slap_decode_greedy_kernel(
    int64_t B, int L, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, float* __restrict__ ll_accum, int32_t* status, SlapEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int64_t base = wid * RPW; base < B; base += nwaves * RPW) {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    SlapRow<RL> sr;
    sr.load(e, valid, r, sl);
    const float acc = (valid && sl == 0 && ll_accum) ? ll_accum[r] : 0.f;
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask_in + r * (int64_t)L;
    g.load(valid, L, lrow, mrow, c0);
    float lp, lse;
    const int sel = greedy_row<OPT>(g, valid, L, clip, temp, sl, c0,
                                           group_scratch<RL, EPL>(lds, grp), lse, lp, lrow, mrow);
    const bool feas0 = g.allowed(0);
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {  // the selected location leaves the mask
      const int off = sel - (c0 + 4 * j);
      if ((unsigned)off < 4u) g.mw[j] &= ~(0xffu << (8 * off));
    }
    if (!valid) continue;  // no group operation below
    g.store_mask(L, e.mask_out + r * (int64_t)L, c0);
    const bool p_ok = sr.store(e, r, sl, sel);
    if (sl == 0) {
      if (lse != lse && !feas0) set_status(status, CO_ST_INFEASIBLE);
      if (!p_ok) set_status(status, CO_ST_INDEX_RANGE);
      action_out[r] = sel;
      if (logp_sel) logp_sel[r] = lp;
      if (ll_accum) ll_accum[r] = acc + lp;
    }
  }
}

// Sampling / evaluate (DecodeRow, exact math unless fast) decode + SLAP step.
template <int RL, int EPL, bool VEC, int OPT>
__global__ __launch_bounds__(256) void slap_decode_step_kernel(
    int64_t B, int L, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, float* __restrict__ ll_accum,
    int32_t* status, SlapEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int64_t base = wid * RPW; base < B; base += nwaves * RPW) {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    const int64_t a_in = (mode == CO_DECODE_EVALUATE && valid) ? action_in[r] : 0;
    SlapRow<RL> sr;
    sr.load(e, valid, r, sl);
    const float acc = (valid && sl == 0 && ll_accum) ? ll_accum[r] : 0.f;
    DecodeRow<RL, EPL, VEC, OPT> d;
    d.run(valid, L, logits + r * lstride, mask_in + r * (int64_t)L, clip, temp, mode, a_in, seed,
          offset, row, sl, grp, group_scratch<RL, EPL>(lds, grp));
    const int64_t a_raw = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d.sel;
    const int64_t a = a_raw < 0 ? a_raw + L : a_raw;  // slap/env.py:62 (python indexing)
    const bool a_ok = a >= 0 && a < L;
#pragma unroll
    for (int k = 0; k < EPL; ++k)
      if (a_ok && c0 + k == a) d.mk[k] = 0;
    if (!valid) continue;
    uint8_t* orow = e.mask_out + r * (int64_t)L;
    if (VEC) {
#pragma unroll
      for (int j = 0; j < EPL / 4; ++j)
        if (c0 + 4 * j < L)
          *reinterpret_cast<uint32_t*>(orow + c0 + 4 * j) =
              (uint32_t)d.mk[4 * j] | ((uint32_t)d.mk[4 * j + 1] << 8) |
              ((uint32_t)d.mk[4 * j + 2] << 16) | ((uint32_t)d.mk[4 * j + 3] << 24);
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (c0 + k < L) orow[c0 + k] = d.mk[k];
    }
    const bool p_ok = sr.store(e, r, sl, a_raw);
    if (sl == 0) {
      if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= L))
        set_status(status, CO_ST_INDEX_RANGE);  // the logp gather (decoding.py:365)
      if (mode != CO_DECODE_EVALUATE && !d.feas) set_status(status, CO_ST_INFEASIBLE);
      if (!a_ok || !p_ok) set_status(status, CO_ST_INDEX_RANGE);
      action_out[r] = a_raw;
      if (logp_sel) logp_sel[r] = d.lp;
      if (ll_accum) ll_accum[r] = acc + d.lp;
    }
  }
}

// ------------------------------------------------------------------ CVRP transition
struct CvrpEpi {
  int N;  // customers; rows are N + 1 columns (depot first)
  const float* demand;
  const float* used_in;
  float* used_out;
  const float* vcap;
  const uint8_t* vis_in;
  uint8_t* vis_out;
  int64_t* cur_out;
  uint8_t* done;
  uint8_t* reward;
  uint8_t* mask_out;
};

// The lane's EPL columns of a CVRP row: visited bytes as 4-column words, the demand of
// each column (column c: demand[c - 1]; the depot column's slot unused), the row
// scalars.  Loads are Chunk<3> accesses (byte-aligned dwords, dword-aligned dwordx4):
// the [B, N+1] byte rows and the [B, N] demand rows are aligned to neither.
template <int EPL>
struct CvrpRow {
  uint32_t vw[EPL / 4];
  float dm[EPL];
  float used = 0.f, cap = 0.f;

  __device__ __forceinline__ void load(const CvrpEpi& e, bool valid, int64_t r, int c0) {
    using F = typename Chunk<3>::F;
    using M = typename Chunk<3>::M;
    const int NC = e.N + 1;
    const uint8_t* vrow = e.vis_in + r * (int64_t)NC;
    const float* drow = e.demand + r * (int64_t)e.N;
    if (valid) {  // every lane: the row's scalars (one address per group: a broadcast)
      used = e.used_in[r];
      cap = e.vcap[r];
    }
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      uint32_t v = 0u;
      float d[4] = {0.f, 0.f, 0.f, 0.f};
      if (valid && c >= 4 && c + 4 <= NC) {  // interior chunk: demand[c-1 .. c+2]
        v = (uint32_t) * reinterpret_cast<const M*>(vrow + c);
        const F x = *reinterpret_cast<const F*>(drow + (c - 1));
        d[0] = x[0];
        d[1] = x[1];
        d[2] = x[2];
        d[3] = x[3];
      } else if (valid && c < NC) {  // the depot's chunk / the row's partial last chunk
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (c + q < NC) {
            v |= (uint32_t)vrow[c + q] << (8 * q);
            if (c + q >= 1) d[q] = drow[c + q - 1];
          }
      }
      vw[j] = v;
#pragma unroll
      for (int q = 0; q < 4; ++q) dm[4 * j + q] = d[q];
    }
  }

  // cvrp/env.py:73-105 + get_action_mask (:137-149) for action a_raw, the same
  // arithmetic as co_cvrp_step.  Group-wide (every lane of the wave active); returns
  // done and writes the visited / mask rows and (sl == 0) the row scalars.
  template <int RL>
  __device__ __forceinline__ void apply(const CvrpEpi& e, bool valid, int64_t r, int sl, int grp,
                                        int c0, int64_t a_raw, int32_t* status) {
    const int N = e.N, NC = N + 1;
    const bool bad = a_raw < 0 || a_raw > N;
    // selected demand demand[clamp(a - 1, 0, N - 1)] (column csel) from its owner lane
    const int csel = (int)(a_raw - 1 < 0 ? 0 : (a_raw - 1 > N - 1 ? N - 1 : a_raw - 1)) + 1;
    const int owner = grp * RL + csel / EPL, slot = csel % EPL;
    float mine = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) mine = k == slot ? dm[k] : mine;
    const float dsel = __shfl(mine, owner, 64);
    const float u = (used + dsel) * ((a_raw != 0) ? 1.0f : 0.0f);
    const int a = bad ? -1 : (int)a_raw;
    uint32_t mk[EPL / 4];
    uint32_t cnt = 0u;
    bool feas = false;
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      const int nown = valid ? (NC - c < 0 ? 0 : (NC - c > 4 ? 4 : NC - c)) : 0;
      const uint32_t own = nown >= 4 ? 0xffffffffu : (1u << (8 * nown)) - 1u;
      const uint32_t cust = c == 0 ? own & ~0xffu : own;  // the depot column excluded
      uint32_t x = vw[j];
      const int ea = a - c;  // the action's byte, if in this chunk: scatter(..., 1)
      if (a >= 0 && ea >= 0 && ea < 4) x = (x & ~(0xffu << (8 * ea))) | (1u << (8 * ea));
      vw[j] = x;
      const uint32_t over = ((dm[4 * j] + u > cap) ? 0x80u : 0u) |
                            ((dm[4 * j + 1] + u > cap) ? 0x8000u : 0u) |
                            ((dm[4 * j + 2] + u > cap) ? 0x800000u : 0u) |
                            ((dm[4 * j + 3] + u > cap) ? 0x80000000u : 0u);
      const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
      const uint32_t m = ((~(nz | over) & 0x80808080u) >> 7) & cust;
      cnt = __builtin_amdgcn_sad_u8(x & own, 0u, cnt);
      feas |= m != 0u;
      mk[j] = m;
    }
    cnt = grp_reduce<RL>(cnt, [](uint32_t x, uint32_t y) { return x + y; });
    const uint64_t gm = RL == 64 ? ~0ull : ((1ull << RL) - 1ull);
    const bool anyf = ((__ballot(feas) >> (RL * grp)) & gm) != 0ull;
    if (!valid) return;
    if (sl == 0) mk[0] |= (uint32_t) !((a_raw == 0) && anyf);  // cvrp/env.py:146-148
    using M = typename Chunk<3>::M;
    uint8_t* vdst = e.vis_out + r * (int64_t)NC;
    uint8_t* mdst = e.mask_out + r * (int64_t)NC;
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      if (c + 4 <= NC) {
        *reinterpret_cast<M*>(vdst + c) = (M)vw[j];
        *reinterpret_cast<M*>(mdst + c) = (M)mk[j];
      } else if (c < NC) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (c + q < NC) {
            vdst[c + q] = (uint8_t)(vw[j] >> (8 * q));
            mdst[c + q] = (uint8_t)(mk[j] >> (8 * q));
          }
      }
    }
    if (sl == 0) {
      if (bad) set_status(status, CO_ST_INDEX_RANGE);
      e.used_out[r] = u;
      if (e.cur_out) e.cur_out[r] = a_raw;
      e.done[r] = (int)cnt == NC;
      e.reward[r] = 0;
    }
  }
};

template <int RL, int EPL, int VW, int OPT>
__global__ __launch_bounds__(256) void cvrp_decode_greedy_kernel(
    int64_t B, int NC, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, float* __restrict__ ll_accum, int32_t* status, CvrpEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int64_t base = wid * RPW; base < B; base += nwaves * RPW) {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    CvrpRow<EPL> cr;
    cr.load(e, valid, r, c0);
    const float acc = (valid && sl == 0 && ll_accum) ? ll_accum[r] : 0.f;
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask_in + r * (int64_t)NC;
    g.load(valid, NC, lrow, mrow, c0);
    float lp, lse;
    const int sel = greedy_row<OPT>(g, valid, NC, clip, temp, sl, c0,
                                           group_scratch<RL, EPL>(lds, grp), lse, lp, lrow, mrow);
    const bool feas0 = g.allowed(0);
    cr.template apply<RL>(e, valid, r, sl, grp, c0, sel, status);
    if (valid && sl == 0) {
      if (lse != lse && !feas0) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = sel;
      if (logp_sel) logp_sel[r] = lp;
      if (ll_accum) ll_accum[r] = acc + lp;
    }
  }
}

template <int RL, int EPL, bool VEC, int OPT>
__global__ __launch_bounds__(256) void cvrp_decode_step_kernel(
    int64_t B, int NC, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, float* __restrict__ ll_accum,
    int32_t* status, CvrpEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int64_t base = wid * RPW; base < B; base += nwaves * RPW) {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    const int64_t a_in = (mode == CO_DECODE_EVALUATE && valid) ? action_in[r] : 0;
    CvrpRow<EPL> cr;
    cr.load(e, valid, r, c0);
    const float acc = (valid && sl == 0 && ll_accum) ? ll_accum[r] : 0.f;
    DecodeRow<RL, EPL, VEC, OPT> d;
    d.run(valid, NC, logits + r * lstride, mask_in + r * (int64_t)NC, clip, temp, mode, a_in,
          seed, offset, row, sl, grp, group_scratch<RL, EPL>(lds, grp));
    const int64_t a_raw = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d.sel;
    cr.template apply<RL>(e, valid, r, sl, grp, c0, a_raw, status);
    if (valid && sl == 0) {
      if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= NC))
        set_status(status, CO_ST_INDEX_RANGE);
      if (mode != CO_DECODE_EVALUATE && !d.feas) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = a_raw;
      if (logp_sel) logp_sel[r] = d.lp;
      if (ll_accum) ll_accum[r] = acc + d.lp;
    }
  }
}

}  // namespace

extern "C" int co_slap_decode_step(int64_t B, int64_t L, int64_t P, const float* logits,
                                   int64_t lstride, const uint8_t* mask_in, float clip, float temp,
                                   int mode, const int64_t* action_in, int64_t* action_out,
                                   float* logp_sel, uint64_t seed, uint64_t offset,
                                   const float* to_choose, int64_t tc_stride,
                                   const int32_t* assign_in, int32_t* assign_out,
                                   uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                                   uint8_t* done, uint8_t* step_reward, float* ll_accum,
                                   int32_t* status, void* stream) {
  if (B < 0 || L <= 0 || L > 64 * 32 || P <= 0 || P > (1 << 24)) return CO_E_INVAL;
  const bool cert = (mode & CO_DECODE_CERTIFIED) != 0 && (mode & CO_DECODE_FAST) == 0;
  const bool fast = (mode & CO_DECODE_FAST) != 0;
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (mode < 0 || mode > 2) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !mask_in || !action_out || !to_choose || !assign_in || !assign_out ||
      !mask_out || !i_in || !i_out || !done || !step_reward ||
      (mode == CO_DECODE_EVALUATE && !action_in))
    return CO_E_INVAL;
  if (mask_out == mask_in) return CO_E_INVAL;  // the mask is read by other lanes' decode
  const SlapEpi epi{(int)P, to_choose, tc_stride, assign_in, assign_out, mask_out,
                    i_in,   i_out,     done,      step_reward};
  const int64_t N = L;  // the row-dispatch macros' name for the row length
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(decode_grid(B, (int)N)), block(256);
  if (mode == CO_DECODE_GREEDY) {
#define CO_SDG(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL,                                                        \
                    (slap_decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), grid, block, \
                    0, s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out,         \
                    logp_sel, ll_accum, status, epi)
    switch (greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr)) {
      case 4: CO_ROW_DISPATCH(CO_SDG, 4); break;
      default: CO_ROW_DISPATCH(CO_SDG, 3);
    }
#undef CO_SDG
    return launch_status();
  }
#define CO_SDS(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (slap_decode_step_kernel<RL, EPL, V, OPT>), grid, block, \
                  0, s, B, (int)N, logits, lstride, mask_in, clip, temp, mode, action_in,       \
                  action_out, logp_sel, seed, offset, ll_accum, status, epi)
  if (decode_vec_ok(logits, lstride, mask_in, N) &&
      (reinterpret_cast<uintptr_t>(mask_out) & 3) == 0) {
    CO_ROW_DISPATCH(CO_SDS, true);
  } else {
    CO_ROW_DISPATCH(CO_SDS, false);
  }
#undef CO_SDS
  (void)cert;
  return launch_status();
}

extern "C" int co_cvrp_decode_step(int64_t B, int64_t Ncust, const float* logits,
                                   int64_t lstride, const uint8_t* mask_in, float clip, float temp,
                                   int mode, const int64_t* action_in, int64_t* action_out,
                                   float* logp_sel, uint64_t seed, uint64_t offset,
                                   const float* demand, const float* used_in, float* used_out,
                                   const float* vcap, const uint8_t* vis_in, uint8_t* vis_out,
                                   int64_t* cur_out, uint8_t* done, uint8_t* step_reward,
                                   uint8_t* mask_out, float* ll_accum, int32_t* status,
                                   void* stream) {
  if (B < 0 || Ncust <= 0 || Ncust + 1 > 64 * 32) return CO_E_INVAL;
  const bool cert = (mode & CO_DECODE_CERTIFIED) != 0 && (mode & CO_DECODE_FAST) == 0;
  const bool fast = (mode & CO_DECODE_FAST) != 0;
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (mode < 0 || mode > 2) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !mask_in || !action_out || !demand || !used_in || !used_out || !vcap ||
      !vis_in || !vis_out || !done || !step_reward || !mask_out ||
      (mode == CO_DECODE_EVALUATE && !action_in))
    return CO_E_INVAL;
  // every lane reads its own columns of the input rows before any lane writes: in-place
  // visited / mask rows are fine within a row, but a lane group's stores must not reach
  // another group's unread row, so the outputs are separate buffers
  if (mask_out == mask_in || vis_out == vis_in) return CO_E_INVAL;
  const CvrpEpi epi{(int)Ncust, demand,  used_in, used_out, vcap,       vis_in,
                    vis_out,    cur_out, done,    step_reward, mask_out};
  const int64_t N = Ncust + 1;  // row length (depot + customers)
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(decode_grid(B, (int)N)), block(256);
  if (mode == CO_DECODE_GREEDY) {
#define CO_CDG(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL,                                                        \
                    (cvrp_decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), grid, block, \
                    0, s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out,         \
                    logp_sel, ll_accum, status, epi)
    switch (greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr)) {
      case 4: CO_ROW_DISPATCH(CO_CDG, 4); break;
      default: CO_ROW_DISPATCH(CO_CDG, 3);
    }
#undef CO_CDG
    return launch_status();
  }
#define CO_CDS(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (cvrp_decode_step_kernel<RL, EPL, V, OPT>), grid, block, \
                  0, s, B, (int)N, logits, lstride, mask_in, clip, temp, mode, action_in,       \
                  action_out, logp_sel, seed, offset, ll_accum, status, epi)
  if (decode_vec_ok(logits, lstride, mask_in, N)) {
    CO_ROW_DISPATCH(CO_CDS, true);
  } else {
    CO_ROW_DISPATCH(CO_CDS, false);
  }
#undef CO_CDS
  (void)cert;
  return launch_status();
}
