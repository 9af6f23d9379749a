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

#ifndef CO_DECODE_STAGE
#define CO_DECODE_STAGE 0  // rows by non-temporal LDS-DMA (r06: TSP decode step 16.0 -> 17.9 us,
                           // SLAP 12.1 -> 13.0 us at B = 65,536: off)
#endif

namespace {

// ------------------------------------------------------------------ env staging
// The env data a row's transition needs is fetched into the wave's LDS by LDS-DMA
// (global_load_lds_dword: each lane one dword from its own address, no VGPR destination)
// before the row's logits are loaded, so it is in flight with them and holds no register
// through the decode -- the decode's registers (and the certified kernels' exact fallback)
// set the kernel's VGPR count, as in co_tsp_decode_step.  The decode's wait for its logits
// (vmcnt counts in issue order) also covers the DMA; the transition reads the stage after
// an explicit drain + wave barrier.
// Whole 64-lane pieces carry no per-lane predicate (a branch per DMA instruction cost more
// VALU / SALU than the copy itself); only the tail piece masks lanes.
#ifndef CO_ENVSTAGE_AUX
#define CO_ENVSTAGE_AUX 0  // cache-policy bits of the env staging DMA (2 = nt)
#endif
template <class F>
__device__ __forceinline__ void dma_dwords(int n, uint32_t* lds_dst, F src) {
  const int lane = lane_id();
  int base = 0;
  for (; base + 64 <= n; base += 64)  // wave-uniform trip count
    __builtin_amdgcn_global_load_lds((const void*)src(base + lane), (lds_void*)(lds_dst + base), 4,
                                     0, CO_ENVSTAGE_AUX);
  if (base < n && lane < n - base)
    __builtin_amdgcn_global_load_lds((const void*)src(base + lane), (lds_void*)(lds_dst + base), 4,
                                     0, CO_ENVSTAGE_AUX);
}

// n4 16-byte units (src(k): the k-th, 16-byte aligned) to a 16-byte aligned LDS destination:
// gfx950's global_load_lds_dwordx4, a quarter of the instructions of dma_dwords
template <class F>
__device__ __forceinline__ void dma_dwordx4(int n4, uint32_t* lds_dst, F src) {
  const int lane = lane_id();
  int base = 0;
  for (; base + 64 <= n4; base += 64)
    __builtin_amdgcn_global_load_lds((const void*)src(base + lane), (lds_void*)(lds_dst + 4 * base),
                                     16, 0, CO_ENVSTAGE_AUX);
  if (base < n4 && lane < n4 - base)
    __builtin_amdgcn_global_load_lds((const void*)src(base + lane), (lds_void*)(lds_dst + 4 * base),
                                     16, 0, CO_ENVSTAGE_AUX);
}

__device__ __forceinline__ void stage_ready() {
  __builtin_amdgcn_s_waitcnt(0);  // every DMA (and any pending load) landed
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
  float* ll_accum;
};

// Per wave (RPW rows): [i_in: 2 RPW dwords][product: RPW][ll: RPW][assignment: RPW * P]
__host__ __device__ inline int slap_stage_dwords(int rpw, int P) { return rpw * (4 + P); }

template <int RL>
struct SlapStage {
  static constexpr int RPW = 64 / RL;
  uint32_t* s;  // the wave's stage
  int P;
  __device__ __forceinline__ void issue(const SlapEpi& e, int64_t base, int nr) const {
    const int Pn = P;
    dma_dwords(2 * nr, s, [&](int k) { return reinterpret_cast<const uint32_t*>(e.i_in + base) + k; });
    if (e.to_choose)  // else the uniform product e.tc_stride: no strided 4-B reads
      dma_dwords(nr, s + 2 * RPW, [&](int k) { return e.to_choose + (base + k) * e.tc_stride; });
    if (e.ll_accum) dma_dwords(nr, s + 3 * RPW, [&](int k) { return e.ll_accum + base + k; });
    if (e.assign_in != e.assign_out)
      dma_dwords(nr * Pn, s + 4 * RPW, [&](int k) { return e.assign_in + base * Pn + k; });
  }
  __device__ __forceinline__ int64_t i_of(int g) const {
    return (int64_t)(((uint64_t)s[2 * g + 1] << 32) | s[2 * g]);
  }
  __device__ __forceinline__ float prod_of(int g) const { return __uint_as_float(s[2 * RPW + g]); }
  __device__ __forceinline__ float ll_of(int g) const { return __uint_as_float(s[3 * RPW + g]); }
  __device__ __forceinline__ int32_t asg_of(int g, int c) const {
    return (int32_t)s[4 * RPW + g * P + c];
  }

  // slap/env.py:50-62 for action a_raw of row r (group g); `sl == 0` writes the row
  // scalars.  Returns false when the product index is out of range (the reference's
  // advanced-index write raises).
  __device__ __forceinline__ bool store(const SlapEpi& e, int64_t r, int g, int sl,
                                        int64_t a_raw) const {
    // .to(torch.int), slap/env.py:52; to_choose NULL: every row's product is tc_stride
    int64_t p = e.to_choose ? (int64_t)(int)prod_of(g) : e.tc_stride;
    if (p < 0) p += e.P;
    const bool p_ok = p >= 0 && p < e.P;
    const int32_t av_new = (int32_t)a_raw;  // .to(torch.int), slap/env.py:53-54
    if (e.assign_in != e.assign_out) {      // the clone with [p] = action
      for (int c = sl; c < e.P; c += RL) e.assign_out[r * e.P + c] = c == p ? av_new : asg_of(g, c);
    } else if (sl == 0 && p_ok) {
      e.assign_out[r * e.P + p] = av_new;
    }
    if (sl == 0) {
      const int64_t it = i_of(g);
      e.done[r] = it == (int64_t)(e.P - 1);  // slap/env.py:57
      e.i_out[r] = it + 1;
      e.reward[r] = 0;
    }
    return p_ok;
  }
};

// Greedy (GreedyRow; certified / exact / fast per OPT) decode + SLAP step.
// STAGE (round 6): the wave's logits and mask rows (contiguous, 16-byte aligned) by
// non-temporal LDS-DMA after the env stage, read from LDS (tsp_decode_greedy_kernel's form)
template <int RL, int EPL, int VW, int OPT, bool STAGE = false>
__global__ __launch_bounds__(256) void slap_decode_greedy_kernel(
    int64_t B, int L, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, int32_t* status, SlapEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_stage[];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const size_t wstage = STAGE ? ((size_t)slap_stage_dwords(RPW, e.P) * 4 + 15) & ~(size_t)15
                              : (size_t)slap_stage_dwords(RPW, e.P) * 4;
  const size_t wbytes = wstage + (STAGE ? tsp_dstage_bytes(RPW, L) : 0);
  unsigned char* wbase_lds = reinterpret_cast<unsigned char*>(s_stage) + wave_in_block() * wbytes;
  const SlapStage<RL> st{reinterpret_cast<uint32_t*>(wbase_lds), e.P};
  // one row group per wave (the grid covers B: no loop, so nothing is hoisted into
  // registers across row groups)
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  {
    const int nr = (int)(B - base < RPW ? B - base : RPW);
    st.issue(e, base, nr);
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask_in + r * (int64_t)L;
    if constexpr (STAGE) {
      unsigned char* sw = wbase_lds + wstage;
      wave_dma<2>(reinterpret_cast<const unsigned char*>(logits + base * L), nr * L * 4, sw);
      wave_dma<2>(mask_in + base * L, nr * L, sw + (size_t)RPW * L * 4);
      wave_dma_wait();
      g.load(valid, L, reinterpret_cast<const float*>(sw) + grp * L,
             sw + (size_t)RPW * L * 4 + grp * L, c0);
    } else {
      g.load(valid, L, lrow, mrow, c0);
    }
    float lp, lse;
    const int sel = greedy_row<OPT>(g, valid, L, clip, temp, sl, c0,
                                    group_scratch<RL, EPL>(lds, grp), lse, lp, lrow, mrow);
    const bool feas0 = g.allowed(0);
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {  // the selected location leaves the mask
      const int off = sel - (c0 + 4 * j);
      if ((unsigned)off < 4u) g.mw[j] &= ~(0xffu << (8 * off));
    }
    stage_ready();
    if (valid) {
      g.store_mask(L, e.mask_out + r * (int64_t)L, c0);
      const bool p_ok = st.store(e, r, grp, sl, sel);
      if (sl == 0) {
        if (lse != lse && !feas0) set_status(status, CO_ST_INFEASIBLE);
        if (!p_ok) set_status(status, CO_ST_INDEX_RANGE);
        action_out[r] = sel;
        if (logp_sel) logp_sel[r] = lp;
        if (e.ll_accum) e.ll_accum[r] = st.ll_of(grp) + lp;
      }
    }
  }
}

// Sampling / evaluate (DecodeRow, exact math unless fast) decode + SLAP step.
template <int RL, int EPL, bool VEC, int OPT>
__global__ __launch_bounds__(256) void slap_decode_step_kernel(
    int64_t B, int L, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, int32_t* status, SlapEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_stage[];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const SlapStage<RL> st{s_stage + wave_in_block() * slap_stage_dwords(RPW, e.P), e.P};
  // one row group per wave (the grid covers B: no loop, so nothing is hoisted into
  // registers across row groups)
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  {
    const int nr = (int)(B - base < RPW ? B - base : RPW);
    st.issue(e, base, nr);
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    const int64_t a_in = (mode == CO_DECODE_EVALUATE && valid) ? action_in[r] : 0;
    DecodeRow<RL, EPL, VEC, OPT> d;
    d.run(valid, L, logits + r * lstride, mask_in + r * (int64_t)L, clip, temp, mode, a_in, seed,
          offset, row, sl, grp, group_scratch<RL, EPL>(lds, grp));
    const int64_t a_raw = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d.sel;
    const int64_t a = a_raw < 0 ? a_raw + L : a_raw;  // slap/env.py:62 (python indexing)
    const bool a_ok = a >= 0 && a < L;
#pragma unroll
    for (int k = 0; k < EPL; ++k)
      if (a_ok && c0 + k == a) d.mk[k] = 0;
    stage_ready();
    if (valid) {
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
      const bool p_ok = st.store(e, r, grp, sl, a_raw);
      if (sl == 0) {
        if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= L))
          set_status(status, CO_ST_INDEX_RANGE);  // the logp gather (decoding.py:365)
        if (mode != CO_DECODE_EVALUATE && !d.feas) set_status(status, CO_ST_INFEASIBLE);
        if (!a_ok || !p_ok) set_status(status, CO_ST_INDEX_RANGE);
        action_out[r] = a_raw;
        if (logp_sel) logp_sel[r] = d.lp;
        if (e.ll_accum) e.ll_accum[r] = st.ll_of(grp) + d.lp;
      }
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
  float* ll_accum;
};

// Per wave (RPW rows; the stage padded to 16 bytes, so a 16-byte aligned demand block
// comes in by dwordx4): [demand: RPW*N][visited bytes: RPW*(N+1) rounded up to dwords]
// [used: RPW][capacity: RPW][ll: RPW].  The visited rows of a wave are one contiguous,
// 4-byte-aligned byte range (the launcher requires RPW*(N+1) % 4 == 0 and an aligned
// buffer), fetched as whole dwords; the last partial wave's trailing bytes (< 4) by bytes.
__host__ __device__ inline int cvrp_vis_dwords(int rpw, int N) { return (rpw * (N + 1) + 3) / 4; }
__host__ __device__ inline int cvrp_stage_dwords(int rpw, int N) {  // 16-byte multiple
  return (rpw * N + cvrp_vis_dwords(rpw, N) + 3 * rpw + 3) & ~3;
}

template <int RL, int EPL>
struct CvrpStage {
  static constexpr int RPW = 64 / RL;
  uint32_t* s;
  int N;
  __device__ __forceinline__ uint32_t* dem() const { return s; }
  __device__ __forceinline__ uint32_t* vis() const { return s + RPW * N; }
  __device__ __forceinline__ uint32_t* sc() const { return s + RPW * N + cvrp_vis_dwords(RPW, N); }

  __device__ __forceinline__ void issue(const CvrpEpi& e, int64_t base, int nr) const {
    const int Nn = N, NC = N + 1;
    const float* dsrc = e.demand + base * Nn;
    const int nd = nr * Nn;
    if ((reinterpret_cast<uintptr_t>(dsrc) & 15) == 0) {  // wave-uniform
      const int n4 = nd >> 2;
      dma_dwordx4(n4, dem(), [&](int k) { return dsrc + 4 * k; });
      dma_dwords(nd & 3, dem() + 4 * n4, [&](int k) { return dsrc + 4 * n4 + k; });
    } else {
      dma_dwords(nd, dem(), [&](int k) { return dsrc + k; });
    }
    const uint8_t* vrow = e.vis_in + base * NC;
    const int nvb = nr * NC, nvw = nvb >> 2;
    dma_dwords(nvw, vis(), [&](int k) { return reinterpret_cast<const uint32_t*>(vrow) + k; });
    if (nvb & 3) {  // the buffer's last bytes (the last partial wave only): plain loads
      const int lane = lane_id();
      uint8_t* vb = reinterpret_cast<uint8_t*>(vis() + nvw);
      if (lane < (nvb & 3)) vb[lane] = vrow[4 * nvw + lane];
    }
    dma_dwords(nr, sc(), [&](int k) { return e.used_in + base + k; });
    dma_dwords(nr, sc() + RPW, [&](int k) { return e.vcap + base + k; });
    if (e.ll_accum) dma_dwords(nr, sc() + 2 * RPW, [&](int k) { return e.ll_accum + base + k; });
  }

  // cvrp/env.py:73-105 + get_action_mask (:137-149) for action a_raw of row r (group g),
  // the same arithmetic as co_cvrp_step, on the staged row.  Group-wide (every lane of the
  // wave active); writes the visited / mask rows and (sl == 0) the row scalars.
  __device__ __forceinline__ void apply(const CvrpEpi& e, bool valid, int64_t r, int g, int sl,
                                        int c0, int64_t a_raw, int32_t* status) const {
    const int Nn = N, NC = N + 1;
    const float* dm_s = reinterpret_cast<const float*>(dem()) + g * Nn;
    const float used = __uint_as_float(sc()[g]), cap = __uint_as_float(sc()[RPW + g]);
    const bool bad = a_raw < 0 || a_raw > Nn;
    // the selected demand demand[clamp(a - 1, 0, N - 1)]
    const int dsi = (int)(a_raw - 1 < 0 ? 0 : (a_raw - 1 > Nn - 1 ? Nn - 1 : a_raw - 1));
    const float u = (used + dm_s[dsi]) * ((a_raw != 0) ? 1.0f : 0.0f);
    const int a = bad ? -1 : (int)a_raw;
    uint32_t vw[EPL / 4], mk[EPL / 4];
    uint32_t cnt = 0u;
    bool feas = false;
    // every stage read first and unconditionally (index -1 / past the row: LDS words of the
    // stage or the static area, whose capacity bits `cust` drops; a per-slot select of them
    // had each demand read sunk into a branch of its own)
    float dr[EPL];
    uint32_t vlo[EPL / 4], vhi[EPL / 4];
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j, o = g * NC + c;
      const uint32_t* v32 = vis() + (o >> 2);
      vlo[j] = v32[0];
      vhi[j] = v32[1];
#pragma unroll
      for (int q = 0; q < 4; ++q) dr[4 * j + q] = dm_s[c + q - 1];
    }
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      const int nown = valid ? (NC - c < 0 ? 0 : (NC - c > 4 ? 4 : NC - c)) : 0;
      const uint32_t own = nown >= 4 ? 0xffffffffu : (1u << (8 * nown)) - 1u;
      const uint32_t cust = c == 0 ? own & ~0xffu : own;  // the depot column excluded
      // the chunk's visited bytes: the two stage dwords it straddles, byte-aligned by one
      // v_alignbyte (reads past the row stay inside the stage / LDS; `own` masks them)
      const int o = g * NC + c;
      uint32_t x = __builtin_amdgcn_alignbyte(vhi[j], vlo[j], (uint32_t)(o & 3)) & own;
      // the depot column's and past-the-row slots' values are whatever the stage holds:
      // their capacity bits are dropped by `cust` below, so no select
      const float* d = dr + 4 * j;
      const int ea = a - c;  // the action's byte, if in this chunk: scatter(..., 1)
      if (a >= 0 && ea >= 0 && ea < 4) x = (x & ~(0xffu << (8 * ea))) | (1u << (8 * ea));
      vw[j] = x;
      const uint32_t over = ((d[0] + u > cap) ? 0x80u : 0u) | ((d[1] + u > cap) ? 0x8000u : 0u) |
                            ((d[2] + u > cap) ? 0x800000u : 0u) |
                            ((d[3] + u > cap) ? 0x80000000u : 0u);
      const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
      const uint32_t m = ((~(nz | over) & 0x80808080u) >> 7) & cust;
      cnt = __builtin_amdgcn_sad_u8(x & own, 0u, cnt);
      feas |= m != 0u;
      mk[j] = m;
    }
    cnt = grp_reduce<RL>(cnt, [](uint32_t x, uint32_t y) { return x + y; });
    const uint64_t gm = RL == 64 ? ~0ull : ((1ull << RL) - 1ull);
    const bool anyf = ((__ballot(feas) >> (RL * g)) & gm) != 0ull;
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
  __device__ __forceinline__ float ll_of(int g) const { return __uint_as_float(sc()[2 * RPW + g]); }
};

template <int RL, int EPL, int VW, int OPT>
__global__ __launch_bounds__(256) void cvrp_decode_greedy_kernel(
    int64_t B, int NC, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, int32_t* status, CvrpEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_stage[];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const CvrpStage<RL, EPL> st{s_stage + wave_in_block() * cvrp_stage_dwords(RPW, e.N), e.N};
  // one row group per wave (the grid covers B: no loop, so nothing is hoisted into
  // registers across row groups)
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  {
    const int nr = (int)(B - base < RPW ? B - base : RPW);
    st.issue(e, base, nr);
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask_in + r * (int64_t)NC;
    g.load(valid, NC, lrow, mrow, c0);
    float lp = 0.f, lse = 0.f;
    int sel = (int)(row % NC);
    if (kDiagCvrpCut != 2)
      sel = greedy_row<OPT>(g, valid, NC, clip, temp, sl, c0, group_scratch<RL, EPL>(lds, grp),
                            lse, lp, lrow, mrow);
    else
      lp = g.v[0];  // keep the loads
    const bool feas0 = g.allowed(0);
    stage_ready();
    if (kDiagCvrpCut != 1) st.apply(e, valid, r, grp, sl, c0, sel, status);
    if (valid && sl == 0) {
      if (lse != lse && !feas0) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = sel;
      if (logp_sel) logp_sel[r] = lp;
      if (e.ll_accum) e.ll_accum[r] = st.ll_of(grp) + lp;
    }
  }
}

template <int RL, int EPL, bool VEC, int OPT>
__global__ __launch_bounds__(256) void cvrp_decode_step_kernel(
    int64_t B, int NC, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, int32_t* status, CvrpEpi e) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  extern __shared__ __attribute__((aligned(16))) uint32_t s_stage[];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const CvrpStage<RL, EPL> st{s_stage + wave_in_block() * cvrp_stage_dwords(RPW, e.N), e.N};
  // one row group per wave (the grid covers B: no loop, so nothing is hoisted into
  // registers across row groups)
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  {
    const int nr = (int)(B - base < RPW ? B - base : RPW);
    st.issue(e, base, nr);
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    const int64_t a_in = (mode == CO_DECODE_EVALUATE && valid) ? action_in[r] : 0;
    DecodeRow<RL, EPL, VEC, OPT> d;
    d.run(valid, NC, logits + r * lstride, mask_in + r * (int64_t)NC, clip, temp, mode, a_in,
          seed, offset, row, sl, grp, group_scratch<RL, EPL>(lds, grp));
    const int64_t a_raw = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d.sel;
    stage_ready();
    st.apply(e, valid, r, grp, sl, c0, a_raw, status);
    if (valid && sl == 0) {
      if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= NC))
        set_status(status, CO_ST_INDEX_RANGE);
      if (mode != CO_DECODE_EVALUATE && !d.feas) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = a_raw;
      if (logp_sel) logp_sel[r] = d.lp;
      if (e.ll_accum) e.ll_accum[r] = st.ll_of(grp) + d.lp;
    }
  }
}

}  // namespace

// lanes per row of the register row engines (decode_common.hpp's buckets)
inline int row_lanes(int64_t N) {
  return N <= 16 ? CO_RL16 : N <= 32 ? CO_RL32 : N <= 64 ? CO_RL64 : N <= 128 ? CO_RL128
       : N <= 256 ? CO_RL256 : 64;
}
inline int row_epl(int64_t N) {
  const int rl = row_lanes(N);
  const int b = N <= 16 ? 16 : N <= 32 ? 32 : N <= 64 ? 64 : N <= 128 ? 128 : N <= 256 ? 256
              : N <= 512 ? 512 : N <= 1024 ? 1024 : 2048;
  const int e = b / rl;
  return e < 4 ? 4 : e;
}
inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

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
  const int mword = mode;
  const bool cert = (mode & CO_DECODE_CERTIFIED) != 0 && (mode & CO_DECODE_FAST) == 0;
  const bool fast = (mode & CO_DECODE_FAST) != 0;
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (mode < 0 || mode > 2) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !mask_in || !action_out || !assign_in || !assign_out || !mask_out || !i_in ||
      !i_out || !done || !step_reward || (mode == CO_DECODE_EVALUATE && !action_in) ||
      (!to_choose && (tc_stride < 0 || tc_stride >= P)))
    return CO_E_INVAL;
  // mask_out may be mask_in: a row's mask is read (and re-read by the certified fallback)
  // by its own lane group before the transition stores it, after the wave's stage barrier
  const int64_t N = L;  // the row-dispatch macros' name for the row length
  const int rpw = 64 / row_lanes(N);
  const size_t shmem = (size_t)4 * slap_stage_dwords(rpw, (int)P) * 4;
  const size_t lds_static = (size_t)4 * 64 * row_epl(N) * 4;
  if (shmem + lds_static > 64 * 1024 || (to_choose && !aligned4(to_choose)) || !aligned4(assign_in) ||
      !aligned4(i_in) || (ll_accum && !aligned4(ll_accum))) {
    // beyond the stage (huge P) or misaligned: the two launches it fuses
    if (ll_accum) return CO_E_INVAL;
    int rc = co_decode_step(B, L, logits, lstride, mask_in, clip, temp, mword, action_in,
                            action_out, logp_sel, nullptr, seed, offset, status, stream);
    if (rc != CO_OK) return rc;
    return co_slap_step(B, L, P, mode == CO_DECODE_EVALUATE ? action_in : action_out, to_choose,
                        tc_stride, assign_in, assign_out, mask_in, mask_out, i_in, i_out, done,
                        step_reward, status, stream);
  }
  const SlapEpi epi{(int)P, to_choose, tc_stride, assign_in, assign_out, mask_out,
                    i_in,   i_out,     done,      step_reward, ll_accum};
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(cover_grid(B, rpw * 4)), block(256);
  if (grid.x == 0) return CO_E_INVAL;
  if (mode == CO_DECODE_GREEDY && CO_DECODE_STAGE && N > 64 && N <= 128 && N % 4 == 0 &&
      lstride == N && greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr) == 4 &&
      ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(mask_in)) & 15) == 0) {
    // the logits and mask rows by non-temporal LDS-DMA (slap_decode_greedy_kernel STAGE)
    const size_t wst = (((size_t)slap_stage_dwords(rpw, (int)P) * 4 + 15) & ~(size_t)15) +
                       tsp_dstage_bytes(rpw, (int)N);
    if (4 * wst + lds_static <= 64 * 1024) {
      CO_OPT_DISPATCH_G(hipLaunchKernelGGL,
                        (slap_decode_greedy_kernel<CO_RL128, 128 / CO_RL128, 4, OPT, true>), grid,
                        block, 4 * wst, s, B, (int)N, logits, lstride, mask_in, clip, temp,
                        action_out, logp_sel, status, epi);
      return launch_status();
    }
  }
  if (mode == CO_DECODE_GREEDY) {
#define CO_SDG(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL,                                                        \
                    (slap_decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), grid, block, \
                    shmem, s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out,     \
                    logp_sel, status, epi)
    switch (greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr)) {
      case 4: CO_ROW_DISPATCH(CO_SDG, 4); break;
      case 2: CO_SDG(CO_RL16, 16 / CO_RL16, 2); break;  // N < 4
      default: CO_ROW_DISPATCH(CO_SDG, 3);
    }
#undef CO_SDG
    return launch_status();
  }
#define CO_SDS(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (slap_decode_step_kernel<RL, EPL, V, OPT>), grid, block, \
                  shmem, s, B, (int)N, logits, lstride, mask_in, clip, temp, mode, action_in,   \
                  action_out, logp_sel, seed, offset, status, epi)
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
  const int mword = mode;
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
  const int64_t N = Ncust + 1;  // row length (depot + customers)
  const int rpw = 64 / row_lanes(N);
  const size_t shmem = (size_t)4 * cvrp_stage_dwords(rpw, (int)Ncust) * 4;
  const size_t lds_static = (size_t)4 * 64 * row_epl(N) * 4;
  if (shmem + lds_static > 64 * 1024 || (rpw * N) % 4 != 0 || !aligned4(vis_in) ||
      !aligned4(demand) || !aligned4(used_in) || !aligned4(vcap) ||
      (ll_accum && !aligned4(ll_accum))) {
    // beyond the stage or misaligned rows: the two launches it fuses
    if (ll_accum) return CO_E_INVAL;
    int rc = co_decode_step(B, N, logits, lstride, mask_in, clip, temp, mword, action_in,
                            action_out, logp_sel, nullptr, seed, offset, status, stream);
    if (rc != CO_OK) return rc;
    return co_cvrp_step(B, Ncust, mode == CO_DECODE_EVALUATE ? action_in : action_out, demand,
                        used_in, used_out, vcap, vis_in, vis_out, cur_out, done, step_reward,
                        mask_out, status, nullptr, stream);
  }
  const CvrpEpi epi{(int)Ncust, demand,  used_in, used_out,    vcap,     vis_in,
                    vis_out,    cur_out, done,    step_reward, mask_out, ll_accum};
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(cover_grid(B, rpw * 4)), block(256);
  if (grid.x == 0) return CO_E_INVAL;
  if (mode == CO_DECODE_GREEDY) {
#define CO_CDG(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL,                                                        \
                    (cvrp_decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), grid, block, \
                    shmem, s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out,     \
                    logp_sel, status, epi)
    switch (greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr)) {
      case 4: CO_ROW_DISPATCH(CO_CDG, 4); break;
      case 2: CO_CDG(CO_RL16, 16 / CO_RL16, 2); break;  // N < 4
      default: CO_ROW_DISPATCH(CO_CDG, 3);
    }
#undef CO_CDG
    return launch_status();
  }
#define CO_CDS(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (cvrp_decode_step_kernel<RL, EPL, V, OPT>), grid, block, \
                  shmem, s, B, (int)N, logits, lstride, mask_in, clip, temp, mode, action_in,   \
                  action_out, logp_sel, seed, offset, status, epi)
  if (decode_vec_ok(logits, lstride, mask_in, N)) {
    CO_ROW_DISPATCH(CO_CDS, true);
  } else {
    CO_ROW_DISPATCH(CO_CDS, false);
  }
#undef CO_CDS
  (void)cert;
  return launch_status();
}
