// Fused decode step for gfx950 (rl4co/utils/decoding.py:141-191,327-399,489-499):
// tanh clip -> mask to -inf -> /temperature -> log_softmax -> greedy argmax |
// Philox inverse-CDF sample | evaluate -> logp gather, in one pass.
//
// RL = 16/32/64 lanes per row (several rows per wave, grid-stride); the row's logits
// stay in registers (EPL per lane), max / sum / argmax are xor-shuffle reductions
// inside the lane group and the sampling CDF is a group inclusive scan.  log_softmax is evaluated with the
// same association as ATen's CPU kernel: logp = (x - max) - log(sum(exp(x - max))),
// so greedy ties resolve exactly like torch.argmax (first index).
#pragma once
// Shared by decode_step.hip (co_decode_step[_ex], beam search) and decode_tsp.hip
// (co_tsp_decode_step): two translation units, compiled in parallel.
#include <type_traits>

#include "co_common.hpp"
#include "co_diag.hpp"
#include "co_math.hpp"

using namespace co;

// decode tuning (tools/build_variants.sh sweeps them): lanes per row for each row-length
// bucket N <= 16, 32, 64, 128, 256 (EPL = bucket / lanes); longer rows use 64 lanes
#ifndef CO_RL16
#define CO_RL16 4
#endif
#ifndef CO_RL32
#define CO_RL32 4
#endif
#ifndef CO_RL64
#define CO_RL64 8
#endif
#ifndef CO_RL128
#define CO_RL128 16
#endif
#ifndef CO_RL256
#define CO_RL256 32
#endif
#ifndef CO_DECODE_UNR
#define CO_DECODE_UNR 1
#endif

__device__ __forceinline__ float co_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
// CO_DECODE_FAST (opt-in, mode flag): tanh(x) = 1 - 2 / (e^{2x} + 1) on v_exp / v_rcp (abs
// error ~1e-7, exact +-1 saturation), the softmax exps on v_exp_f32 (<= 2 ulp) summed in
// lane order -- log-probabilities within ~1e-6 of the reference, greedy picks exact only
// where the top two are further apart than that
__device__ __forceinline__ float co_tanh_fast(float x) {
  const float e = co_exp2(x * 2.8853900817779268f);  // e^{2x}
  return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}
__device__ __forceinline__ float co_exp_fast(float x) { return co_exp2(x * 1.4426950408889634f); }

// OPT template flags of the row engines: bit 0 tanh clipping, bit 1 temperature != 1,
// bit 2 the fast math above (default: ATen-exact, co_math.hpp), bit 3 certified greedy
// (GreedyRow kernels only, CO_DECODE_CERTIFIED: fast math, then the exact recomputation
// for every wave holding a row whose fast argmax the error bound cannot certify)
constexpr int kOptClip = 1, kOptTemp = 2, kOptFast = 4, kOptCert = 8;
// kOptLean (internal: the certified path's fast pass in GreedyRow): the padded slots hold
// -inf already (no per-slot row-bound select in the exp sum), the log on v_log_f32, the
// group max on ordered ints, the lane's top two kept for the certification
constexpr int kOptLean = 16;
#ifndef CO_TANH_COMPACT
#define CO_TANH_COMPACT 1  // GreedyRow: exact tanh of allowed elements only, wave-compacted
#endif
#ifndef CO_TANH_CHAINS
#define CO_TANH_CHAINS 2  // packed tanh evaluations per lane and loop iteration (1 or 2)
#endif

template <int OPT>
__device__ __forceinline__ float clip_tanh(float x) {
  return ((OPT & kOptFast) || kDiagFastTanh) ? co_tanh_fast(x) : tanh_cr(x);
}

// exp-sum of a row (x already shifted by the row max; out-of-row slots excluded) and its
// log: ATen's order and SLEEF math (exact) or v_exp + lane-order butterfly (fast)
template <int RL, int EPL, int OPT>
__device__ __forceinline__ float row_log_sum_exp(const float (&d)[EPL], int N, int sl,
                                                 float* lds_row) {
  const int c0 = sl * EPL;
  float e[EPL];
  if ((OPT & kOptFast) || kDiagFastExp) {
    float s = 0.f;
    if constexpr ((OPT & kOptLean) != 0) {
      // every slot past N is -inf (masked) here: e^-inf = 0 needs no row-bound select;
      // the sum is >= 1 (the maximum's term), so v_log_f32 needs no denormal scaling
      const f32x2 l2 = {1.4426950408889634f, 1.4426950408889634f};
#pragma unroll
      for (int k = 0; k < EPL; k += 2) {  // the exponents' products packed, the sum in order
        const f32x2 a = f32x2{d[k], d[k + 1]} * l2;
        s += co_exp2(a.x);
        s += co_exp2(a.y);
      }
      return __builtin_amdgcn_logf(grp_sum<RL>(s)) * 0.69314718055994531f;
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) s += c0 + k < N ? co_exp_fast(d[k]) : 0.f;
    return logf(grp_sum<RL>(s));
  }
#pragma unroll
  for (int k = 0; k < EPL; ++k) e[k] = c0 + k < N ? aten_expf(d[k]) : 0.f;
  return aten_logf(aten_row_sum<RL, EPL>(e, N, sl, lds_row));
}

// LDS scratch of the exact sums: one RL*EPL-float row per lane group = 64*EPL floats per
// wave; kernels of 256 threads (4 waves) declare it as `__shared__ float[4 * 64 * EPL]`
// (unused, and dropped by the compiler, on the fast path)
template <int RL, int EPL>
__device__ __forceinline__ float* group_scratch(float* lds, int grp) {
  return lds + wave_in_block() * (64 * EPL) + grp * (RL * EPL);
}

// Exact tanh (tanh_cr) of the elements a lane marks `ok`, wave-compacted: a masked
// element's clipped logit becomes -inf whatever its tanh, so only the allowed ones are
// evaluated.  Each element slot's ballot + mbcnt packs the wave's allowed values into
// `wave_lds` (64 * EPL floats), every lane takes every 64th packed entry, and the results go
// back to their slots: the same bits per element, ceil(allowed / 64) f64 evaluations per
// lane instead of EPL (about half over a TSP episode: N - t actions allowed at step t).
// All lanes of the wave must be active.
template <int EPL>
__device__ __forceinline__ void wave_tanh_compact(float (&v)[EPL], const bool (&ok)[EPL],
                                                  float* wave_lds) {
  const int lane = lane_id();
  int pos[EPL], total = 0;
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const uint64_t bal = __ballot(ok[k]);
    pos[k] = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (ok[k]) wave_lds[pos[k]] = v[k];
    total += __popcll(bal);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if CO_TANH_CHAINS == 2
  for (int j = lane; j < total; j += 128) {  // two independent f64 chains per lane
    const bool two = j + 64 < total;
    const float x0 = wave_lds[j], x1 = two ? wave_lds[j + 64] : 0.f;
    const float y0 = tanh_cr(x0), y1 = tanh_cr(x1);
    wave_lds[j] = y0;
    if (two) wave_lds[j + 64] = y1;
  }
#else
  for (int j = lane; j < total; j += 64) wave_lds[j] = tanh_cr(wave_lds[j]);
#endif
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < EPL; ++k)
    if (ok[k]) v[k] = wave_lds[pos[k]];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // the reads above stay before the scratch's next writes
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

namespace {

// Philox-4x32-10 (Salmon et al. 2011), counter = (offset_lo, offset_hi, row_lo, row_hi).
__device__ __forceinline__ uint32_t philox_u32(uint64_t seed, uint64_t offset, uint64_t row) {
  uint32_t c0 = (uint32_t)offset, c1 = (uint32_t)(offset >> 32), c2 = (uint32_t)row,
           c3 = (uint32_t)(row >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c0;
}

// ---------------------------------------------------------------------------
// Row engine: RL lanes per row (4 ... 64), 64/RL rows per wave, EPL consecutive
// elements per lane; reductions are the DPP / permlane-swap group butterflies of
// co_common.hpp.  Every lane of a wave runs the same number of row iterations (rows
// past B run on dummy data and are not stored), so no stage reads an inactive lane.
//
// Lane `sl` of the group owns the EPL consecutive elements c = sl*EPL + k.  VEC: the
// row's logits are read as float4 and its mask bytes as u32 (needs N % 4 == 0 and a
// 16-byte aligned logits row stride); otherwise scalar loads.
template <int RL, int EPL, bool VEC, int OPT>
struct DecodeRow {  // OPT: clip / temperature flags as in GreedyRow::softmax_shift
  float x[EPL];     // log-probabilities after `run`
  uint8_t mk[EPL];  // the row's action_mask bytes (1 when no mask)
  int sel;          // selected action (valid on every lane of the group)
  float lp;         // its log-probability
  bool feas;        // mask[sel]

  __device__ __forceinline__ void load(bool valid, int N, const float* lrow, const uint8_t* mrow,
                                       int sl) {
    const int c0 = sl * EPL;
    if (VEC) {
#pragma unroll
      for (int j = 0; j < EPL / 4; ++j) {
        const int c = c0 + 4 * j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t mm = 0;
        if (valid && c < N) {
          v = *reinterpret_cast<const float4*>(lrow + c);
          mm = mrow ? *reinterpret_cast<const uint32_t*>(mrow + c) : 0x01010101u;
        }
        x[4 * j] = v.x;
        x[4 * j + 1] = v.y;
        x[4 * j + 2] = v.z;
        x[4 * j + 3] = v.w;
#pragma unroll
        for (int q = 0; q < 4; ++q) mk[4 * j + q] = (uint8_t)(mm >> (8 * q));
      }
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        const int c = c0 + k;
        const bool in = valid && c < N;
        x[k] = in ? lrow[c] : 0.f;
        mk[k] = in ? (mrow ? mrow[c] : 1) : 0;
      }
    }
  }

  // tanh clip -> mask -> /T -> log_softmax -> select (decoding.py:141-191,371-399,489-499)
  __device__ __forceinline__ void run(bool valid, int N, const float* lrow, const uint8_t* mrow,
                                      float clip, float temp, int mode, int64_t a_in,
                                      uint64_t seed, uint64_t offset, int64_t row, int sl,
                                      int grp, float* lds_row, int top_k = 0,
                                      double top_p = 0.0) {
    load(valid, N, lrow, mrow, sl);
    compute(valid, N, clip, temp, mode, a_in, seed, offset, row, sl, grp, lds_row, top_k, top_p);
  }

  // decoding.py:112-117 modify_logits_for_top_k_filtering on x (the processed logits):
  // threshold = the k-th largest value counted with multiplicity (torch.topk), values
  // strictly below it -> -inf.  Distinct levels are peeled from the top with a group max
  // and a group count; a row with fewer than k finite values keeps everything.
  __device__ __forceinline__ void filter_top_k(int N, int top_k, int sl) {
    const float NEG_INF = -__builtin_inff();
    const int c0 = sl * EPL;
    float hi = __builtin_inff(), thr = NEG_INF;
    int remaining = top_k;
    for (int it = 0; it < top_k; ++it) {
      float lm = NEG_INF;
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (c0 + k < N && x[k] < hi) lm = fmaxf(lm, x[k]);
      lm = grp_max<RL>(lm);
      if (lm == NEG_INF) break;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < EPL; ++k) cnt += (c0 + k < N) && (x[k] == lm);
      cnt = (int)grp_reduce<RL>((uint32_t)cnt, [](uint32_t a, uint32_t b) { return a + b; });
      if (cnt >= remaining) {
        thr = lm;
        break;
      }
      remaining -= cnt;
      hi = lm;
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = x[k] < thr ? NEG_INF : x[k];
  }

  // decoding.py:120-138 modify_logits_for_top_p_filtering: with p = softmax(x) and the
  // ascending order (ties by index), drop every element whose cumulative probability up
  // to and including itself is <= 1 - top_p.  Each lane accumulates, for its elements,
  // the probabilities of the row's elements that precede them (group broadcasts of the
  // row); the summation order differs from ATen's sorted cumsum, so an element whose
  // cumulative sum lies within rounding of the threshold can be decided differently.
  __device__ __forceinline__ void filter_top_p(bool valid, int N, double top_p, float m, int sl,
                                               int grp) {
    const float NEG_INF = -__builtin_inff();
    const int c0 = sl * EPL;
    float pr[EPL], s = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      pr[k] = (valid && c0 + k < N) ? expf(x[k] - m) : 0.f;
      s += pr[k];
    }
    s = grp_sum<RL>(s);
#pragma unroll
    for (int k = 0; k < EPL; ++k) pr[k] = pr[k] / s;
    float cum[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) cum[k] = 0.f;
    for (int j = 0; j < N; ++j) {
      const int owner = grp * RL + j / EPL, slot = j % EPL;
      float xs = 0.f, ps = 0.f;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        xs = k == slot ? x[k] : xs;
        ps = k == slot ? pr[k] : ps;
      }
      const float vj = __shfl(xs, owner, 64), pj = __shfl(ps, owner, 64);
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        const bool before = vj < x[k] || (vj == x[k] && j <= c0 + k);
        cum[k] += before ? pj : 0.f;
      }
    }
    const float keep_above = (float)(1.0 - top_p);
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = cum[k] <= keep_above ? NEG_INF : x[k];
  }

  // the math on data already `load`ed (callers overlap several rows' loads)
  __device__ __forceinline__ void compute(bool valid, int N, float clip, float temp, int mode,
                                          int64_t a_in, uint64_t seed, uint64_t offset,
                                          int64_t row, int sl, int grp, float* lds_row,
                                          int top_k = 0, double top_p = 0.0) {
    const float NEG_INF = -__builtin_inff();
    const int c0 = sl * EPL;
    // (the wave-compacted tanh of GreedyRow measured no faster here: sampling with clip
    // 10 at B=102,400, 70 % allowed, 46.4 vs 45.3 us -- the per-slot tanh stays)
    float m = NEG_INF;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      float v = NEG_INF;
      if (valid && c0 + k < N) {
        v = x[k];
        if (OPT & kOptClip) v = clip_tanh<OPT>(v) * clip;
        if (!mk[k]) v = NEG_INF;
        if (OPT & kOptTemp) v = v / temp;  // x / 1 == x exactly: skip the IEEE divide
        m = fmaxf(m, v);
      }
      x[k] = v;
    }
    m = grp_max<RL>(m);
    if (top_k > 0 && top_k < N) filter_top_k(N, top_k, sl);
    if (top_p > 0.0 && top_p < 1.0) filter_top_p(valid, N, top_p, m, sl, grp);
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = x[k] - m;
    const float L = row_log_sum_exp<RL, EPL, OPT>(x, N, sl, lds_row);
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = x[k] - L;  // ATen association: (x - m) - L
    sel = 0;
    if (mode == CO_DECODE_GREEDY) {
      float bv = NEG_INF;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        const int c = c0 + k;
        if (c < N && argmax_better(x[k], c, bv, bi)) { bv = x[k]; bi = c; }
      }
      grp_argmax<RL>(bv, bi);
      sel = bi == 0x7fffffff ? 0 : bi;
    } else if (mode == CO_DECODE_SAMPLING) {
      // inverse CDF: lane partial sums, group exclusive scan, then the lane's own walk;
      // the first element whose running sum passes u*total (and p > 0) is sampled
      const uint32_t r = philox_u32(seed, offset, (uint64_t)row);
      const float u = (float)(r >> 8) * (1.0f / 16777216.0f);
      float p[EPL], own = 0.f;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        p[k] = (valid && c0 + k < N) ? expf(x[k]) : 0.f;
        own += p[k];
      }
      float incl = own;
#pragma unroll
      for (int d = 1; d < RL; d <<= 1) {
        const float t = __shfl_up(incl, d, RL);
        if (sl >= d) incl += t;
      }
      const float total = __shfl(incl, grp * RL + RL - 1, 64);
      const float target = u * total;
      float run = incl - own;
      int hit = 0x7fffffff, last = -1;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        run += p[k];
        if (p[k] > 0.f) {
          last = c0 + k;
          if (run > target && hit == 0x7fffffff) hit = c0 + k;
        }
      }
      hit = grp_min_int<RL>(hit);
      last = grp_max_int<RL>(last);
      sel = hit != 0x7fffffff ? hit : (last >= 0 ? last : 0);
    } else {
      sel = (a_in < 0 || a_in >= N) ? 0 : (int)a_in;
    }
    const int owner = grp * RL + sel / EPL, slot = sel % EPL;
    float mine = 0.f;
    int f = 0;
#pragma unroll
    for (int k = 0; k < EPL; ++k)
      if (k == slot) {
        mine = x[k];
        f = mk[k];
      }
    lp = __shfl(mine, owner, 64);
    feas = __shfl(f, owner, 64) != 0;
  }
};

// ---------------------------------------------------------------------------
// Greedy row engine (decoding.py:327-335: argmax of log_softmax, first index on ties).
// The max log-probability of a row is exactly fl(0 - L) (L = log of the exp-sum, the
// max element has x - m = 0) and every logp = fl((x - m) - L) is monotone in x, so the
// greedy action is the first index whose logp equals fl(0 - L): one subtract + compare
// per element and an integer group min, instead of a (value, index) argmax butterfly, and
// the selected log-probability needs no broadcast.  Same association and exp sums as
// DecodeRow, so actions and logp are the bits DecodeRow produces.  A row whose L is not
// finite (every action masked, a NaN / +inf logit) has NaN log-probabilities throughout:
// index 0 (torch.argmax picks the first NaN), logp NaN.  The mask is kept as 4-byte
// words (pad slots past N read as masked).  VW = 4: float4 + u32 mask loads on 16-byte /
// 4-byte aligned rows (N % 4 == 0); VW = 3: the same 4-element chunks on rows of any N
// (logits rows 4-byte aligned, mask rows byte aligned: gfx950 takes dword-aligned
// dwordx4 and byte-aligned dword global accesses), the row's last partial chunk element
// by element.
template <int VW>
struct Chunk;
template <>
struct Chunk<4> {
  using F = float4;
  using M = uint32_t;
};
typedef float f4_align4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32_align1 __attribute__((aligned(1)));
template <>
struct Chunk<3> {
  using F = f4_align4;
  using M = u32_align1;
};
template <>
struct Chunk<2> : Chunk<3> {};

// v_cndmask_b32 on a per-lane condition, kept a select: LLVM turned the load's select
// chains into divergent branches, whose joins then wait for every load in flight
__device__ __forceinline__ float lane_select(bool c, float t, float f) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3"
      : "=v"(r)
      : "v"(f), "v"(t), "s"(__builtin_amdgcn_ballot_w64(c)));
  return r;
}

#ifndef CO_DECODE_NT
#define CO_DECODE_NT 0  // logits chunks by non-temporal loads (r06: POMO 1.80 -> 1.83 ms, CVRP
                        // decode step 10.1 -> 10.6 us: kept off)
#endif
template <class F>
__device__ __forceinline__ F ld_logit4(const F* p) {
  if constexpr (CO_DECODE_NT && std::is_same<F, float4>::value) {
    return ld_s<true>(p);
  } else if constexpr (CO_DECODE_NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

template <int RL, int EPL, int VW>
struct GreedyRow {
  static_assert(EPL % 4 == 0, "GreedyRow keeps the mask in u32 words");
  float v[EPL];
  uint32_t mw[EPL / 4];
  float top1 = 0.f, top2 = 0.f;  // kOptLean: the lane's largest two shifted values

  __device__ __forceinline__ void load(bool valid, int N, const float* lrow, const uint8_t* mrow,
                                       int c0) {
    using F = typename Chunk<VW>::F;
    using M = typename Chunk<VW>::M;
    if constexpr (VW == 3) {
      load_clamped(valid, N, lrow, mrow, c0);
      return;
    }
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      uint32_t m = 0u;
      float xf[4] = {0.f, 0.f, 0.f, 0.f};
      if (valid && c + 4 <= N) {
        const F x = ld_logit4(reinterpret_cast<const F*>(lrow + c));
        xf[0] = x[0];
        xf[1] = x[1];
        xf[2] = x[2];
        xf[3] = x[3];
        m = mrow ? (uint32_t) * reinterpret_cast<const M*>(mrow + c) : 0x01010101u;
      } else if (VW == 2 && valid && c < N) {  // the row's partial last chunk
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (c + q < N) {
            xf[q] = lrow[c + q];
            m |= (mrow ? (uint32_t)mrow[c + q] : 1u) << (8 * q);
          }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[4 * j + q] = xf[q];
      mw[j] = m;
    }
  }
  // VW = 3 (rows of any alignment, N >= 4; VW = 2: N < 4, element by element): every chunk
  // by one 16-byte and one 4-byte access, no branch.  A chunk's start is clamped to the
  // row's last four columns (cb = min(c, N - 4)): the row's partial last chunk reads columns
  // N - 4 .. N - 1 and shifts them down by S = 4 - N % 4 (its slots past the row are
  // masked); a chunk past the row reads the row's tail again and is masked whole.  r05: the
  // element-wise tail of the branchy form made the compiler wait for each chunk's load
  // before issuing the next (CVRP-100 rows, N + 1 = 101 columns).
  __device__ __forceinline__ void load_clamped(bool valid, int N, const float* lrow,
                                               const uint8_t* mrow, int c0) {
    using F = typename Chunk<3>::F;
    using M = typename Chunk<3>::M;
    const int S = (4 - (N & 3)) & 3;
    F x[EPL / 4];
    uint32_t w[EPL / 4];
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {  // every load issued before the first use
      const int c = c0 + 4 * j;
      const int cb = c < N - 4 ? c : N - 4;
      x[j] = ld_logit4(reinterpret_cast<const F*>(lrow + cb));
      w[j] = mrow ? (uint32_t) * reinterpret_cast<const M*>(mrow + cb) : 0x01010101u;
    }
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      const int s = c - (c < N - 4 ? c : N - 4);  // 0: whole chunk, S: partial, >= 4: past
      const int p = s != 0 ? S : 0;               // the slots' shift
      v[4 * j + 0] = lane_select(p == 0, x[j][0],
                                 lane_select(p == 1, x[j][1], lane_select(p == 2, x[j][2], x[j][3])));
      v[4 * j + 1] = lane_select(p == 0, x[j][1], lane_select(p == 1, x[j][2], x[j][3]));
      v[4 * j + 2] = lane_select(p == 0, x[j][2], x[j][3]);
      v[4 * j + 3] = x[j][3];
      mw[j] = (valid && s < 4) ? w[j] >> ((8 * s) & 31) : 0u;
    }
  }

  // the row's mask words / logp values back to memory (pad chunks skipped)
  __device__ __forceinline__ void store_mask(int N, uint8_t* orow, int c0) const {
    using M = typename Chunk<VW>::M;
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      if (c + 4 <= N) {
        *reinterpret_cast<M*>(orow + c) = (M)mw[j];
      } else if (VW != 4 && c < N) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (c + q < N) orow[c + q] = (uint8_t)(mw[j] >> (8 * q));
      }
    }
  }
  __device__ __forceinline__ void store_logp(int N, float L, float* frow, int c0) const {
    using F = typename Chunk<VW>::F;
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int c = c0 + 4 * j;
      if (c + 4 <= N) {
        F x;
        x[0] = v[4 * j] - L;
        x[1] = v[4 * j + 1] - L;
        x[2] = v[4 * j + 2] - L;
        x[3] = v[4 * j + 3] - L;
        *reinterpret_cast<F*>(frow + c) = x;
      } else if (VW != 4 && c < N) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (c + q < N) frow[c + q] = v[4 * j + q] - L;
      }
    }
  }

  __device__ __forceinline__ bool allowed(int k) const {
    return ((mw[k >> 2] >> (8 * (k & 3))) & 0xffu) != 0u;
  }

  // leaves v[k] = x_k - m; returns L (NaN for the degenerate rows above)
  // OPT bit 0: tanh clipping, bit 1: temperature != 1 (template flags: as runtime
  // conditions the compiler evaluates both arms per element and selects)
  // exact tanh of the allowed elements only, wave-compacted (wave_tanh_compact)
  __device__ __forceinline__ void tanh_allowed_compact(float* wave_lds) {
    bool ok[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) ok[k] = allowed(k);
    wave_tanh_compact<EPL>(v, ok, wave_lds);
  }

  // the processed logit z of a raw logit x (softmax_shift's arithmetic, in its order):
  // clip * tanh(x), then / temp; z_scale: the same from an already computed tanh
  template <int OPT>
  static __device__ __forceinline__ float z_scale(float t, float clip, float temp) {
    if (OPT & kOptClip) t = t * clip;
    if (OPT & kOptTemp) t = t / temp;
    return t;
  }
  template <int OPT>
  static __device__ __forceinline__ float z_of(float x, float clip, float temp) {
    if constexpr ((OPT & kOptLean) != 0 && (OPT & kOptClip) != 0 && (OPT & kOptTemp) == 0) {
      // the certified fast pass: clip * tanh(x) = clip - 2 clip / (e^{2x} + 1), one fma for
      // co_tanh_fast's fma and the clip product.  |z' - clip tanh x| <= clip (2.2e-7 + 2^-25)
      // + ulp(z') / 2: inside delta_z's clip * 1.5e-6 + 3 ulp(clip) (-2 clip is exact; an
      // overflowing clip gives NaN, which the certification rejects)
      const float e = co_exp2(x * 2.8853900817779268f);
      return __builtin_fmaf(-2.f * clip, __builtin_amdgcn_rcpf(e + 1.f), clip);
    }
    return z_scale<OPT>((OPT & kOptClip) ? clip_tanh<OPT>(x) : x, clip, temp);
  }

  // COMPACT = false: the certified path's rare exact fallback (the compaction there made
  // the whole certified kernel slower: 2.09 -> 2.37 ms per POMO episode)
  template <int OPT, bool COMPACT = true>
  __device__ __forceinline__ float softmax_shift(float clip, float temp, int N, int sl,
                                                 float* lds_row) {
    const float NEG_INF = -__builtin_inff();
    // exact tanh clipping: tanh of the allowed elements, wave-compacted (above)
    constexpr bool kCompact = COMPACT && (OPT & kOptClip) && !(OPT & kOptFast) && CO_TANH_COMPACT;
    if constexpr (kCompact) tanh_allowed_compact(lds_row - (lane_id() / RL) * (RL * EPL));
    float m = NEG_INF, m2 = NEG_INF;
    constexpr bool kPairs = (OPT & kOptLean) != 0 && (OPT & kOptClip) != 0 && (OPT & kOptTemp) == 0;
    if constexpr (kPairs) {
      // z_of<Lean> two slots at a time on packed f32 (v_pk_mul / v_pk_add / v_pk_fma: the
      // same IEEE results as the scalar ops, at about half the issue cost per slot)
      const f32x2 k2 = {2.8853900817779268f, 2.8853900817779268f};
      const f32x2 one = {1.f, 1.f}, c2 = {clip, clip}, n2c = {-2.f * clip, -2.f * clip};
#pragma unroll
      for (int k = 0; k < EPL; k += 2) {
        const f32x2 a = f32x2{v[k], v[k + 1]} * k2;
        const f32x2 e = f32x2{co_exp2(a.x), co_exp2(a.y)} + one;
        const f32x2 z = __builtin_elementwise_fma(
            f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)}, n2c, c2);
        v[k] = z.x;
        v[k + 1] = z.y;
      }
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      float t = kPairs ? v[k] : kCompact ? z_scale<OPT>(v[k], clip, temp) : z_of<OPT>(v[k], clip, temp);
      t = allowed(k) ? t : NEG_INF;
      v[k] = t;
      if constexpr ((OPT & kOptLean) != 0) {
        m2 = __builtin_amdgcn_fmed3f(m, m2, t);  // the lane's second largest (m2 <= m)
        m = __builtin_fmaxf(m, t);
      } else {
        m = fmaxf(m, t);
      }
    }
    if constexpr ((OPT & kOptLean) != 0) {
      // NaN anywhere makes L NaN below whichever member the max returns
      const float lm = m;
      m = grp_max_ord<RL>(m);
      top1 = lm - m;
      top2 = m2 - m;
    } else {
      m = grp_max<RL>(m);
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) v[k] = v[k] - m;
    return row_log_sum_exp<RL, EPL, OPT>(v, N, sl, lds_row);
  }

  // CO_DECODE_CERTIFIED: after softmax_shift with the fast math (v[k] = z'_k - m', L' the
  // fast log-sum-exp) and select (sel), is `sel` provably the exact path's greedy action
  // (as far as this lane's elements go)?
  // The exact action is the first index of max fl(fl(z_k - m) - L) (z: the clipped /
  // masked / scaled logits the exact path computes).  Certified when the fast runner-up
  // trails the selected value by more than
  //   2 eps_z / T            (|z'_k - z_k| <= eps_z: fast tanh abs error <= 1.5e-6 --
  //                          measured max over every f32 in [-9.1, 9.1]: 2.2e-7,
  //                          tools/diag/tanh_fast_err.hip -- times the clip, plus the
  //                          roundings of the product; 0 without clip)
  //   + 2 ulp bound of L     (then fl(d_k - L) < fl(0 - L) for every k != sel: no rounding
  //                          tie with the maximum)
  // and L' is finite.  Non-finite rows (all masked, NaN / inf logits) are never certified.
  // Evaluated per lane over the lane's own elements (no group reduction: the caller
  // only needs whether any lane of the wave failed, one ballot): the lane is certified
  // when each of its elements other than sel trails by more than delta (masked entries
  // are -inf; a NaN fails the comparison).
  // the L part of the bound: 2 x (2 ulp) of |L| + 1, margin included
  static __device__ __forceinline__ float delta_l(float L) {
    int e;
    frexpf(fabsf(L) + 1.f, &e);  // |L| + 1 < 2^e: ulp(L) <= 2^(e - 24)
    return ldexpf(1.f, e - 22) + 1e-7f;
  }
  template <int OPT>
  static __device__ __forceinline__ float delta_z(float clip, float temp) {
    if (!(OPT & kOptClip)) return 0.f;
    int ec;
    frexpf(clip, &ec);
    const float ez = clip * 1.5e-6f + ldexpf(3.f, ec - 24);
    return 2.f * ((OPT & kOptTemp) ? ez / temp : ez);
  }
  template <int OPT>
  __device__ __forceinline__ bool certify(float L, int sel, int c0, int N, float clip,
                                          float temp) const {
    const float delta = delta_l(L) + delta_z<OPT>(clip, temp);
    if constexpr ((OPT & kOptLean) != 0) {
      // the lane's runner-up from its top two: the second if the lane holds sel (a tie
      // with sel in the same lane leaves top2 = 0), else its largest (a tie in another
      // lane: 0)
      const float r = (unsigned)(sel - c0) < (unsigned)EPL ? top2 : top1;
      return __builtin_isfinite(L) && r < -delta;
    }
    // the lane's runner-up: the largest v[k] other than sel's (masked and past-the-row slots
    // are -inf; a NaN anywhere makes L NaN, which fails the finiteness test).  One max chain
    // instead of a per-slot test (r04: certified kernel 20.3 -> 18.4 us at 102,400 x 100)
    float r = -__builtin_inff();
#pragma unroll
    for (int k = 0; k < EPL; ++k) r = fmaxf(r, c0 + k == sel ? -__builtin_inff() : v[k]);
    return __builtin_isfinite(L) && r < -delta;
  }

  // greedy action of the row (valid on every lane of the group) and its logp.  LEAN (the
  // certified fast pass): the first index of the maximum itself (v = 0) -- a rounding tie
  // with it (fl(v - L) == fl(-L) for some v < 0) fails the certification anyway
  template <bool LEAN = false>
  __device__ __forceinline__ int select(float L, int c0, float& lp) const {
    lp = 0.f - L;
    // the lane's first matching slot k (inline constants), c0 added once
    constexpr int kNone = 0x40000000;
    int kk = kNone;
#pragma unroll
    for (int k = EPL - 1; k >= 0; --k) kk = (LEAN ? v[k] == 0.f : v[k] - L == lp) ? k : kk;
    const int idx = grp_min_int<RL>(c0 + kk);
    return idx >= kNone ? 0 : idx;  // no match only when L is NaN: all logp NaN
  }
};

// One row's greedy step on the GreedyRow engine: softmax_shift + select, or, with
// kOptCert, the fast math certified per row and, for any wave that holds an uncertified
// valid row (wave-uniform branch: the group reductions need every lane), the exact z of
// the row's candidates (tier 1) or the exact math for the whole wave (tier 2), both from
// the raw logits read again.  Returns
// the action; L and lp as select().  g.v afterwards: the fast shifted values, or after
// tier 2 the exact ones (the full log-probabilities, either within the certified
// tolerance).  r04: the old fallback (the exact row reloaded from HBM for the whole wave)
// cost 2.5 us of tail on a 19 us launch for 15 of 25,600 waves.  Measured and dropped (r04):
// the fallback as a called (noinline) function -- the callee's registers count toward the
// kernel's, 72 VGPRs; a waves-per-EU floor of 8 -- spills, 22.6-24.4 us; the compacted
// tanh in the fallback -- 79 VGPRs.

template <int OPT, int RL, int EPL, int VW>
__device__ __forceinline__ int greedy_row(GreedyRow<RL, EPL, VW>& g, bool valid, int N, float clip,
                                          float temp, int sl, int c0, float* lds_row, float& L,
                                          float& lp, const float* lrow, const uint8_t* mrow) {
  if constexpr ((OPT & kOptCert) != 0) {
    constexpr int OF = (OPT & ~kOptCert) | kOptFast | kOptLean,
                  OE = OPT & ~(kOptCert | kOptFast);
    using GR = GreedyRow<RL, EPL, VW>;
    // the raw logits for the fallbacks: read again from the row (an L2 / HBM read, only in
    // the rare fallback waves).  Stashing them in the group's LDS row instead (2
    // ds_write_b128 per lane on the hot path) measured +1.8 us on a 14.8 us launch (r04).
    const float* stash = lrow + c0;
    L = g.template softmax_shift<OF>(clip, temp, N, sl, lds_row);
    int sel = g.template select<true>(L, c0, lp);
    const bool ok = !valid || g.template certify<OF>(L, sel, c0, N, clip, temp);
    // rare (15 of 25,600 waves at the POMO timing shape): laid out after the hot path
    if (__builtin_expect(__any(!ok), 0)) {
      const int grp = lane_id() / RL;
      const uint64_t gmask = (RL == 64 ? ~0ull : ((1ull << RL) - 1ull)) << (grp * RL);
      const bool row_ok = (__ballot(!ok) & gmask) == 0ull;
      // Tier 1: the exact processed logit z of the candidates only -- the elements the
      // bound did not rule out (v[k] >= -delta): the exact maximum is one of them.  The
      // action is the first index of the exact maximum unless a candidate before it could
      // round to the same log-probability (|z_k - m| within the L part of the bound); then,
      // and for rows whose L is not finite, tier 2.  The row keeps the fast log-sum-exp:
      // logp = the fast v of the exact action - L (the certified rows' accuracy).
      const float dz = GR::template delta_z<OF>(clip, temp), dl = GR::delta_l(L);
      uint32_t pend = 0u;
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (valid && !row_ok && g.v[k] >= -(dl + dz)) pend |= 1u << k;
      // one exact z per lane (one tanh code copy; the candidates are usually the top two
      // and in different lanes): a lane with two or more sends the row to tier 2
      const int kc = pend ? __builtin_ctz(pend) : 0;
      const float zc = pend ? GR::template z_of<OE>(stash[kc], clip, temp) : -__builtin_inff();
      const bool multi = (pend & (pend - 1u)) != 0u;
      const float mz = grp_max<RL>(zc);
      const int wi = grp_min_int<RL>(pend && zc == mz ? c0 + kc : 0x7fffffff);
      const bool amb = (__ballot(multi || (pend && c0 + kc < wi && zc - mz >= -dl)) & gmask) !=
                       0ull;  // group-uniform from here on
      const bool fix = valid && !row_ok;
      const bool tier2 = fix && (amb || !__builtin_isfinite(L) || wi == 0x7fffffff);
      float lw = -__builtin_inff();
#pragma unroll
      for (int k = 0; k < EPL; ++k) lw = c0 + k == wi ? g.v[k] - L : lw;
      lw = grp_max<RL>(lw);  // every lane joins the group reduction
      if (fix && !tier2) {
        lp = lw;
        sel = wi;
        if constexpr (kDiagCertCount) lp = -23456.f;
      }
      // Tier 2 (rarer still): the whole wave in the exact math on the row read again (for
      // the other rows the same action, their exact logp)
      if (__any(tier2)) {
        g.load(valid, N, lrow, mrow, c0);
        L = g.template softmax_shift<OE, false>(clip, temp, N, sl, lds_row);
        sel = g.select(L, c0, lp);
        if (kDiagCertCount && tier2) lp = -12345.f;
      }
    }
    (void)lrow;
    (void)mrow;
    return sel;
  } else {
    L = g.template softmax_shift<OPT>(clip, temp, N, sl, lds_row);
    return g.select(L, c0, lp);
  }
}

template <int RL, int EPL, int VW, int OPT>
__global__ __launch_bounds__(256) void decode_greedy_kernel(
    int64_t B, int N, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, float* __restrict__ full, int32_t* status) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  // one row group per wave: the grid covers B (no grid-stride loop, so no values are
  // hoisted into registers across row groups -- r04: certified 71 -> fewer VGPRs)
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  do {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask ? mask + r * (int64_t)N : nullptr;
    g.load(valid, N, lrow, mrow, c0);
    float lp, L;
    const int sel = greedy_row<OPT>(g, valid, N, clip, temp, sl, c0, group_scratch<RL, EPL>(lds, grp),
                                    L, lp, lrow, mrow);
    if (!valid) continue;
    if (full) g.store_logp(N, L, full + r * (int64_t)N, c0);
    if (sl == 0) {
      // L is finite or NaN (the exp-sum is >= 1 unless NaN); finite means the argmax
      // element is unmasked, NaN means index 0 was taken
      if (mask && L != L && !g.allowed(0)) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = sel;
      if (logp_sel) logp_sel[r] = lp;
    }
  } while (0);
}

template <int RL, int EPL, bool VEC, int OPT>
__global__ __launch_bounds__(256) void decode_kernel(int64_t B, int N, const float* logits,
                                                     int64_t lstride, const uint8_t* mask,
                                                     float clip, float temp, int mode,
                                                     const int64_t* action_in, int64_t* action_out,
                                                     float* logp_sel, float* full, uint64_t seed,
                                                     uint64_t offset, int32_t* status, int top_k,
                                                     double top_p) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL;
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  // one row group per wave: the grid covers B (no grid-stride loop, so no values are
  // hoisted into registers across row groups -- r04: certified 71 -> fewer VGPRs)
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  do {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    const int64_t a_in = (mode == CO_DECODE_EVALUATE && valid) ? action_in[r] : 0;
    DecodeRow<RL, EPL, VEC, OPT> d;
    d.run(valid, N, logits + r * lstride, mask ? mask + r * (int64_t)N : nullptr, clip, temp,
          mode, a_in, seed, offset, row, sl, grp, group_scratch<RL, EPL>(lds, grp), top_k, top_p);
    if (!valid) continue;
    if (full) {
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (sl * EPL + k < N) full[r * (int64_t)N + sl * EPL + k] = d.x[k];
    }
    if (sl == 0) {
      if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= N))
        set_status(status, CO_ST_INDEX_RANGE);
      if (mode != CO_DECODE_EVALUATE && mask && !d.feas) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d.sel;
      if (logp_sel) logp_sel[r] = d.lp;
    }
  } while (0);
}

// Decode step fused with TSPEnv._step: the row's logits and action_mask are read once;
// the selected action's env transition (tsp/env.py:67-93) is applied by the same lane
// group: mask_out = mask_in minus the action, done = nothing left (group ballot),
// i + 1, first_node.  654 B per TSP-100 row-step.
template <int RL, int EPL, bool VEC, int OPT, int UNR = CO_DECODE_UNR>
__global__ __launch_bounds__(256) void tsp_decode_step_kernel(
    int64_t B, int N, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, uint8_t* __restrict__ mask_out,
    const int64_t* __restrict__ i_in, int64_t* __restrict__ i_out,
    const int64_t* __restrict__ first_in, int64_t* __restrict__ first_out, int take_first,
    uint8_t* __restrict__ done, uint8_t* __restrict__ step_reward, float* __restrict__ ll_accum,
    int32_t* status) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL;
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const unsigned long long gmask = RL == 64 ? ~0ull : (((1ull << RL) - 1ull) << (grp * RL));
  // UNR rows per lane group per iteration: every load of all UNR rows (logits, mask,
  // i, first_node, action, ll accumulator) is issued before any row's math
  // one row group per wave: the grid covers B (no grid-stride loop, so no values are
  // hoisted into registers across row groups -- r04: certified 71 -> fewer VGPRs)
  const int64_t base = wid * RPW * UNR;
  if (base >= B) return;  // wave-uniform
  do {
    DecodeRow<RL, EPL, VEC, OPT> d[UNR];
    int64_t rr[UNR], ain[UNR], iv[UNR], fv[UNR];
    bool vv[UNR];
    float acc[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t row = base + u * RPW + grp;
      vv[u] = row < B;
      rr[u] = vv[u] ? row : 0;
      ain[u] = (mode == CO_DECODE_EVALUATE && vv[u]) ? action_in[rr[u]] : 0;
      iv[u] = vv[u] ? i_in[rr[u]] : 0;
      fv[u] = (vv[u] && !take_first) ? first_in[rr[u]] : 0;
      acc[u] = (vv[u] && ll_accum) ? ll_accum[rr[u]] : 0.f;
      d[u].load(vv[u], N, logits + rr[u] * lstride, mask_in + rr[u] * (int64_t)N, sl);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool valid = vv[u];
      const int64_t r = rr[u], a_in = ain[u];
      d[u].compute(valid, N, clip, temp, mode, a_in, seed, offset, base + u * RPW + grp, sl,
                   grp, group_scratch<RL, EPL>(lds, grp));
      bool any_left = false;
      uint8_t* orow = mask_out + r * (int64_t)N;
      const int c0 = sl * EPL;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        if (c0 + k == d[u].sel) d[u].mk[k] = 0;
        any_left |= (valid && c0 + k < N && d[u].mk[k] != 0);
      }
      if (VEC) {
#pragma unroll
        for (int j = 0; j < EPL / 4; ++j)
          if (valid && c0 + 4 * j < N)
            *reinterpret_cast<uint32_t*>(orow + c0 + 4 * j) =
                (uint32_t)d[u].mk[4 * j] | ((uint32_t)d[u].mk[4 * j + 1] << 8) |
                ((uint32_t)d[u].mk[4 * j + 2] << 16) | ((uint32_t)d[u].mk[4 * j + 3] << 24);
      } else {
#pragma unroll
        for (int k = 0; k < EPL; ++k)
          if (valid && c0 + k < N) orow[c0 + k] = d[u].mk[k];
      }
      const bool left = (__ballot(any_left) & gmask) != 0;
      if (valid && sl == 0) {
        if (mode == CO_DECODE_EVALUATE && (a_in < 0 || a_in >= N))
          set_status(status, CO_ST_INDEX_RANGE);
        if (mode != CO_DECODE_EVALUATE && !d[u].feas) set_status(status, CO_ST_INFEASIBLE);
        const int64_t a = mode == CO_DECODE_EVALUATE ? a_in : (int64_t)d[u].sel;
        action_out[r] = a;
        if (logp_sel) logp_sel[r] = d[u].lp;
        if (ll_accum) ll_accum[r] = acc[u] + d[u].lp;  // get_log_likelihood's sum, per step
        i_out[r] = iv[u] + 1;
        first_out[r] = take_first ? a : fv[u];
        done[r] = !left;
        step_reward[r] = 0;
      }
    }
  } while (0);
}

// Greedy decode step fused with TSPEnv._step on the GreedyRow engine (the POMO /
// multistart-greedy hot loop); same outputs as tsp_decode_step_kernel in greedy mode.
// The mask words are updated in registers (the selected byte cleared) and stored back.
// STAGE (round 6): the wave's RPW logits rows and mask rows (contiguous: lstride == N,
// N % 4 == 0, 16-byte aligned) arrive by non-temporal LDS-DMA -- whole-line streams --
// and the lanes read their chunks from LDS; the certified fallback re-reads the row from
// memory as before.
__host__ __device__ inline size_t tsp_dstage_bytes(int rpw, int N) {
  return (size_t)rpw * N * 4 + (((size_t)rpw * N + 15) & ~(size_t)15);
}
template <int RL, int EPL, int VW, int OPT, bool STAGE = false>
__global__ __launch_bounds__(256) void tsp_decode_greedy_kernel(
    int64_t B, int N, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint8_t* __restrict__ mask_out, const int64_t* __restrict__ i_in,
    int64_t* __restrict__ i_out, const int64_t* __restrict__ first_in,
    int64_t* __restrict__ first_out, int take_first, uint8_t* __restrict__ done,
    uint8_t* __restrict__ step_reward, float* __restrict__ ll_accum, int32_t* status) {
  constexpr int RPW = 64 / RL;
  __shared__ __attribute__((aligned(16))) float lds[4 * 64 * EPL];
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dstage[];
  const int lane = lane_id(), sl = lane % RL, grp = lane / RL, c0 = sl * EPL;
  const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_in_block();
  const unsigned long long gmask = RL == 64 ? ~0ull : (((1ull << RL) - 1ull) << (grp * RL));
  // one row group per wave: the grid covers B (no grid-stride loop, so no values are
  // hoisted into registers across row groups -- r04: certified 71 -> fewer VGPRs)
  const int64_t base = wid * RPW;
  if (base >= B) return;  // wave-uniform
  do {
    const int64_t row = base + grp;
    const bool valid = row < B;
    const int64_t r = valid ? row : 0;
    int64_t iv = 0, fv = 0;
    float acc = 0.f;
    if (valid && sl == 0) {
      iv = i_in[r];
      if (!take_first) fv = first_in[r];
      if (ll_accum) acc = ll_accum[r];
    }
    GreedyRow<RL, EPL, VW> g;
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask_in + r * (int64_t)N;
    if constexpr (STAGE) {
      const int nr = (int)(B - base < RPW ? B - base : RPW);
      unsigned char* sw = s_dstage + (size_t)wave_in_block() * tsp_dstage_bytes(RPW, N);
      wave_dma<2>(reinterpret_cast<const unsigned char*>(logits + base * N), nr * N * 4, sw);
      wave_dma<2>(mask_in + base * N, nr * N, sw + (size_t)RPW * N * 4);
      wave_dma_wait();
      g.load(valid, N, reinterpret_cast<const float*>(sw) + grp * N, sw + (size_t)RPW * N * 4 + grp * N,
             c0);
    } else {
      g.load(valid, N, lrow, mrow, c0);
    }
    float lp, L;
    const int sel = greedy_row<OPT>(g, valid, N, clip, temp, sl, c0,
                                           group_scratch<RL, EPL>(lds, grp), L, lp, lrow, mrow);
    const bool feas0 = g.allowed(0);
    uint32_t left = 0u;
#pragma unroll
    for (int j = 0; j < EPL / 4; ++j) {
      const int off = sel - (c0 + 4 * j);
      if ((unsigned)off < 4u) g.mw[j] &= ~(0xffu << (8 * off));
      left |= g.mw[j];
    }
    if (valid) g.store_mask(N, mask_out + r * (int64_t)N, c0);
    const bool any_left = (__ballot(left != 0u) & gmask) != 0;
    if (valid && sl == 0) {
      if (L != L && !feas0) set_status(status, CO_ST_INFEASIBLE);
      action_out[r] = sel;
      if (logp_sel) logp_sel[r] = lp;
      if (ll_accum) ll_accum[r] = acc + lp;  // get_log_likelihood's sum, per step
      i_out[r] = iv + 1;
      first_out[r] = take_first ? (int64_t)sel : fv;
      done[r] = !any_left;
      step_reward[r] = 0;
    }
  } while (0);
}

// ---------------------------------------------------------------------------
// Rows longer than the register row engines hold (N > 2048): one 256-thread workgroup
// per row, the processed logits recomputed from the row in each pass instead of kept in
// registers.  Always the exact math (ATen's log_softmax bits: SLEEF exp/log, the 16
// accumulator chains of map_reduce_all walked over 1,024-element LDS chunks by 16
// threads, the xor-8/4/2/1 butterfly; correctly rounded tanh).  Greedy = first index of
// the maximal logp (as GreedyRow::select), evaluate, sampling = inverse CDF over the row
// in index order (statistical parity, like the short rows: a different summation order
// than DecodeRow's lane layout), top-k by level peeling.  top-p is not offered here.
namespace {

constexpr int kLongThreads = 256, kLongChunk = 1024;

template <int OPT>
__device__ __forceinline__ float long_proc(float x, uint8_t mk, float clip, float temp) {
  float v = x;
  if (OPT & kOptClip) v = tanh_cr(v) * clip;
  if (!mk) v = -__builtin_inff();
  if (OPT & kOptTemp) v = v / temp;  // x / 1 == x: skipped for temp == 1
  return v;
}

// block reductions of the 4 waves (every thread returns the result)
__device__ __forceinline__ float blk_max(float v, float* sh) {
  v = wave_max(v);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float blk_sum(float v, float* sh) {
  v = wave_sum(v);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ int blk_min_int(int v, int* sh) {
  v = wave_min_int(v);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const int r = min(min(sh[0], sh[1]), min(sh[2], sh[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ int blk_max_int(int v, int* sh) {
  return -blk_min_int(-v, sh);
}

template <int OPT>
__global__ __launch_bounds__(kLongThreads) void decode_long_kernel(
    int64_t B, int N, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, float* __restrict__ full, uint64_t seed, uint64_t offset,
    int32_t* status, int top_k) {
  __shared__ float chunk[kLongChunk];
  __shared__ float shf[4];
  __shared__ int shi[4];
  __shared__ float bcast;
  const float NEG_INF = -__builtin_inff();
  const int tid = threadIdx.x, lane = lane_id();
  for (int64_t r = blockIdx.x; r < B; r += gridDim.x) {
    const float* lrow = logits + r * lstride;
    const uint8_t* mrow = mask ? mask + r * (int64_t)N : nullptr;
    auto proc = [&](int c) { return long_proc<OPT>(lrow[c], mrow ? mrow[c] : 1, clip, temp); };
    float m = NEG_INF;
    for (int c = tid; c < N; c += kLongThreads) m = fmaxf(m, proc(c));
    m = blk_max(m, shf);
    // top-k (decoding.py:112-117): the k-th largest counted with multiplicity
    float thr = NEG_INF;
    if (top_k > 0 && top_k < N) {
      float hi = __builtin_inff();
      int remaining = top_k;
      for (int it = 0; it < top_k; ++it) {
        float lm = NEG_INF;
        for (int c = tid; c < N; c += kLongThreads) {
          const float v = proc(c);
          if (v < hi) lm = fmaxf(lm, v);
        }
        lm = blk_max(lm, shf);
        if (lm == NEG_INF) break;
        float cnt = 0.f;  // counts < 2^24: exact in f32
        for (int c = tid; c < N; c += kLongThreads) cnt += proc(c) == lm ? 1.f : 0.f;
        const int total = (int)blk_sum(cnt, shf);
        if (total >= remaining) {
          thr = lm;
          break;
        }
        remaining -= total;
        hi = lm;
      }
    }
    auto val = [&](int c) {
      const float v = proc(c);
      return v < thr ? NEG_INF : v;
    };
    // exp-sum in map_reduce_all's order: accumulator j (thread j < 16) adds the
    // elements c = j (mod 16) left to right, one 1,024-element LDS chunk at a time
    float acc = 0.f;
    for (int base = 0; base < N; base += kLongChunk) {
#pragma unroll
      for (int q = 0; q < kLongChunk / kLongThreads; ++q) {
        const int c = base + tid + kLongThreads * q;
        chunk[tid + kLongThreads * q] = c < N ? aten_expf(val(c) - m) : 0.f;
      }
      __syncthreads();
      if (tid < 16) {
        const int lim = min(kLongChunk, N - base);
        for (int i = 0; 16 * i + tid < lim; ++i) {
          const float e = chunk[16 * i + tid];
          acc = (base == 0 && i == 0) ? e : acc + e;
        }
      }
      __syncthreads();
    }
    if (tid < 64) {  // wave 0: the butterfly of vec_reduce_all on lanes 0..15
      float v = acc;
      v += __shfl_xor(v, 8, 16);
      v += __shfl_xor(v, 4, 16);
      v += __shfl_xor(v, 2, 16);
      v += __shfl_xor(v, 1, 16);
      if (tid == 0) bcast = aten_logf(v);
    }
    __syncthreads();
    const float L = bcast;
    __syncthreads();
    auto logp = [&](int c) { return (val(c) - m) - L; };  // ATen association
    int sel = 0;
    if (mode == CO_DECODE_GREEDY) {
      // first index whose logp equals the maximum fl(0 - L) (GreedyRow::select); a NaN L
      // (all masked / NaN logits) matches nothing: index 0, like torch.argmax over NaNs
      const float top = 0.f - L;
      int idx = 0x7fffffff;
      for (int c = tid; c < N; c += kLongThreads)
        if (logp(c) == top) {
          idx = c;
          break;
        }
      idx = blk_min_int(idx, shi);
      sel = idx == 0x7fffffff ? 0 : idx;
    } else if (mode == CO_DECODE_SAMPLING) {
      const uint32_t rr = philox_u32(seed, offset, (uint64_t)r);
      const float u = (float)(rr >> 8) * (1.0f / 16777216.0f);
      float own = 0.f;
      for (int c = tid; c < N; c += kLongThreads) own += expf(logp(c));
      const float target = u * blk_sum(own, shf);
      float carry = 0.f;
      int hit = 0x7fffffff, last = -1;
      for (int base = 0; base < N; base += kLongThreads) {
        const int c = base + tid;
        const float p = c < N ? expf(logp(c)) : 0.f;
        float incl = p;  // wave inclusive scan, then the earlier waves' totals
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const float t = __shfl_up(incl, d, 64);
          if (lane >= d) incl += t;
        }
        if (lane == 63) shf[tid >> 6] = incl;
        __syncthreads();
        float before = carry;
        for (int w = 0; w < (tid >> 6); ++w) before += shf[w];
        const float tot = (shf[0] + shf[1]) + (shf[2] + shf[3]);
        __syncthreads();
        const float run = before + incl;
        int h = (p > 0.f && run > target) ? c : 0x7fffffff;
        h = blk_min_int(h, shi);
        last = max(last, blk_max_int(p > 0.f ? c : -1, shi));
        carry += tot;
        if (h != 0x7fffffff) {
          hit = h;
          break;
        }
      }
      sel = hit != 0x7fffffff ? hit : (last >= 0 ? last : 0);
    } else {
      const int64_t a = action_in[r];
      sel = (a < 0 || a >= N) ? 0 : (int)a;
    }
    if (full)
      for (int c = tid; c < N; c += kLongThreads) full[r * (int64_t)N + c] = logp(c);
    if (tid == 0) {
      if (mode == CO_DECODE_EVALUATE) {
        const int64_t a = action_in[r];
        if (a < 0 || a >= N) set_status(status, CO_ST_INDEX_RANGE);
        action_out[r] = a;
      } else {
        if (mrow && !mrow[sel]) set_status(status, CO_ST_INFEASIBLE);
        action_out[r] = sel;
      }
      if (logp_sel) logp_sel[r] = logp(sel);
    }
    __syncthreads();  // the LDS scratch is reused by the next row
  }
}

}  // namespace

// RL lanes x EPL consecutive elements per row, by row-length bucket (CO_RL* above).
#define CO_ROW_DISPATCH(LAUNCH, V)                           \
  if (N <= 16) LAUNCH(CO_RL16, 16 / CO_RL16, V);             \
  else if (N <= 32) LAUNCH(CO_RL32, 32 / CO_RL32, V);        \
  else if (N <= 64) LAUNCH(CO_RL64, 64 / CO_RL64, V);        \
  else if (N <= 128) LAUNCH(CO_RL128, 128 / CO_RL128, V);    \
  else if (N <= 256) LAUNCH(CO_RL256, 256 / CO_RL256, V);    \
  else if (N <= 512) LAUNCH(64, 8, V);                       \
  else if (N <= 1024) LAUNCH(64, 16, V);                     \
  else LAUNCH(64, 32, V)

// the uniform clip / temperature / fast-math options as the OPT template flags
#define CO_OPT_CASE(V, LAUNCH, KERNEL, ...) \
  case V: {                                 \
    constexpr int OPT = V;                  \
    LAUNCH(KERNEL, __VA_ARGS__);            \
    break;                                  \
  }
#define CO_OPT_DISPATCH(LAUNCH, KERNEL, ...)                                            \
  do {                                                                                  \
    switch ((clip > 0.f ? kOptClip : 0) | (temp != 1.f ? kOptTemp : 0) |                \
            (fast ? kOptFast : 0)) {                                                    \
      CO_OPT_CASE(0, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(1, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(2, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(3, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(4, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(5, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(6, LAUNCH, KERNEL, __VA_ARGS__)                                       \
      CO_OPT_CASE(7, LAUNCH, KERNEL, __VA_ARGS__)                                       \
    }                                                                                   \
  } while (0)

// greedy kernels: the same eight, or (cert) the four certified variants
#define CO_OPT_DISPATCH_G(LAUNCH, KERNEL, ...)                                          \
  do {                                                                                  \
    const int opt_ = (clip > 0.f ? kOptClip : 0) | (temp != 1.f ? kOptTemp : 0);        \
    if (cert) {                                                                         \
      switch (opt_ | kOptCert) {                                                        \
        CO_OPT_CASE(8, LAUNCH, KERNEL, __VA_ARGS__)                                     \
        CO_OPT_CASE(9, LAUNCH, KERNEL, __VA_ARGS__)                                     \
        CO_OPT_CASE(10, LAUNCH, KERNEL, __VA_ARGS__)                                    \
        CO_OPT_CASE(11, LAUNCH, KERNEL, __VA_ARGS__)                                    \
      }                                                                                 \
    } else {                                                                            \
      CO_OPT_DISPATCH(LAUNCH, KERNEL, __VA_ARGS__);                                     \
    }                                                                                   \
  } while (0)

inline unsigned decode_grid(int64_t B, int N, int unr = 1) {
  const int rl = N <= 16 ? CO_RL16 : N <= 32 ? CO_RL32 : N <= 64 ? CO_RL64
               : N <= 128 ? CO_RL128 : N <= 256 ? CO_RL256 : 64;
  const int64_t waves = ((B + unr - 1) / unr * rl + 63) / 64;
  return cover_grid(waves, 4);  // every row group gets its wave; 0: B too large
}

// widest GreedyRow load (4 / 2 / 1 elements) the row length, stride and pointers allow
inline int greedy_vw(int64_t N, int64_t lstride, const float* logits, const uint8_t* m_in,
                     const uint8_t* m_out, const float* full) {
  const uintptr_t f = reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(full);
  const uintptr_t m = reinterpret_cast<uintptr_t>(m_in) | reinterpret_cast<uintptr_t>(m_out);
  if (N % 4 == 0 && lstride % 4 == 0 && (f & 15) == 0 && (m & 3) == 0) return 4;
  return N >= 4 ? 3 : 2;  // 4-element chunks on rows of any N and alignment (2: N < 4)
}

inline bool decode_vec_ok(const float* logits, int64_t lstride, const uint8_t* mask, int64_t N) {
  return (N % 4 == 0) && (lstride % 4 == 0) &&
         ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(mask)) & 15) == 0;
}

}  // namespace
