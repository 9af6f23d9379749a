// Device restatements of the f32 math that ATen's CPU log_softmax evaluates, so the
// decode step reproduces the reference's log-probabilities bit for bit.
//
// F.log_softmax on a contiguous [B, N] f32 tensor (the reference's process_logits,
// rl4co/utils/decoding.py:191) runs ATen's _vec_log_softmax_lastdim: per row
//   m = max(x);  s = sum(exp(x - m));  L = log(s);  logp = (x - m) - L
// with exp / log = SLEEF's expf_u10 / logf_u10 (FMA variants, as ATen's AVX2 / AVX512
// builds call them) and the sum in the order of vec::map_reduce_all over 16-wide vectors
// (AVX512; the GPU box's host and this container both report ATen capability AVX512):
// accumulator l (0..15) adds elements l, l+16, l+32, ... left to right, then the
// accumulators reduce as a butterfly (xor 8, 4, 2, 1); rows with N < 16 sum e_0 + e_1 + ...
// sequentially.  oracle/c/aten_math.c is the CPU restatement of the same three functions;
// tests/test_aten_math.py pins it bit-exact against torch (every f32 input <= 0 for exp,
// F.log_softmax rows of every width class) -- SLEEF is a dependency of torch, not of the
// reference, and is restated here from its published algorithm (sleef/src/libm/sleefsimdsp.c,
// xexpf / xlogf_u1 with ENABLE_FMA_SP).
//
// tanh: torch.tanh on CPU dispatches to MKL VML's vmsTanh (HA), a closed implementation
// whose results differ from the correctly rounded tanh in ~0.75 % of inputs (1 ulp).  It
// cannot be restated, so the exact path evaluates tanh in f64 and rounds once: the
// correctly rounded value (up to f64 double-rounding, ~2^-29 of inputs).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace co {

// SLEEF xexpf (u10, FMA): q = rint(d / ln2); s = d - q*ln2 (two-part ln2); degree-5
// polynomial; 1 + (s*s*u + s) scaled by 2^q; 0 below -104, +inf above 100.
__device__ __forceinline__ float aten_expf(float d) {
  const float qf = __builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  const int q = (int)qf;
  float s = __builtin_fmaf(qf, -0.693145751953125f, d);
  s = __builtin_fmaf(qf, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
  u = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
  u = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
  u = __builtin_fmaf(u, s, 0.166666671633720397949219f);
  u = __builtin_fmaf(u, s, 0.5f);
  u = 1.0f + __builtin_fmaf(s * s, u, s);
  // vldexp2: u * 2^(q>>1) * 2^(q - (q>>1)); both factors are normal for |q| <= 252, so
  // this is the single rounding of v_ldexp_f32
  u = __builtin_amdgcn_ldexpf(u, q);
  u = d < -104.f ? 0.f : u;
  u = 100.f < d ? __builtin_inff() : u;
  return u;
}

// SLEEF xlogf_u1 (FMA) for the exp-sums log_softmax takes the log of (>= 1, or inf/NaN):
// d = m * 2^e with m in [0.75, 1.5); log(d) = e*ln2 + 2*atanh((m-1)/(m+1)) in
// double-float arithmetic (head + tail f32 pairs).
__device__ __forceinline__ float aten_logf(float d) {
  struct F2 {
    float x, y;
  };
  auto fmapn = [](float a, float b, float c) { return __builtin_fmaf(a, b, -c); };
  auto fmanp = [](float a, float b, float c) { return __builtin_fmaf(-a, b, c); };
  // e = floor(log2(d * 4/3)) (vgetexp), m = d * 2^-e (vgetmant, exact)
  const float dd = d * (1.0f / 0.75f);
  const int e = (int)((__float_as_uint(dd) >> 23) & 0xffu) - 127;
  const float m = __builtin_amdgcn_ldexpf(d, -e);
  // s = dfmul((ln2 hi, ln2 lo), e)
  const float ef = (float)e;
  F2 s;
  s.x = 0.69314718246459960938f * ef;
  s.y = __builtin_fmaf(-1.904654323148236017e-09f, ef, fmapn(0.69314718246459960938f, ef, s.x));
  // x = dfdiv(dfadd2(-1, m), dfadd2(1, m))
  F2 n, q;
  n.x = -1.0f + m;
  {
    const float v = n.x - -1.0f;
    n.y = (-1.0f - (n.x - v)) + (m - v);
  }
  q.x = 1.0f + m;
  {
    const float v = q.x - 1.0f;
    q.y = (1.0f - (q.x - v)) + (m - v);
  }
  F2 x;
  {
    const float t = 1.0f / q.x;
    x.x = n.x * t;
    const float u = fmapn(t, n.x, x.x);
    const float v = fmanp(q.y, t, fmanp(q.x, t, 1.0f));
    x.y = __builtin_fmaf(x.x, v, __builtin_fmaf(n.y, t, u));
  }
  const float x2 = x.x * x.x;
  float t = +0.3027294874e+0f;
  t = __builtin_fmaf(t, x2, +0.3996108174e+0f);
  t = __builtin_fmaf(t, x2, +0.6666694880e+0f);
  // s = dfadd(s, dfscale(x, 2)); s = dfadd(s, x2 * x.x * t)
  {
    const float sx = s.x + x.x * 2.0f;
    s.y = (((s.x - sx) + x.x * 2.0f) + s.y) + x.y * 2.0f;
    s.x = sx;
  }
  {
    const float w = (x2 * x.x) * t;
    const float sx = s.x + w;
    s.y = ((s.x - sx) + w) + s.y;
    s.x = sx;
  }
  float r = s.x + s.y;
  r = d == __builtin_inff() ? __builtin_inff() : r;
  r = (d < 0.f || d != d) ? __builtin_nanf("") : r;
  r = d == 0.f ? -__builtin_inff() : r;
  return r;
}

// tanh rounded once from an f64 evaluation accurate to a few f64 ulps (see the header
// comment for why not ATen's own tanh): tanh|x| = -expm1(-2|x|) / (2 + expm1(-2|x|)),
// expm1(y) = 2^k (expm1(r) + 1) - 1 with y = k ln2 + r, |r| <= ln2/2, expm1(r) by its
// degree-13 Taylor polynomial (truncation < 2^-56), the quotient by v_rcp_f64 + Newton.
// ~30 f64 operations against ~140 for the libm tanh(double) (double-double inside).
// |x| < 2^-12 returns x (tanh x = x(1 - x^2/3 ...) rounds to x there) and |x| >= 9.1 returns
// +-1 (tanh rounds to 1 from 9.0109); NaN propagates.
__device__ __forceinline__ double sconst(double c) {
  asm volatile("" : "+s"(c));  // a scalar register here: SALU moves, not a live VGPR pair
  return c;
}
__device__ __forceinline__ float tanh_cr(float x) {
  const float ax = __builtin_fabsf(x);
  if (!(ax >= 0x1p-12f)) return x;            // tiny, or NaN
  if (ax >= 9.1f) return __builtin_copysignf(1.0f, x);
  const double y = -2.0 * (double)ax;         // exact
  const double kd = __builtin_rint(y * 1.4426950408889634074);
  const int k = (int)kd;
  double r = __builtin_fma(kd, -6.93147180559890330187e-01, y);   // ln2 hi (exact product)
  r = __builtin_fma(kd, -5.49792301870837115524e-14, r);          // ln2 lo
  // the Taylor coefficients are materialised into SGPRs at each use (sconst): hoisted out
  // of the kernels' loops they occupied 20 VGPRs for the whole kernel, plus a register
  // copy per Horner step (v_fmac accumulates into its constant's register)
  double q = sconst(1.0 / 6227020800.0);                          // 1/13!
  q = __builtin_fma(q, r, sconst(1.0 / 479001600.0));
  q = __builtin_fma(q, r, sconst(1.0 / 39916800.0));
  q = __builtin_fma(q, r, sconst(1.0 / 3628800.0));
  q = __builtin_fma(q, r, sconst(1.0 / 362880.0));
  q = __builtin_fma(q, r, sconst(1.0 / 40320.0));
  q = __builtin_fma(q, r, sconst(1.0 / 5040.0));
  q = __builtin_fma(q, r, sconst(1.0 / 720.0));
  q = __builtin_fma(q, r, sconst(1.0 / 120.0));
  q = __builtin_fma(q, r, sconst(1.0 / 24.0));
  q = __builtin_fma(q, r, sconst(1.0 / 6.0));
  q = __builtin_fma(q, r, 0.5);
  const double p = __builtin_fma(r * r, q, r);                    // expm1(r)
  // expm1(y) = 2^k p + (2^k - 1), both terms exact-scaled; k <= 0
  const double em1 = __builtin_amdgcn_ldexp(p, k) + (__builtin_amdgcn_ldexp(1.0, k) - 1.0);
  const double num = -em1, den = 2.0 + em1;                       // den in (1, 2]
  double rc = __builtin_amdgcn_rcp(den);
  rc = __builtin_fma(__builtin_fma(-den, rc, 1.0), rc, rc);
  rc = __builtin_fma(__builtin_fma(-den, rc, 1.0), rc, rc);
  double t = num * rc;
  t = __builtin_fma(__builtin_fma(-den, t, num), rc, t);
  return __builtin_copysignf((float)t, x);
}

// ATen's exp-sum for one row held by an RL-lane group, EPL consecutive elements per lane
// (lane sl owns c = sl*EPL + k, out-of-row slots hold anything: they are skipped).
// `e` are the lane's exp(x - m) values; `row` is the group's LDS scratch of RL*EPL floats.
// The 16 accumulator chains are re-read from LDS by the lanes that own them: for RL >= 16
// lane sl sums residue sl % 16 (every 16-lane row computes the same chains); for RL < 16
// lane sl sums the 16/RL residues pi(sl) + RL*j.  The butterfly is then DPP moves whose
// lane pairing equals the xor pairing on residues (row_ror:8 / row_ror:4 on a 16-lane
// row, row_half_mirror on an 8-lane group with pi = s < 4 ? s : s ^ 3, quad_perm xor 2 /
// xor 1), so every lane ends with exactly ATen's lane-0 sum.  The group's lanes must all
// be active (wave-uniform control flow).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// Register-only variant for 16-lane groups of 8 consecutive elements (the N in (64, 128]
// bucket, TSP-100): lane sl holds residues 8(sl&1) .. +7 at chain position sl>>1, so the 16
// accumulator chains run along lanes of equal parity.  Seven rounds of
// acc = row_shr:2(acc) + e (lanes 0-1 shift in 0: 0 + e = e exactly) leave every chain
// summed left to right in lanes 14 (residues 0-7) and 15 (residues 8-15); the butterfly is
// one lane swap (xor 8) and in-lane adds (xor 4, 2, 1); row_newbcast:14 hands the sum to the
// whole row.  Out-of-row elements must be 0.
template <int CTRL, bool BC>
__device__ __forceinline__ float dpp_fb(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, BC));
}

__device__ __forceinline__ float aten_row_sum_16x8(const float (&e)[8]) {
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = e[k];
#pragma unroll
  for (int it = 0; it < 7; ++it)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = dpp_fb<0x112, true>(acc[k]) + e[k];  // row_shr:2
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = acc[k] + dpp_fb<0xB1, false>(acc[k]);  // xor 8: lane ^ 1
  float w0 = v[0] + v[4], w1 = v[1] + v[5], w2 = v[2] + v[6], w3 = v[3] + v[7];
  const float s = (w0 + w2) + (w1 + w3);
  return dpp_fb<0x15E, false>(s);  // row_newbcast:14
}

template <int RL, int EPL>
__device__ __forceinline__ float aten_row_sum(const float (&e)[EPL], int N, int sl, float* row) {
  if constexpr (RL == 16 && EPL == 8) {
    (void)N, (void)sl, (void)row;
    return aten_row_sum_16x8(e);
  }
  const int c0 = sl * EPL;
  __builtin_amdgcn_wave_barrier();  // the previous row's chain reads stay before these writes
  if (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4)
      *reinterpret_cast<float4*>(row + c0 + k) = make_float4(e[k], e[k + 1], e[k + 2], e[k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) row[c0 + k] = e[k];
  }
  // the group's lanes read what other lanes of the same wave wrote: LDS operations of one
  // wave complete in order; the fence keeps the compiler from reordering across it
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (N < 16) {  // map_reduce_all with size < Vec::size(): sequential
    float s = row[0];
    for (int c = 1; c < N; ++c) s += row[c];
    return s;
  }
  const int chain = (N + 15) >> 4;
  if constexpr (RL >= 16) {
    const int r = sl & 15;
    float acc = row[r];
    for (int p = 1; p < chain; ++p) {
      const int c = r + 16 * p;
      acc += c < N ? row[c] : 0.f;  // + 0 leaves a sum of exps unchanged
    }
    acc += dpp_f<0x128>(acc);  // row_ror:8  (xor 8)
    acc += dpp_f<0x124>(acc);  // row_ror:4  (xor 4 on the period-8 values)
    acc += dpp_f<0x4E>(acc);   // quad_perm [2,3,0,1] (xor 2)
    acc += dpp_f<0xB1>(acc);   // quad_perm [1,0,3,2] (xor 1)
    return acc;
  } else {
    constexpr int A = RL < 16 ? 16 / RL : 1;
    const int pi = (RL == 8 && sl >= 4) ? (sl ^ 3) : sl;
    float acc[A];
#pragma unroll
    for (int j = 0; j < A; ++j) {
      const int r = pi + RL * j;
      float a = row[r];
      for (int p = 1; p < chain; ++p) {
        const int c = r + 16 * p;
        a += c < N ? row[c] : 0.f;
      }
      acc[j] = a;
    }
#pragma unroll
    for (int h = A / 2; h >= 1; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; ++j) acc[j] += acc[j + h];
    float v = acc[0];
    if (RL >= 8) v += dpp_f<0x141>(v);  // row_half_mirror (xor 4 under pi)
    if (RL >= 4) v += dpp_f<0x4E>(v);
    if (RL >= 2) v += dpp_f<0xB1>(v);
    return v;
  }
}

}  // namespace co
