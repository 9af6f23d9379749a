/* CPU restatement of the f32 math ATen's CPU log_softmax evaluates -- TEST INFRASTRUCTURE
 * ONLY (the checker for rl4co_slap_amd/csrc/co_math.hpp; never linked into the product).
 *
 * The reference's process_logits ends in F.log_softmax(logits, dim=-1)
 * (rl4co/utils/decoding.py:191).  On a contiguous f32 [B, N] CPU tensor that is ATen's
 * _vec_log_softmax_lastdim (aten/src/ATen/native/cpu/SoftMaxKernel.cpp):
 *   m = vec::reduce_all(maximum, row)
 *   s = vec::map_reduce_all(exp(x - m), +, row)  -- Vectorized<float>::exp = SLEEF expf_u10
 *   L = Vectorized<float>::log(s)                -- SLEEF logf_u10
 *   out = (x - m) - L
 * map_reduce_all over W-wide vectors (W = 16 under ATen's AVX512 capability, which both the
 * build container and the GPU box's EPYC 9575F report): accumulator lane l sums elements
 * l, l+W, l+2W, ... left to right (a partial last vector only updates its first lanes),
 * then vec_reduce_all combines the lanes as a butterfly (xor W/2, ..., 1); rows with
 * N < W are summed sequentially.  SLEEF (a torch dependency, not reference code) is
 * restated from its published sleefsimdsp.c (xexpf, xlogf_u1, FMA variants).
 * tests/test_aten_math.py pins every function here against torch itself. */
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline float b2f(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static inline uint32_t f2b(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }

float aten_expf(float d) {
  float qf = rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  int q = (int)qf;
  float s = fmaf(qf, -0.693145751953125f, d);
  s = fmaf(qf, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = fmaf(u, s, 0.00139304355252534151077271f);
  u = fmaf(u, s, 0.00833336077630519866943359f);
  u = fmaf(u, s, 0.0416664853692054748535156f);
  u = fmaf(u, s, 0.166666671633720397949219f);
  u = fmaf(u, s, 0.5f);
  u = 1.0f + fmaf(s * s, u, s);
  if (d < -104.f || isnan(d)) return isnan(d) ? d : 0.f;
  if (100.f < d) return INFINITY;
  /* vldexp2: two power-of-two factors (each normal) */
  int h = q >> 1;
  u = u * b2f((uint32_t)(h + 0x7f) << 23);
  return u * b2f((uint32_t)(q - h + 0x7f) << 23);
}

float aten_logf(float d) {
  if (isnan(d) || d < 0.f) return NAN;
  if (d == 0.f) return -INFINITY;
  if (isinf(d)) return INFINITY;
  float dd = d * (1.0f / 0.75f);
  int e = (int)((f2b(dd) >> 23) & 0xff) - 127;
  float m = ldexpf(d, -e);
  float ef = (float)e;
  float sx = 0.69314718246459960938f * ef;
  float sy = fmaf(-1.904654323148236017e-09f, ef, fmaf(0.69314718246459960938f, ef, -sx));
  float nx = -1.0f + m, v = nx - -1.0f, ny = (-1.0f - (nx - v)) + (m - v);
  float qx = 1.0f + m; v = qx - 1.0f; float qy = (1.0f - (qx - v)) + (m - v);
  float t = 1.0f / qx;
  float xx = nx * t;
  float uu = fmaf(t, nx, -xx);
  float vv = fmaf(-qy, t, fmaf(-qx, t, 1.0f));
  float xy = fmaf(xx, vv, fmaf(ny, t, uu));
  float x2 = xx * xx;
  float p = +0.3027294874e+0f;
  p = fmaf(p, x2, +0.3996108174e+0f);
  p = fmaf(p, x2, +0.6666694880e+0f);
  float s2 = sx + xx * 2.0f;
  sy = (((sx - s2) + xx * 2.0f) + sy) + xy * 2.0f;
  sx = s2;
  float w = (x2 * xx) * p;
  s2 = sx + w;
  sy = ((sx - s2) + w) + sy;
  return s2 + sy;
}

/* correctly rounded tanh (f64 evaluation rounded once), the decode kernel's default */
float tanh_cr(float x) { return (float)tanh((double)x); }

/* exp-sum of one row in vec::map_reduce_all's order for W-wide vectors */
static float row_sum(const float* e, long n, int W) {
  if (n < W) {
    float s = e[0];
    for (long c = 1; c < n; ++c) s += e[c];
    return s;
  }
  float acc[64];
  for (int l = 0; l < W; ++l) acc[l] = e[l];
  for (long c = W; c < n; ++c) acc[c % W] += e[c];
  for (int k = W / 2; k >= 1; k >>= 1) {
    float nxt[64];
    for (int l = 0; l < W; ++l) nxt[l] = acc[l] + acc[l ^ k];
    memcpy(acc, nxt, sizeof(float) * W);
  }
  return acc[0];
}

/* F.log_softmax(x, -1) for contiguous f32 [B, N] rows, ATen's CPU evaluation */
void aten_log_softmax(const float* x, float* out, long B, long N, int W) {
  float e[4096];
  for (long b = 0; b < B; ++b) {
    const float* r = x + b * N;
    float m = r[0];
    for (long c = 1; c < N; ++c) m = (r[c] > m || isnan(r[c])) ? r[c] : m;
    for (long c = 0; c < N; ++c) e[c] = aten_expf(r[c] - m);
    float L = aten_logf(row_sum(e, N, W));
    for (long c = 0; c < N; ++c) out[b * N + c] = (r[c] - m) - L;
  }
}

void aten_expf_batch(const float* x, float* y, long n) { for (long i = 0; i < n; ++i) y[i] = aten_expf(x[i]); }
void aten_logf_batch(const float* x, float* y, long n) { for (long i = 0; i < n; ++i) y[i] = aten_logf(x[i]); }
void tanh_cr_batch(const float* x, float* y, long n) { for (long i = 0; i < n; ++i) y[i] = tanh_cr(x[i]); }
