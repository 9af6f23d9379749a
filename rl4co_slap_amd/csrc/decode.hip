// Fused decode step for gfx950 (rl4co/utils/decoding.py:141-191,327-399,489-499):
// tanh clip -> mask to -inf -> /temperature -> log_softmax -> greedy argmax |
// Philox inverse-CDF sample | evaluate -> logp gather, in one pass.
//
// One wavefront per row (grid-stride); the row's N <= 64*NPL logits stay in
// registers (NPL per lane), max / sum / argmax are wave reductions and the
// sampling CDF is a wave inclusive scan.  log_softmax is evaluated with the
// same association as ATen's CPU kernel: logp = (x - max) - log(sum(exp(x - max))),
// so greedy ties resolve exactly like torch.argmax (first index).
#include "co_common.hpp"

using namespace co;

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

template <int NPL>
__global__ __launch_bounds__(256) void decode_kernel(int64_t B, int N, const float* logits,
                                                     int64_t lstride, const uint8_t* mask,
                                                     float clip, float temp, int mode,
                                                     const int64_t* action_in, int64_t* action_out,
                                                     float* logp_sel, float* full, uint64_t seed,
                                                     uint64_t offset, int32_t* status) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  const float NEG_INF = -__builtin_inff();
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const float* lrow = logits + b * lstride;
    const uint8_t* mrow = mask ? mask + b * (int64_t)N : nullptr;
    float x[NPL];
    float m = NEG_INF;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int c = lane + 64 * k;
      float v = NEG_INF;
      if (c < N) {
        v = lrow[c];
        if (clip > 0.f) v = tanhf(v) * clip;
        if (mrow && !mrow[c]) v = NEG_INF;
        v = v / temp;
        m = fmaxf(m, v);
      }
      x[k] = v;
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      if (lane + 64 * k < N) s += expf(x[k] - m);
    s = wave_sum(s);
    const float L = logf(s);
#pragma unroll
    for (int k = 0; k < NPL; ++k) x[k] = (x[k] - m) - L;  // ATen association
    if (full) {
#pragma unroll
      for (int k = 0; k < NPL; ++k)
        if (lane + 64 * k < N) full[b * (int64_t)N + lane + 64 * k] = x[k];
    }
    int sel = 0;
    if (mode == CO_DECODE_GREEDY) {
      float bv = NEG_INF;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int c = lane + 64 * k;
        if (c < N && argmax_better(x[k], c, bv, bi)) { bv = x[k]; bi = c; }
      }
      wave_argmax(bv, bi);
      sel = bi;
    } else if (mode == CO_DECODE_SAMPLING) {
      const uint32_t r = philox_u32(seed, offset, (uint64_t)b);
      const float u = (float)(r >> 8) * (1.0f / 16777216.0f);
      float p[NPL];
      float tot = 0.f;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        p[k] = (lane + 64 * k < N) ? expf(x[k]) : 0.f;
        tot += p[k];
      }
      tot = wave_sum(tot);
      const float target = u * tot;
      float carry = 0.f;
      int found = -1;
      int lastpos = -1;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        float v = p[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const float t = __shfl_up(v, d, 64);
          if (lane >= d) v += t;
        }
        const float cum = carry + v;
        const bool hit = (p[k] > 0.f) && (cum > target);
        const unsigned long long bal = __ballot(hit);
        if (found < 0 && bal) found = 64 * k + __builtin_ctzll(bal);
        const unsigned long long pos = __ballot(p[k] > 0.f);
        if (pos) lastpos = 64 * k + 63 - __builtin_clzll(pos);
        carry += __shfl(v, 63, 64);
      }
      sel = found >= 0 ? found : (lastpos >= 0 ? lastpos : 0);
    } else {
      const int64_t a = action_in[b];
      sel = (a < 0 || a >= N) ? -1 : (int)a;
      if (sel < 0 && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    }
    // logp of the selected action: fetch from the owning lane's register
    float lp = 0.f;
    if (sel >= 0) {
      const int owner = sel & 63, slot = sel >> 6;
      float mine = 0.f;
#pragma unroll
      for (int k = 0; k < NPL; ++k)
        if (k == slot) mine = x[k];
      lp = __shfl(mine, owner, 64);
    }
    if (lane == 0) {
      if (mode != CO_DECODE_EVALUATE && mrow && !mrow[sel]) set_status(status, CO_ST_INFEASIBLE);
      action_out[b] = mode == CO_DECODE_EVALUATE ? action_in[b] : (int64_t)sel;
      if (logp_sel) logp_sel[b] = lp;
    }
  }
}


// Decode step fused with TSPEnv._step: the row's logits and action_mask are read once;
// the selected action's env transition (tsp/env.py:67-93) is applied in the same wave:
// mask_out = mask_in minus the action (the wave already holds the row), done = no bit
// left (ballot), i + 1, first_node.  654 B per TSP-100 row-step.
template <int NPL>
__global__ __launch_bounds__(256) void tsp_decode_step_kernel(
    int64_t B, int N, const float* __restrict__ logits, int64_t lstride,
    const uint8_t* __restrict__ mask_in, float clip, float temp, int mode,
    const int64_t* __restrict__ action_in, int64_t* __restrict__ action_out,
    float* __restrict__ logp_sel, uint64_t seed, uint64_t offset, uint8_t* __restrict__ mask_out,
    const int64_t* __restrict__ i_in, int64_t* __restrict__ i_out,
    const int64_t* __restrict__ first_in, int64_t* __restrict__ first_out, int take_first,
    uint8_t* __restrict__ done, uint8_t* __restrict__ step_reward, float* __restrict__ ll_accum,
    int32_t* status) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  const float NEG_INF = -__builtin_inff();
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const float* lrow = logits + b * lstride;
    const uint8_t* mrow = mask_in + b * (int64_t)N;
    float x[NPL];
    uint8_t mk[NPL];
    float m = NEG_INF;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int c = lane + 64 * k;
      float v = NEG_INF;
      mk[k] = 0;
      if (c < N) {
        v = lrow[c];
        mk[k] = mrow[c];
        if (clip > 0.f) v = tanhf(v) * clip;
        if (!mk[k]) v = NEG_INF;
        v = v / temp;
        m = fmaxf(m, v);
      }
      x[k] = v;
    }
    m = wave_max(m);
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      if (lane + 64 * k < N) sum += expf(x[k] - m);
    sum = wave_sum(sum);
    const float L = logf(sum);
#pragma unroll
    for (int k = 0; k < NPL; ++k) x[k] = (x[k] - m) - L;
    int sel = 0;
    if (mode == CO_DECODE_GREEDY) {
      float bv = NEG_INF;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int c = lane + 64 * k;
        if (c < N && argmax_better(x[k], c, bv, bi)) { bv = x[k]; bi = c; }
      }
      wave_argmax(bv, bi);
      sel = bi;
    } else if (mode == CO_DECODE_SAMPLING) {
      const uint32_t r = philox_u32(seed, offset, (uint64_t)b);
      const float u = (float)(r >> 8) * (1.0f / 16777216.0f);
      float p[NPL], tot = 0.f;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        p[k] = (lane + 64 * k < N) ? expf(x[k]) : 0.f;
        tot += p[k];
      }
      tot = wave_sum(tot);
      const float target = u * tot;
      float carry = 0.f;
      int found = -1, lastpos = -1;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        float v = p[k];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const float t = __shfl_up(v, d, 64);
          if (lane >= d) v += t;
        }
        const bool hit = (p[k] > 0.f) && (carry + v > target);
        const unsigned long long bal = __ballot(hit);
        if (found < 0 && bal) found = 64 * k + __builtin_ctzll(bal);
        const unsigned long long pos = __ballot(p[k] > 0.f);
        if (pos) lastpos = 64 * k + 63 - __builtin_clzll(pos);
        carry += __shfl(v, 63, 64);
      }
      sel = found >= 0 ? found : (lastpos >= 0 ? lastpos : 0);
    } else {
      const int64_t a = action_in[b];
      sel = (a < 0 || a >= N) ? 0 : (int)a;
      if ((a < 0 || a >= N) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    }
    const int owner = sel & 63, slot = sel >> 6;
    float mine = 0.f;
    int feas = 0;
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      if (k == slot) {
        mine = x[k];
        feas = mk[k];
      }
    const float lp = __shfl(mine, owner, 64);
    feas = __shfl(feas, owner, 64);
    // env step on the row the wave already holds
    bool any_left = false;
    uint8_t* orow = mask_out + b * (int64_t)N;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int c = lane + 64 * k;
      if (c < N) {
        const uint8_t v = (c == sel) ? 0 : mk[k];
        orow[c] = v;
        any_left |= v != 0;
      }
    }
    const bool left = __any(any_left);
    if (lane == 0) {
      if (mode != CO_DECODE_EVALUATE && !feas) set_status(status, CO_ST_INFEASIBLE);
      const int64_t a = mode == CO_DECODE_EVALUATE ? action_in[b] : (int64_t)sel;
      action_out[b] = a;
      if (logp_sel) logp_sel[b] = lp;
      if (ll_accum) ll_accum[b] += lp;  // get_log_likelihood's sum, step by step
      const int64_t iv = i_in[b];
      i_out[b] = iv + 1;
      first_out[b] = take_first ? a : first_in[b];
      done[b] = !left;
      step_reward[b] = 0;
    }
  }
}
}  // namespace

extern "C" int co_decode_step(int64_t B, int64_t N, const float* logits, int64_t lstride,
                              const uint8_t* mask, float clip, float temp, int mode,
                              const int64_t* action_in, int64_t* action_out, float* logp_sel,
                              float* full, uint64_t seed, uint64_t offset, int32_t* status,
                              void* stream) {
  if (B < 0 || N <= 0 || N > 64 * 32) return CO_E_INVAL;
  if (mode < 0 || mode > 2) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !action_out) return CO_E_INVAL;
  if (mode == CO_DECODE_EVALUATE && !action_in) return CO_E_INVAL;
  const dim3 grid(grid_for(B, 4, 256 * 32)), block(256);
  hipStream_t s = (hipStream_t)stream;
#define CO_DECODE(NPL)                                                                         \
  hipLaunchKernelGGL(decode_kernel<NPL>, grid, block, 0, s, B, (int)N, logits, lstride, mask, \
                     clip, temp, mode, action_in, action_out, logp_sel, full, seed, offset,    \
                     status)
  if (N <= 64) CO_DECODE(1);
  else if (N <= 128) CO_DECODE(2);
  else if (N <= 256) CO_DECODE(4);
  else if (N <= 512) CO_DECODE(8);
  else if (N <= 1024) CO_DECODE(16);
  else CO_DECODE(32);
#undef CO_DECODE
  return launch_status();
}

extern "C" int co_tsp_decode_step(int64_t B, int64_t N, const float* logits, int64_t lstride,
                                  const uint8_t* mask_in, float clip, float temp, int mode,
                                  const int64_t* action_in, int64_t* action_out,
                                  float* logp_sel, uint64_t seed, uint64_t offset,
                                  uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                                  const int64_t* first_in, int64_t* first_out, int first_mode,
                                  uint8_t* done, uint8_t* step_reward, float* ll_accum,
                                  int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > 64 * 32) return CO_E_INVAL;
  if (mode < 0 || mode > 2 || first_mode < 0 || first_mode > 1) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !mask_in || !action_out || !mask_out || !i_in || !i_out || !first_out ||
      !done || !step_reward || (first_mode == 0 && !first_in) ||
      (mode == CO_DECODE_EVALUATE && !action_in))
    return CO_E_INVAL;
  const dim3 grid(grid_for(B, 4, 256 * 32)), block(256);
  hipStream_t s = (hipStream_t)stream;
#define CO_TDS(NPL)                                                                            \
  hipLaunchKernelGGL(tsp_decode_step_kernel<NPL>, grid, block, 0, s, B, (int)N, logits,        \
                     lstride, mask_in, clip, temp, mode, action_in, action_out, logp_sel,      \
                     seed, offset, mask_out, i_in, i_out, first_in, first_out, first_mode,     \
                     done, step_reward, ll_accum, status)
  if (N <= 64) CO_TDS(1);
  else if (N <= 128) CO_TDS(2);
  else if (N <= 256) CO_TDS(4);
  else if (N <= 512) CO_TDS(8);
  else if (N <= 1024) CO_TDS(16);
  else CO_TDS(32);
#undef CO_TDS
  return launch_status();
}
