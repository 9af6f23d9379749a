// co_decode_step / co_decode_step_ex (the decode step of rl4co/utils/decoding.py:141-191,
// 327-399,489-499 on the row engines of decode_common.hpp) and beam search's candidate
// ranking.
#include "decode_common.hpp"

#if defined(CO_DIAG_FASTTANH) || defined(CO_DIAG_FASTEXP) || defined(CO_DIAG_CVRP_CUT) || \
    defined(CO_DIAG_CERT_COUNT)  // co_diag.hpp: kDiagTimingCut || kDiagCertCount
// diagnostic build: the "exact" decode is not exact, the CVRP decode step lacks its decode
// or transition, or certified rows carry marker log-probabilities (see _native.load())
extern "C" __attribute__((visibility("default"))) const int co_variant_timing_cut_decode = 1;
#endif

extern "C" int co_decode_step_ex(int64_t B, int64_t N, const float* logits, int64_t lstride,
                                 const uint8_t* mask, float clip, float temp, int top_k,
                                 double top_p, int mode, const int64_t* action_in,
                                 int64_t* action_out, float* logp_sel, float* full, uint64_t seed,
                                 uint64_t offset, int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > (1 << 24) || top_k < 0 || top_p < 0.0 || top_p > 1.0)
    return CO_E_INVAL;
  // CO_DECODE_CERTIFIED changes only greedy picks' math (actions stay exact); other modes
  // and the filtered path run the exact math under it
  const bool cert = (mode & CO_DECODE_CERTIFIED) != 0 && (mode & CO_DECODE_FAST) == 0;
  const bool fast = (mode & CO_DECODE_FAST) != 0;
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (mode < 0 || mode > 2) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !action_out) return CO_E_INVAL;
  if (mode == CO_DECODE_EVALUATE && !action_in) return CO_E_INVAL;
  hipStream_t s = (hipStream_t)stream;
  if (N > 64 * 32) {  // long rows: workgroup per row, exact math (cert / fast: same actions)
    if (top_p > 0.0 && top_p < 1.0) return CO_E_INVAL;
    const dim3 lgrid((unsigned)(B < 65536 ? B : 65536)), lblock(kLongThreads);
    const int opt = (clip > 0.f ? kOptClip : 0) | (temp != 1.f ? kOptTemp : 0);
#define CO_LONG(O)                                                                             \
  hipLaunchKernelGGL(decode_long_kernel<O>, lgrid, lblock, 0, s, B, (int)N, logits, lstride,   \
                     mask, clip, temp, mode, action_in, action_out, logp_sel, full, seed, offset, \
                     status, top_k)
    switch (opt) {
      case 0: CO_LONG(0); break;
      case 1: CO_LONG(1); break;
      case 2: CO_LONG(2); break;
      default: CO_LONG(3);
    }
#undef CO_LONG
    return launch_status();
  }
  const dim3 grid(decode_grid(B, (int)N)), block(256);
  if (grid.x == 0) return CO_E_INVAL;
  const bool filtered = (top_k > 0 && top_k < N) || (top_p > 0.0 && top_p < 1.0);
  if (mode == CO_DECODE_GREEDY && !filtered) {
#define CO_GREEDY(RL, EPL, V)                                                                  \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL, (decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), \
                  grid, block, 0, s, B, (int)N, logits, lstride, mask, clip, temp, action_out,  \
                  logp_sel, full, status)
    switch (greedy_vw(N, lstride, logits, mask, mask, full)) {
      case 4: CO_ROW_DISPATCH(CO_GREEDY, 4); break;
      case 2: CO_GREEDY(CO_RL16, 16 / CO_RL16, 2); break;  // N < 4
      default: CO_ROW_DISPATCH(CO_GREEDY, 3);
    }
#undef CO_GREEDY
    return launch_status();
  }
#define CO_DECODE(RL, EPL, V)                                                                  \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (decode_kernel<RL, EPL, V, OPT>), grid, block, 0, s, B,   \
                  (int)N, logits, lstride, mask, clip, temp, mode, action_in, action_out,      \
                  logp_sel, full, seed, offset, status, top_k, top_p)
  if (decode_vec_ok(logits, lstride, mask, N)) {
    CO_ROW_DISPATCH(CO_DECODE, true);
  } else {
    CO_ROW_DISPATCH(CO_DECODE, false);
  }
#undef CO_DECODE
  return launch_status();
}

extern "C" int co_decode_step(int64_t B, int64_t N, const float* logits, int64_t lstride,
                              const uint8_t* mask, float clip, float temp, int mode,
                              const int64_t* action_in, int64_t* action_out, float* logp_sel,
                              float* full, uint64_t seed, uint64_t offset, int32_t* status,
                              void* stream) {
  return co_decode_step_ex(B, N, logits, lstride, mask, clip, temp, 0, 0.0, mode, action_in,
                           action_out, logp_sel, full, seed, offset, status, stream);
}

// --------------------------------------------------------------------- beam search
// BeamSearch._make_beam_step (decoding.py:611-641) + the feasibility assert of _step
// (:512-524): for instance b, candidate t = s*N + c (beam s, node c) scores
// logp[s*B + b, c] + parent[s*B + b] (f32 add, as the reference's broadcast add); the
// BW best (torch.topk, sorted; equal scores -> lower t) go to rows j*B + b:
// selected = t % N, beam_parent = t / N, beam row = b + beam_parent*B, new parent score.
// One wave per instance: the BW*N scores are staged in LDS, then BW rounds of a wave
// argmax over the untaken ones (a taken bitmap in LDS).
namespace {
__global__ __launch_bounds__(64) void beam_select_kernel(
    int64_t B, int BW, int N, const float* __restrict__ logp, int64_t lstride,
    const float* __restrict__ parent, const uint8_t* __restrict__ mask,
    int64_t* __restrict__ selected, int32_t* __restrict__ beam_parent,
    int64_t* __restrict__ beam_row, float* __restrict__ score_out, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = BW * N;
  float* sc = reinterpret_cast<float*>(smem);
  uint32_t* taken = reinterpret_cast<uint32_t*>(sc + T);
  const int lane = threadIdx.x;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    for (int t = lane; t < T; t += 64) {
      const int s = t / N, c = t - s * N;
      const int64_t r = (int64_t)s * B + b;
      sc[t] = logp[r * lstride + c] + parent[r];
    }
    for (int w = lane; w < (T + 31) / 32; w += 64) taken[w] = 0u;
    __syncthreads();
    bool bad = false;
    for (int j = 0; j < BW; ++j) {
      float bv = -__builtin_inff();
      int bi = 0x7fffffff;
      for (int t = lane; t < T; t += 64) {
        const bool free_t = !((taken[t >> 5] >> (t & 31)) & 1u);
        const float v = sc[t];
        if (free_t && (v > bv || (v == bv && t < bi) || bi == 0x7fffffff)) {
          bv = v;
          bi = t;
        }
      }
      wave_argmax(bv, bi);  // ties -> lower index
      if (bi == 0x7fffffff) bi = 0;
      const int s = bi / N, c = bi - s * N;
      if (lane == 0) {
        taken[bi >> 5] |= 1u << (bi & 31);
        const int64_t row = (int64_t)j * B + b;
        selected[row] = c;
        beam_parent[row] = s;
        beam_row[row] = b + (int64_t)s * B;
        score_out[row] = bv;
        if (mask && !mask[(b + (int64_t)s * B) * N + c]) bad = true;
      }
      __syncthreads();
    }
    if (bad) set_status(status, CO_ST_INFEASIBLE);
    __syncthreads();
  }
}
}  // namespace

extern "C" int co_beam_select(int64_t B, int64_t BW, int64_t N, const float* logp,
                              int64_t lstride, const float* parent, const uint8_t* mask,
                              int64_t* selected, int32_t* beam_parent, int64_t* beam_row,
                              float* score_out, int32_t* status, void* stream) {
  if (B < 0 || BW <= 0 || N <= 0 || BW > N * BW || BW * N > 36 * 1024) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!logp || !parent || !selected || !beam_parent || !beam_row || !score_out ||
      (mask && !status))
    return CO_E_INVAL;
  const int T = (int)(BW * N);
  const size_t shmem = (size_t)T * 4 + (size_t)((T + 31) / 32) * 4;
  if (shmem > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)beam_select_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
  hipLaunchKernelGGL(beam_select_kernel, dim3((unsigned)(B < 65536 ? B : 65536)), dim3(64),
                     shmem, (hipStream_t)stream, B, (int)BW, (int)N, logp, lstride, parent,
                     mask, selected, beam_parent, beam_row, score_out, status);
  return launch_status();
}

