// co_tsp_decode_step: the decode step fused with TSPEnv._step (decode_common.hpp engines).
#include "decode_common.hpp"

#ifndef CO_DECODE_STAGE
#define CO_DECODE_STAGE 0  // rows by non-temporal LDS-DMA (r06: TSP decode 16.0 -> 17.9 us: off)
#endif

extern "C" int co_tsp_decode_step(int64_t B, int64_t N, const float* logits, int64_t lstride,
                                  const uint8_t* mask_in, float clip, float temp, int mode,
                                  const int64_t* action_in, int64_t* action_out,
                                  float* logp_sel, uint64_t seed, uint64_t offset,
                                  uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                                  const int64_t* first_in, int64_t* first_out, int first_mode,
                                  uint8_t* done, uint8_t* step_reward, float* ll_accum,
                                  int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || N > 64 * 32) return CO_E_INVAL;
  const bool cert = (mode & CO_DECODE_CERTIFIED) != 0 && (mode & CO_DECODE_FAST) == 0;
  const bool fast = (mode & CO_DECODE_FAST) != 0;
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (mode < 0 || mode > 2 || first_mode < 0 || first_mode > 1) return CO_E_MODE;
  if (B == 0) return CO_OK;
  if (!logits || !mask_in || !action_out || !mask_out || !i_in || !i_out || !first_out ||
      !done || !step_reward || (first_mode == 0 && !first_in) ||
      (mode == CO_DECODE_EVALUATE && !action_in))
    return CO_E_INVAL;
  hipStream_t s = (hipStream_t)stream;
  if (mode == CO_DECODE_GREEDY) {
    const dim3 grid(decode_grid(B, (int)N)), block(256);
    if (grid.x == 0) return CO_E_INVAL;
    // the row-group width of 64 < N <= 128 with contiguous, 16-byte aligned rows: the
    // logits and mask rows by non-temporal LDS-DMA (tsp_decode_greedy_kernel STAGE)
    if (CO_DECODE_STAGE && N > 64 && N <= 128 && N % 4 == 0 && lstride == N &&
        greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr) == 4 &&
        ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(mask_in)) & 15) == 0) {
      const size_t dsh = 4 * tsp_dstage_bytes(64 / CO_RL128, (int)N);
      CO_OPT_DISPATCH_G(hipLaunchKernelGGL,
                        (tsp_decode_greedy_kernel<CO_RL128, 128 / CO_RL128, 4, OPT, true>), grid,
                        block, dsh, s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out,
                        logp_sel, mask_out, i_in, i_out, first_in, first_out, first_mode, done,
                        step_reward, ll_accum, status);
      return launch_status();
    }
#define CO_TDG(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH_G(hipLaunchKernelGGL,                                                        \
                    (tsp_decode_greedy_kernel<RL, (EPL < 4 ? 4 : EPL), V, OPT>), grid, block, 0, \
                  s, B, (int)N, logits, lstride, mask_in, clip, temp, action_out, logp_sel,     \
                  mask_out, i_in, i_out, first_in, first_out, first_mode, done, step_reward,    \
                  ll_accum, status)
    switch (greedy_vw(N, lstride, logits, mask_in, mask_out, nullptr)) {
      case 4: CO_ROW_DISPATCH(CO_TDG, 4); break;
      case 2: CO_TDG(CO_RL16, 16 / CO_RL16, 2); break;  // N < 4
      default: CO_ROW_DISPATCH(CO_TDG, 3);
    }
#undef CO_TDG
    return launch_status();
  }
  const dim3 grid(decode_grid(B, (int)N, CO_DECODE_UNR)), block(256);
  if (grid.x == 0) return CO_E_INVAL;
#define CO_TDS(RL, EPL, V)                                                                     \
  CO_OPT_DISPATCH(hipLaunchKernelGGL, (tsp_decode_step_kernel<RL, EPL, V, OPT>), grid, block,   \
                  0, s, B, (int)N, logits, lstride, mask_in, clip, temp, mode, action_in,       \
                  action_out, logp_sel, seed, offset, mask_out, i_in, i_out, first_in,         \
                  first_out, first_mode, done, step_reward, ll_accum, status)
  if (decode_vec_ok(logits, lstride, mask_in, N) &&
      (reinterpret_cast<uintptr_t>(mask_out) & 3) == 0) {
    CO_ROW_DISPATCH(CO_TDS, true);
  } else {
    CO_ROW_DISPATCH(CO_TDS, false);
  }
#undef CO_TDS
  return launch_status();
}
