// Diagnostic timing harness (not part of the product): times co_tsp_rollout built with
// CO_DIAG_PHASE = 1 (LDS staging only), 2 (+ step loop), 3 (full kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <numeric>
#include <random>
#include "../include/co_env.h"
extern "C" int diag1_co_tsp_rollout(int64_t, int64_t, const float*, const int64_t*, int64_t*, uint8_t*, int64_t*, int64_t*, int64_t*, uint8_t*, uint8_t*, float*, int, int32_t*, void*);
extern "C" int diag2_co_tsp_rollout(int64_t, int64_t, const float*, const int64_t*, int64_t*, uint8_t*, int64_t*, int64_t*, int64_t*, uint8_t*, uint8_t*, float*, int, int32_t*, void*);
extern "C" int diag3_co_tsp_rollout(int64_t, int64_t, const float*, const int64_t*, int64_t*, uint8_t*, int64_t*, int64_t*, int64_t*, uint8_t*, uint8_t*, float*, int, int32_t*, void*);
typedef int (*fn_t)(int64_t, int64_t, const float*, const int64_t*, int64_t*, uint8_t*, int64_t*, int64_t*, int64_t*, uint8_t*, uint8_t*, float*, int, int32_t*, void*);
int main() {
  for (int64_t B : {65536L, 16384L, 4096L}) for (int64_t N : {100L, 20L}) {
    std::vector<float> locs(B * N * 2); std::mt19937 g(1);
    for (auto& x : locs) x = (g() % 100000) / 100000.f;
    std::vector<int64_t> acts(B * N);  // step-major [N, B]
    std::vector<int> perm(N); 
    for (int64_t b = 0; b < B; ++b) { std::iota(perm.begin(), perm.end(), 0); std::shuffle(perm.begin(), perm.end(), g);
      for (int64_t t = 0; t < N; ++t) acts[t * B + b] = perm[t]; }
    float* dl; int64_t* da; uint8_t *mask, *done, *sr; int64_t *first, *cur, *it; float* rew; int32_t* st;
    hipMalloc(&dl, locs.size() * 4); hipMalloc(&da, acts.size() * 8); hipMalloc(&mask, B * N);
    hipMalloc(&done, B); hipMalloc(&sr, B); hipMalloc(&first, B * 8); hipMalloc(&cur, B * 8); hipMalloc(&it, B * 8);
    hipMalloc(&rew, B * 4); hipMalloc(&st, 4); hipMemset(st, 0, 4);
    hipMemcpy(dl, locs.data(), locs.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(da, acts.data(), acts.size() * 8, hipMemcpyHostToDevice);
    fn_t fns[3] = {diag1_co_tsp_rollout, diag2_co_tsp_rollout, diag3_co_tsp_rollout};
    for (int ph = 0; ph < 3; ++ph) {
      for (int w = 0; w < 3; ++w) fns[ph](B, N, dl, da, nullptr, mask, first, cur, it, done, sr, rew, 1, st, nullptr);
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      const int K = 50;
      hipEventRecord(e0, nullptr);
      for (int k = 0; k < K; ++k) fns[ph](B, N, dl, da, nullptr, mask, first, cur, it, done, sr, rew, 1, st, nullptr);
      hipEventRecord(e1, nullptr); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("B=%ld N=%ld phase=%d  %.2f us/launch\n", (long)B, (long)N, ph + 1, ms * 1000 / K);
    }
    hipFree(dl); hipFree(da); hipFree(mask); hipFree(done); hipFree(sr); hipFree(first); hipFree(cur); hipFree(it); hipFree(rew); hipFree(st);
  }
  return 0;
}
