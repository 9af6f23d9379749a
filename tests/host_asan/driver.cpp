// Sanitizer driver for the host build (csrc/host/co_env_host.cpp), compiled together with
// it under -fsanitize=address,undefined by tests/test_host_asan.py: every entry point on
// exactly-sized heap buffers (so any out-of-bounds index is an ASan report), with the edge
// cases the kernels' indexing must survive -- out-of-range / negative actions, strided
// and step-major action layouts, multistart coordinate rows, in-place and out-of-place
// state, empty batches, N = 1, all-masked / NaN / inf logit rows.  Exit 0 = clean.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../include/co_env.h"

static std::mt19937_64 rng(12345);
static int64_t ri(int64_t lo, int64_t hi) {  // [lo, hi]
  return std::uniform_int_distribution<int64_t>(lo, hi)(rng);
}
static float rf() { return std::uniform_real_distribution<float>(0.f, 1.f)(rng); }

#define CHECK(x)                                                    \
  do {                                                              \
    int rc_ = (x);                                                  \
    if (rc_ != CO_OK) {                                             \
      std::fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
      return 1;                                                     \
    }                                                               \
  } while (0)

static int tsp(int64_t B, int64_t N) {
  std::vector<uint8_t> m0(B * N), m1(B * N);
  std::vector<int64_t> first(B), cur(B), i0(B), i1(B), act(B), f2(B);
  std::vector<float> rw(B);
  std::vector<uint8_t> done(B), srw(B);
  int32_t st = 0, flag = 0;
  CHECK(co_tsp_reset(B, N, m0.data(), first.data(), cur.data(), i0.data(), rw.data(), nullptr));
  std::vector<int64_t> acts(B * N);  // row-major [B, N]
  for (int64_t b = 0; b < B; ++b) {
    std::vector<int64_t> p(N);
    for (int64_t k = 0; k < N; ++k) p[k] = k;
    std::shuffle(p.begin(), p.end(), rng);
    for (int64_t k = 0; k < N; ++k) acts[b * N + k] = p[k];
  }
  for (int64_t t = 0; t < N; ++t) {
    for (int64_t b = 0; b < B; ++b) act[b] = acts[b * N + t];
    if (t == 1 && B > 0) act[0] = N + 7;   // out of range
    if (t == 2 && B > 1) act[1] = -3;
    CHECK(co_any_eq_i64(i0.data(), B, 0, &flag, nullptr));
    const bool inplace = t % 2;
    CHECK(co_tsp_step(B, N, act.data(), m0.data(), inplace ? m0.data() : m1.data(), i0.data(),
                      i1.data(), first.data(), f2.data(), cur.data(), done.data(), srw.data(),
                      2, &flag, &st, nullptr));
    if (!inplace) m0.swap(m1);
    i0.swap(i1);
    first.swap(f2);
  }
  // row-major, step-major and a multistart coordinate batch (LB = B / 2)
  std::vector<float> locs(B * N * 2);
  for (auto& v : locs) v = rf();
  std::vector<int64_t> sm(N * B);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t t = 0; t < N; ++t) sm[t * B + b] = acts[b * N + t];
  if (B > 2) acts[2 * N + 1] = -1;
  const int64_t LB = B > 0 ? B : 1;
  CHECK(co_tsp_reward(B, N, N, locs.data(), LB, acts.data(), N, 1, 1, rw.data(), &st, nullptr));
  CHECK(co_tsp_reward(B, N, N, locs.data(), LB, sm.data(), 1, B, 0, rw.data(), &st, nullptr));
  if (B % 2 == 0 && B > 0)
    CHECK(co_tsp_reward(B, N, N, locs.data(), B / 2, sm.data(), 1, B, 1, rw.data(), &st,
                        nullptr));
  return 0;
}

static int cvrp(int64_t B, int64_t N) {
  const int64_t NC = N + 1;
  std::vector<float> depot(B * 2), lin(B * N * 2), dem(B * N), lout(B * NC * 2), u0(B), u1(B),
      vc(B), rw(B);
  for (auto& v : depot) v = rf();
  for (auto& v : lin) v = rf();
  for (auto& v : dem) v = (float)ri(1, 9) / 20.f;
  std::vector<int64_t> cur(B), act(B);
  std::vector<uint8_t> v0(B * NC), v1(B * NC), mask(B * NC), done(B), srw(B);
  int32_t st = 0, nd = 0;
  CHECK(co_cvrp_reset(B, N, depot.data(), lin.data(), dem.data(), 1.0f, lout.data(), cur.data(),
                      u0.data(), vc.data(), v0.data(), mask.data(), nullptr));
  const int64_t T = 3 * N;
  std::vector<int64_t> acts(B * T);
  for (int64_t t = 0; t < T; ++t) {
    for (int64_t b = 0; b < B; ++b) {
      int64_t a = ri(0, N);
      if (ri(0, 40) == 0) a = ri(0, 1) ? N + 1 + ri(0, 5) : -1 - ri(0, 5);
      act[b] = a;
      acts[b * T + t] = a;
    }
    const bool inplace = t % 3 == 0;
    CHECK(co_cvrp_step(B, N, act.data(), dem.data(), u0.data(), u1.data(), vc.data(), v0.data(),
                       inplace ? v0.data() : v1.data(), cur.data(), done.data(), srw.data(),
                       mask.data(), &st, &nd, nullptr));
    if (!inplace) v0.swap(v1);
    u0.swap(u1);
    CHECK(co_cvrp_action_mask(B, N, dem.data(), u0.data(), vc.data(), v0.data(), cur.data(),
                              mask.data(), nullptr));
  }
  std::vector<int64_t> sm(T * B);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t t = 0; t < T; ++t) sm[t * B + b] = acts[b * T + t];
  CHECK(co_cvrp_reward(B, N, T, lout.data(), acts.data(), T, 1, dem.data(), vc.data(), 1,
                       rw.data(), &st, nullptr));
  CHECK(co_cvrp_reward(B, N, T, lout.data(), sm.data(), 1, B, dem.data(), vc.data(), 0, rw.data(),
                       &st, nullptr));
  return 0;
}

static int slap(int64_t B, int64_t L, int64_t P, int64_t O, int64_t K) {
  std::vector<uint8_t> m0(B * L), m1(B * L), done(B), srw(B), dn(B), tm(B);
  std::vector<float> tc(B * P), rw(B), ratio(B * L), locs(B * L * 2);
  for (auto& v : locs) v = rf();
  std::vector<int64_t> i0(B), i1(B), act(B), pick(B * O * K);
  std::vector<int32_t> a0(B * P, -1), a1(B * P);
  int32_t st = 0;
  CHECK(co_slap_reset(B, L, P, m0.data(), tc.data(), i0.data(), rw.data(), ratio.data(), dn.data(), tm.data(), nullptr));
  for (int64_t t = 0; t < P; ++t) {
    for (int64_t b = 0; b < B; ++b) act[b] = ri(-L - 2, L + 2);  // wraps and out of range
    if (t == 1 && B > 0) tc[0 * P + t] = (float)(P + 3);        // product out of range
    const bool inplace = t % 2;
    CHECK(co_slap_step(B, L, P, act.data(), tc.data() + t, P, a0.data(),
                       inplace ? a0.data() : a1.data(), m0.data(), inplace ? m0.data() : m1.data(),
                       i0.data(), i1.data(), done.data(), srw.data(), &st, nullptr));
    if (!inplace) {
      a0.swap(a1);
      m0.swap(m1);
    }
    i0.swap(i1);
  }
  for (auto& p : pick) p = ri(-P - 2, P + 1);
  CHECK(co_slap_reward(B, L, P, O, K, a0.data(), pick.data(), locs.data(), rw.data(), &st,
                       nullptr));
  return 0;
}

static int gather(int64_t outer, int64_t len, int64_t inner, int64_t m) {
  std::vector<float> src(outer * len * inner), dst(outer * m * inner);
  std::vector<int64_t> idx(outer * m);
  for (auto& j : idx) j = ri(-2, len + 1);
  int32_t st = 0;
  CHECK(co_gather_by_index(src.data(), outer, len, inner * 4, len * inner * 4, inner * 4,
                           idx.data(), m, m, 1, dst.data(), &st, nullptr));
  return 0;
}

static int decode(int64_t B, int64_t N) {
  std::vector<float> lg(B * N), lp(B), full(B * N);
  std::vector<uint8_t> mask(B * N);
  std::vector<int64_t> ain(B), aout(B);
  for (int64_t k = 0; k < B * N; ++k) {
    lg[k] = rf() * 6.f - 3.f;
    mask[k] = ri(0, 3) != 0;
  }
  if (B > 0)
    for (int64_t c = 0; c < N; ++c) mask[c] = 0;  // an all-masked row
  if (B > 1) lg[N] = NAN;
  if (B > 2) lg[2 * N] = INFINITY;
  for (auto& a : ain) a = ri(-1, N);
  int32_t st = 0;
  for (int mode = 0; mode < 3; ++mode)
    for (float clip : {0.f, 10.f})
      for (float temp : {1.f, 0.5f}) {
        CHECK(co_decode_step(B, N, lg.data(), N, mask.data(), clip, temp, mode, ain.data(),
                             aout.data(), lp.data(), full.data(), 99, (uint64_t)mode, &st,
                             nullptr));
        CHECK(co_decode_step(B, N, lg.data(), N, nullptr, clip, temp, mode | CO_DECODE_FAST,
                             ain.data(), aout.data(), lp.data(), nullptr, 7, 1, &st, nullptr));
      }
  return 0;
}

int main() {
  for (int64_t B : {0, 1, 2, 7, 33})
    for (int64_t N : {1, 2, 13, 40})
      if (tsp(B, N) || cvrp(B, N) || decode(B, N)) return 1;
  for (int64_t B : {0, 1, 9})
    if (slap(B, 12, 5, 4, 3) || slap(B, 100, 20, 20, 5)) return 1;
  if (gather(5, 9, 3, 11) || gather(1, 1, 1, 4)) return 1;
  std::printf("host build: all entry points ran clean\n");
  return 0;
}
