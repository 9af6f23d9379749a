// Host (CPU) build of the env step / mask / reward / decode entry points of
// include/co_env.h, for TensorDicts that live on the CPU (BASELINE config 1: the
// reference's CPU TensorDict path, tsp/env.py:95-120 allocating on td.device).
//
// Same C ABI and the same semantics as the gfx950 kernels (every function below cites
// the reference lines it restates; the header documents the contract), plain host
// pointers, the trailing `stream` argument ignored.  Data-dependent failures are OR-ed
// into *status exactly as on the device.  Single-threaded, reentrant, no allocation
// beyond per-call row scratch, no global state.  Built by g++ (rl4co_slap_amd/csrc/
// build.py, -ffp-contract=off, no fast-math); tests/test_host_asan.py rebuilds it with
// -fsanitize=address,undefined and runs its indexing paths.
//
// Decode math is ATen's CPU log_softmax evaluation: SLEEF expf_u10 / logf_u1 (FMA
// variants) and vec::map_reduce_all's 16-lane summation order, the same restatement as
// csrc/co_math.hpp; tanh clipping is the correctly rounded tanh (f64 evaluation, one
// rounding), as on the device.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../../include/co_env.h"

#define CO_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

inline void set_status(int32_t* status, int32_t bits) {
  if (status) *status |= bits;
}

inline float edge_len(float x0, float y0, float x1, float y1) {
  const float dx = x1 - x0, dy = y1 - y0;
  return std::sqrt(dx * dx + dy * dy);  // torch.norm(p=2) over 2 elements, no FMA
}

// ---- SLEEF xexpf (u10, FMA) / xlogf_u1 (FMA), as ATen's vectorised CPU kernels call them
float aten_expf(float d) {
  const float qf = std::nearbyint(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  const int q = (int)qf;
  float s = std::fma(qf, -0.693145751953125f, d);
  s = std::fma(qf, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = std::fma(u, s, 0.00139304355252534151077271f);
  u = std::fma(u, s, 0.00833336077630519866943359f);
  u = std::fma(u, s, 0.0416664853692054748535156f);
  u = std::fma(u, s, 0.166666671633720397949219f);
  u = std::fma(u, s, 0.5f);
  u = 1.0f + std::fma(s * s, u, s);
  u = std::ldexp(u, q);  // one rounding: both halves of SLEEF's vldexp2 are normal
  if (d < -104.f) u = 0.f;
  if (100.f < d) u = INFINITY;
  return u;
}

float aten_logf(float d) {
  const float dd = d * (1.0f / 0.75f);
  uint32_t bits;
  std::memcpy(&bits, &dd, 4);
  const int e = (int)((bits >> 23) & 0xffu) - 127;
  const float m = std::ldexp(d, -e);
  const float ef = (float)e;
  float sx = 0.69314718246459960938f * ef;
  float sy = std::fma(-1.904654323148236017e-09f, ef, std::fma(0.69314718246459960938f, ef, -sx));
  const float nx = -1.0f + m;
  float ny;
  {
    const float v = nx - -1.0f;
    ny = (-1.0f - (nx - v)) + (m - v);
  }
  const float qx = 1.0f + m;
  float qy;
  {
    const float v = qx - 1.0f;
    qy = (1.0f - (qx - v)) + (m - v);
  }
  float xx, xy;
  {
    const float t = 1.0f / qx;
    xx = nx * t;
    const float u = std::fma(t, nx, -xx);
    const float v = std::fma(-qy, t, std::fma(-qx, t, 1.0f));
    xy = std::fma(xx, v, std::fma(ny, t, u));
  }
  const float x2 = xx * xx;
  float t = +0.3027294874e+0f;
  t = std::fma(t, x2, +0.3996108174e+0f);
  t = std::fma(t, x2, +0.6666694880e+0f);
  {
    const float s2 = sx + xx * 2.0f;
    sy = (((sx - s2) + xx * 2.0f) + sy) + xy * 2.0f;
    sx = s2;
  }
  {
    const float w = (x2 * xx) * t;
    const float s2 = sx + w;
    sy = ((sx - s2) + w) + sy;
    sx = s2;
  }
  float r = sx + sy;
  if (d == INFINITY) r = INFINITY;
  if (d < 0.f || d != d) r = NAN;
  if (d == 0.f) r = -INFINITY;
  return r;
}

// correctly rounded tanh (up to f64 double rounding): one rounding of the f64 tanh
float tanh_cr(float x) { return (float)std::tanh((double)x); }

// vec::map_reduce_all's exp-sum order (AVX512: 16 accumulators, then the xor-8/4/2/1
// butterfly); rows narrower than 16 are summed left to right
float aten_row_sum(const float* e, int n) {
  if (n < 16) {
    float s = e[0];
    for (int c = 1; c < n; ++c) s += e[c];
    return s;
  }
  float acc[16];
  for (int r = 0; r < 16; ++r) acc[r] = e[r];
  int c = 16;
  for (; c + 16 <= n; c += 16)
    for (int r = 0; r < 16; ++r) acc[r] += e[c + r];
  for (int r = 0; c + r < n; ++r) acc[r] += e[c + r];  // the tail vector (zero padded)
  for (int h = 8; h >= 1; h >>= 1)
    for (int r = 0; r < h; ++r) acc[r] += acc[r + h];
  return acc[0];
}

// torch.argmax ordering: NaN beats everything, equal values keep the lower index
inline bool argmax_better(float a, int ia, float b, int ib) {
  const bool na = a != a, nb = b != b;
  if (na || nb) return na && (!nb || ia < ib);
  return a > b || (a == b && ia < ib);
}

// Philox-4x32-10 (Salmon et al. 2011), counter (offset, row): the device's draw
uint32_t philox_u32(uint64_t seed, uint64_t offset, uint64_t row) {
  uint32_t c0 = (uint32_t)offset, c1 = (uint32_t)(offset >> 32), c2 = (uint32_t)row,
           c3 = (uint32_t)(row >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
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

}  // namespace

// ---------------------------------------------------------------------------- TSP
// tsp/env.py:95-120
CO_HOST_API int co_tsp_reset(int64_t B, int64_t N, uint8_t* mask, int64_t* first, int64_t* cur,
                             int64_t* i, float* reward, void*) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!mask || !first || !cur || !i || !reward) return CO_E_INVAL;
  std::memset(mask, 1, (size_t)(B * N));
  for (int64_t b = 0; b < B; ++b) {
    first[b] = 0;
    cur[b] = 0;
    i[b] = 0;
    reward[b] = 0.f;
  }
  return CO_OK;
}

// tsp/env.py:67-93
CO_HOST_API int co_tsp_step(int64_t B, int64_t N, const int64_t* action, const uint8_t* mask_in,
                            uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                            const int64_t* first_in, int64_t* first_out, int64_t* current_out,
                            uint8_t* done, uint8_t* reward, int first_mode,
                            const int32_t* first_flag, int32_t* status, void*) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !mask_in || !mask_out || !i_in || !i_out || !first_out || !done || !reward)
    return CO_E_INVAL;
  if (first_mode == 2 && !first_flag) return CO_E_INVAL;
  if (first_mode == 0 && !first_in) return CO_E_INVAL;
  const bool take = first_mode == 1 || (first_mode == 2 && *first_flag != 0);
  for (int64_t b = 0; b < B; ++b) {
    const int64_t a = action[b];
    const uint8_t* mi = mask_in + b * N;
    uint8_t* mo = mask_out + b * N;
    if (mo != mi) std::memcpy(mo, mi, (size_t)N);
    if (a < 0 || a >= N)
      set_status(status, CO_ST_INDEX_RANGE);  // torch.scatter raises; nothing cleared
    else
      mo[a] = 0;
    int64_t left = 0;
    for (int64_t c = 0; c < N; ++c) left += mo[c] != 0;
    const int64_t f = take ? a : first_in[b];
    first_out[b] = f;
    i_out[b] = i_in[b] + 1;
    if (current_out) current_out[b] = a;
    done[b] = left == 0;
    reward[b] = 0;
  }
  return CO_OK;
}

// envs/common/base.py:182-188 + tsp/env.py:157-173 (validity: sorted row == arange(T))
CO_HOST_API int co_tsp_reward(int64_t B, int64_t N, int64_t T, const float* locs, int64_t LB,
                              const int64_t* actions, int64_t sb, int64_t st, int check,
                              float* reward, int32_t* status, void*) {
  if (B < 0 || N <= 0 || T <= 0 || T > (1 << 24)) return CO_E_INVAL;
  if (LB <= 0 || (B > 0 && B % LB != 0)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !actions || !reward || (check && !status)) return CO_E_INVAL;
  std::vector<uint8_t> seen(check ? (size_t)T : 0);
  for (int64_t b = 0; b < B; ++b) {
    const float* lr = locs + (b % LB) * N * 2;
    const int64_t* ar = actions + b * sb;
    bool bad = false;
    if (check) std::fill(seen.begin(), seen.end(), 0);
    double len = 0.0;
    int64_t prev = -1, first = -1;
    for (int64_t t = 0; t < T; ++t) {
      const int64_t a = ar[t * st];
      if (a < 0 || a >= N) {
        set_status(status, CO_ST_INDEX_RANGE);
        bad = true;
        prev = -1;
        continue;
      }
      if (check) {
        if (a >= T || seen[a]) bad = true;
        else seen[a] = 1;
      }
      if (t == 0) first = a;
      if (prev >= 0) len += edge_len(lr[2 * prev], lr[2 * prev + 1], lr[2 * a], lr[2 * a + 1]);
      prev = a;
    }
    if (prev >= 0 && first >= 0)  // closing edge (roll by -1)
      len += edge_len(lr[2 * prev], lr[2 * prev + 1], lr[2 * first], lr[2 * first + 1]);
    reward[b] = -(float)len;
    if (check && bad) set_status(status, CO_ST_INVALID_TOUR);
  }
  return CO_OK;
}

CO_HOST_API int co_any_eq_i64(const int64_t* x, int64_t n, int64_t value, int32_t* flag, void*) {
  if (n < 0 || !flag || (n > 0 && !x)) return CO_E_INVAL;
  int32_t f = 0;
  for (int64_t k = 0; k < n; ++k) f |= x[k] == value;
  *flag = f;
  return CO_OK;
}

// ---------------------------------------------------------------------------- CVRP
namespace {
// cvrp/env.py:137-149: mask_loc = visited[1:] | (demand + used > capacity);
// depot feasible unless (current == 0 and some customer is feasible)
void cvrp_mask_row(int64_t N, const float* dem, float used, float cap, const uint8_t* vis,
                   int64_t cur, uint8_t* mask) {
  bool any = false;
  for (int64_t c = 1; c <= N; ++c) {
    const bool masked = vis[c] != 0 || (dem[c - 1] + used > cap);
    mask[c] = !masked;
    any |= !masked;
  }
  mask[0] = !((cur == 0) && any);
}
}  // namespace

// cvrp/env.py:107-135
CO_HOST_API int co_cvrp_reset(int64_t B, int64_t N, const float* depot, const float* locs_in,
                              const float* demand, float vcap, float* locs_out, int64_t* cur,
                              float* used, float* vcap_out, uint8_t* visited, uint8_t* mask,
                              void*) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!depot || !locs_in || !demand || !locs_out || !cur || !used || !vcap_out || !visited ||
      !mask)
    return CO_E_INVAL;
  for (int64_t b = 0; b < B; ++b) {
    float* lo = locs_out + b * (N + 1) * 2;
    lo[0] = depot[2 * b];
    lo[1] = depot[2 * b + 1];
    std::memcpy(lo + 2, locs_in + b * N * 2, sizeof(float) * 2 * (size_t)N);
    uint8_t* vr = visited + b * (N + 1);
    std::memset(vr, 0, (size_t)(N + 1));
    cur[b] = 0;
    used[b] = 0.f;
    vcap_out[b] = vcap;
    cvrp_mask_row(N, demand + b * N, 0.f, vcap, vr, 0, mask + b * (N + 1));
  }
  return CO_OK;
}

// cvrp/env.py:73-105 (+ get_action_mask)
CO_HOST_API int co_cvrp_step(int64_t B, int64_t N, const int64_t* action, const float* demand,
                             const float* used_in, float* used_out, const float* vcap,
                             const uint8_t* vis_in, uint8_t* vis_out, int64_t* cur_out,
                             uint8_t* done, uint8_t* reward, uint8_t* mask, int32_t* status,
                             int32_t* not_done, void*) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !demand || !used_in || !used_out || !vcap || !vis_in || !vis_out || !done ||
      !reward || !mask)
    return CO_E_INVAL;
  int32_t left_all = 0;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t a = action[b];
    const bool bad = a < 0 || a > N;
    if (bad) set_status(status, CO_ST_INDEX_RANGE);
    const float* dem = demand + b * N;
    int64_t di = a - 1;
    di = di < 0 ? 0 : (di > N - 1 ? N - 1 : di);
    const float u = (used_in[b] + dem[di]) * ((a != 0) ? 1.0f : 0.0f);  // env.py:83-85
    const uint8_t* vi = vis_in + b * (N + 1);
    uint8_t* vo = vis_out + b * (N + 1);
    if (vo != vi) std::memcpy(vo, vi, (size_t)(N + 1));
    if (!bad) vo[a] = 1;
    int64_t vsum = 0;
    for (int64_t c = 0; c <= N; ++c) vsum += vo[c];
    used_out[b] = u;
    if (cur_out) cur_out[b] = a;
    done[b] = vsum == N + 1;
    left_all += vsum != N + 1;
    reward[b] = 0;
    cvrp_mask_row(N, dem, u, vcap[b], vo, a, mask + b * (N + 1));
  }
  if (not_done) *not_done += left_all;
  return CO_OK;
}

CO_HOST_API int co_cvrp_action_mask(int64_t B, int64_t N, const float* demand, const float* used,
                                    const float* vcap, const uint8_t* visited, const int64_t* cur,
                                    uint8_t* mask, void*) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!demand || !used || !vcap || !visited || !cur || !mask) return CO_E_INVAL;
  for (int64_t b = 0; b < B; ++b)
    cvrp_mask_row(N, demand + b * N, used[b], vcap[b], visited + b * (N + 1), cur[b],
                  mask + b * (N + 1));
  return CO_OK;
}

// cvrp/env.py:151-190: reward over [depot] + locs[actions] (closed), validity (sorted tail
// == 1..N, zeros before) and the sequential f32 capacity scan
CO_HOST_API int co_cvrp_reward(int64_t B, int64_t N, int64_t T, const float* locs,
                               const int64_t* actions, int64_t sb, int64_t st,
                               const float* demand, const float* vcap, int check, float* reward,
                               int32_t* status, void*) {
  if (B < 0 || N <= 0 || T <= 0 || T > (1 << 20)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !actions || !reward) return CO_E_INVAL;
  if (check && (!demand || !vcap || !status)) return CO_E_INVAL;
  std::vector<uint8_t> seen(check ? (size_t)(N + 1) : 0);
  for (int64_t b = 0; b < B; ++b) {
    const float* lr = locs + b * (N + 1) * 2;
    const int64_t* ar = actions + b * sb;
    double len = 0.0;
    int64_t prev = 0;  // the depot
    bool prev_ok = true, range = false, bad = false;
    int64_t nonzero = 0;
    if (check) std::fill(seen.begin(), seen.end(), 0);
    for (int64_t t = 0; t < T; ++t) {
      const int64_t a = ar[t * st];
      const bool ok = a >= 0 && a <= N;
      if (!ok) {
        range = true;
        bad = true;
        prev_ok = false;
        continue;
      }
      if (prev_ok)
        len += edge_len(lr[2 * prev], lr[2 * prev + 1], lr[2 * a], lr[2 * a + 1]);
      if (check && a != 0) {
        ++nonzero;
        if (seen[a]) bad = true;
        seen[a] = 1;
      }
      prev = a;
      prev_ok = true;
    }
    if (prev_ok) len += edge_len(lr[2 * prev], lr[2 * prev + 1], lr[0], lr[1]);
    reward[b] = -(float)len;
    if (range) set_status(status, CO_ST_INDEX_RANGE);
    if (!check) continue;
    if (bad || nonzero != N) {
      set_status(status, CO_ST_INVALID_TOUR);
      continue;
    }
    const float cap = vcap[b], lim = cap + 1e-5f;
    float used = 0.f;
    for (int64_t t = 0; t < T; ++t) {
      const int64_t a = ar[t * st];
      used += a == 0 ? -cap : demand[b * N + a - 1];
      if (used < 0.f) used = 0.f;
      if (!(used <= lim)) {
        set_status(status, CO_ST_OVER_CAPACITY);
        break;
      }
    }
  }
  return CO_OK;
}

// ---------------------------------------------------------------------------- SLAP
// slap/env.py:95-129
CO_HOST_API int co_slap_reset(int64_t B, int64_t L, int64_t P, uint8_t* mask, float* to_choose,
                              int64_t* it, float* reward, float* ratio, uint8_t* done,
                              uint8_t* terminated, void*) {
  if (B < 0 || L <= 0 || P <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!mask || !to_choose || !it || !reward) return CO_E_INVAL;
  for (int64_t b = 0; b < B; ++b) {
    for (int64_t l = 0; l < L; ++l) mask[b * L + l] = l != 0;
    for (int64_t p = 0; p < P; ++p) to_choose[b * P + p] = (float)p;
    if (ratio)
      for (int64_t l = 0; l < L; ++l) ratio[b * L + l] = 0.f;
    it[b] = 0;
    reward[b] = 0.f;
    if (done) done[b] = 0;
    if (terminated) terminated[b] = 0;
  }
  return CO_OK;
}

// slap/env.py:38-93 (negative indices wrap like python advanced indexing)
CO_HOST_API int co_slap_step(int64_t B, int64_t L, int64_t P, const int64_t* action,
                             const float* to_choose, int64_t tc_stride, const int32_t* assign_in,
                             int32_t* assign_out, const uint8_t* mask_in, uint8_t* mask_out,
                             const int64_t* i_in, int64_t* i_out, uint8_t* done, uint8_t* reward,
                             int32_t* status, void*) {
  if (B < 0 || L <= 0 || P <= 0 || L > (1 << 30)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !assign_in || !assign_out || !mask_in || !mask_out || !i_in || !i_out ||
      !done || !reward || (!to_choose && (tc_stride < 0 || tc_stride >= P)))
    return CO_E_INVAL;
  for (int64_t b = 0; b < B; ++b) {
    if (assign_out != assign_in)
      std::memcpy(assign_out + b * P, assign_in + b * P, sizeof(int32_t) * (size_t)P);
    if (mask_out != mask_in) std::memcpy(mask_out + b * L, mask_in + b * L, (size_t)L);
    int64_t a = action[b];
    if (a < 0) a += L;
    if (a < 0 || a >= L)
      set_status(status, CO_ST_INDEX_RANGE);
    else
      mask_out[b * L + a] = 0;
    // .to(torch.int), env.py:52; to_choose NULL: the uniform product tc_stride
    int64_t p = to_choose ? (int64_t)(int)to_choose[b * tc_stride] : tc_stride;
    if (p < 0) p += P;
    if (p < 0 || p >= P)
      set_status(status, CO_ST_INDEX_RANGE);
    else
      assign_out[b * P + p] = (int32_t)action[b];  // env.py:53-54
    done[b] = i_in[b] == P - 1;
    i_out[b] = i_in[b] + 1;
    reward[b] = 0;
  }
  return CO_OK;
}

// slap/env.py:131-143: orders added one by one in f32, each a closed tour in pick order
CO_HOST_API int co_slap_reward(int64_t B, int64_t L, int64_t P, int64_t O, int64_t K,
                               const int32_t* assignment, const int64_t* picklist,
                               const float* locs, float* reward, int32_t* status, void*) {
  if (B < 0 || L <= 0 || P <= 0 || O <= 0 || K <= 0 || O * K > (1 << 16)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!assignment || !picklist || !locs || !reward) return CO_E_INVAL;
  std::vector<int64_t> loc((size_t)K);
  for (int64_t b = 0; b < B; ++b) {
    const float* lr = locs + b * L * 2;
    float total = 0.f;
    for (int64_t o = 0; o < O; ++o) {
      for (int64_t k = 0; k < K; ++k) {
        int64_t p = picklist[(b * O + o) * K + k];
        if (p < 0) p += P;
        int64_t l = 0;
        if (p < 0 || p >= P) {
          set_status(status, CO_ST_INDEX_RANGE);
        } else {
          l = assignment[b * P + p];
          if (l < 0) l += L;  // the -1 of an unassigned product wraps
          if (l < 0 || l >= L) {
            set_status(status, CO_ST_INDEX_RANGE);
            l = 0;
          }
        }
        loc[(size_t)k] = l;
      }
      float len = 0.f;
      for (int64_t k = 0; k < K; ++k) {
        const int64_t p0 = loc[(size_t)k], p1 = loc[(size_t)((k + 1) % K)];
        len += edge_len(lr[2 * p0], lr[2 * p0 + 1], lr[2 * p1], lr[2 * p1 + 1]);
      }
      total += -len;
    }
    reward[b] = total;
  }
  return CO_OK;
}

// ---------------------------------------------------------------------------- ops
// utils/ops.py:65-77
CO_HOST_API int co_gather_by_index(const void* src, int64_t outer, int64_t src_len,
                                   int64_t inner_bytes, int64_t src_stride_outer,
                                   int64_t src_stride_len, const int64_t* idx, int64_t idx_len,
                                   int64_t idx_stride_outer, int64_t idx_stride_len, void* dst,
                                   int32_t* status, void*) {
  if (outer < 0 || src_len < 0 || inner_bytes <= 0 || idx_len < 0) return CO_E_INVAL;
  if (outer == 0 || idx_len == 0) return CO_OK;
  if (!src || !idx || !dst) return CO_E_INVAL;
  const unsigned char* s = static_cast<const unsigned char*>(src);
  unsigned char* d = static_cast<unsigned char*>(dst);
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t m = 0; m < idx_len; ++m) {
      const int64_t j = idx[o * idx_stride_outer + m * idx_stride_len];
      unsigned char* out = d + (o * idx_len + m) * inner_bytes;
      if (j < 0 || j >= src_len) {
        set_status(status, CO_ST_INDEX_RANGE);
        std::memset(out, 0, (size_t)inner_bytes);
      } else {
        std::memcpy(out, s + o * src_stride_outer + j * src_stride_len, (size_t)inner_bytes);
      }
    }
  return CO_OK;
}

// ---------------------------------------------------------------------------- decode
// decoding.py:141-191 (tanh clip -> mask -> /T -> log_softmax), 327-399 (greedy argmax,
// sampling by inverse CDF of a Philox draw keyed by (seed, offset, row), evaluate)
CO_HOST_API int co_decode_step(int64_t B, int64_t N, const float* logits, int64_t stride,
                               const uint8_t* mask, float clip, float temp, int mode,
                               const int64_t* action_in, int64_t* action_out, float* logp_sel,
                               float* logp_full, uint64_t seed, uint64_t offset, int32_t* status,
                               void*) {
  // the host path is always exact: the fast / certified math flags select nothing here
  mode &= ~(CO_DECODE_FAST | CO_DECODE_CERTIFIED);
  if (B < 0 || N <= 0 || mode < 0 || mode > 2) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!logits || !action_out || !logp_sel) return CO_E_INVAL;
  if (mode == CO_DECODE_EVALUATE && !action_in) return CO_E_INVAL;
  std::vector<float> x((size_t)N), e((size_t)N);
  for (int64_t b = 0; b < B; ++b) {
    const float* lr = logits + b * stride;
    float m = -INFINITY;
    for (int64_t c = 0; c < N; ++c) {
      float v = lr[c];
      if (clip > 0.f) v = tanh_cr(v) * clip;
      if (mask && !mask[b * N + c]) v = -INFINITY;
      if (temp != 1.f) v = v / temp;
      x[(size_t)c] = v;
      m = std::fmax(m, v);  // as the device (fmaxf): a NaN logit makes every logp NaN anyway
    }
    for (int64_t c = 0; c < N; ++c) {
      x[(size_t)c] = x[(size_t)c] - m;
      e[(size_t)c] = aten_expf(x[(size_t)c]);
    }
    const float Lg = aten_logf(aten_row_sum(e.data(), (int)N));
    for (int64_t c = 0; c < N; ++c) x[(size_t)c] = x[(size_t)c] - Lg;  // (x - m) - L
    int64_t sel = 0;
    if (mode == CO_DECODE_GREEDY) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = 0; c < (int)N; ++c)
        if (argmax_better(x[(size_t)c], c, bv, bi)) {
          bv = x[(size_t)c];
          bi = c;
        }
      sel = bi == 0x7fffffff ? 0 : bi;
    } else if (mode == CO_DECODE_SAMPLING) {
      const uint32_t r = philox_u32(seed, offset, (uint64_t)b);
      const float u = (float)(r >> 8) * (1.0f / 16777216.0f);
      float total = 0.f;
      for (int64_t c = 0; c < N; ++c) total += std::exp(x[(size_t)c]);
      const float target = u * total;
      float run = 0.f;
      int64_t hit = -1, last = -1;
      for (int64_t c = 0; c < N; ++c) {
        const float p = std::exp(x[(size_t)c]);
        run += p;
        if (p > 0.f) {
          last = c;
          if (run > target && hit < 0) hit = c;
        }
      }
      sel = hit >= 0 ? hit : (last >= 0 ? last : 0);
    } else {
      const int64_t a = action_in[b];
      if (a < 0 || a >= N) set_status(status, CO_ST_INDEX_RANGE);
      sel = (a < 0 || a >= N) ? 0 : a;
    }
    action_out[b] = mode == CO_DECODE_EVALUATE ? action_in[b] : sel;
    logp_sel[b] = x[(size_t)sel];
    if (logp_full) std::memcpy(logp_full + b * N, x.data(), sizeof(float) * (size_t)N);
    if (mode != CO_DECODE_EVALUATE && mask && !mask[b * N + sel])
      set_status(status, CO_ST_INFEASIBLE);
  }
  return CO_OK;
}

CO_HOST_API const char* co_build_info(void) {
  return "rl4co_slap_amd co_env: host (CPU) build of the env / decode entry points";
}
