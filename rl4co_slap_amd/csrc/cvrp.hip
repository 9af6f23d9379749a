// CVRP env kernels for gfx950: reset (+mask), fused step + get_action_mask,
// stand-alone mask, episode reward with the validity/capacity check, and the
// nearest-feasible bench policy.
//
// Step layout: one wavefront per instance (grid-stride), lanes over the N+1
// columns: visited update, capacity test `demand + used > capacity` (strict, f32,
// no contraction), visited-sum and any-feasible-customer are wave reductions
// (ballot / shuffle).  The capacity arithmetic follows cvrp/env.py:83-85 exactly:
// used = (used + d) * float(a != 0).
#include "co_common.hpp"

using namespace co;

namespace {

// Writes visited_out (optional update at column `a`), the action mask and returns
// the visited sum for the row.  `a` < 0 means no visited update (reset / mask).
__device__ __forceinline__ int cvrp_row(int N, const float* dem, float used, float cap,
                                        const uint8_t* vis_in, uint8_t* vis_out, int64_t a,
                                        int64_t cur, uint8_t* mask) {
  const int lane = lane_id();
  int vsum = 0;
  bool any_feas = false;
  for (int c = lane; c <= N; c += 64) {
    uint8_t v = vis_in[c];
    if (c == a) v = 1;
    if (vis_out) vis_out[c] = v;
    vsum += v;
    if (c >= 1) {
      const bool exceeds = dem[c - 1] + used > cap;
      const bool masked = (v != 0) || exceeds;
      mask[c] = !masked;
      any_feas |= !masked;
    }
  }
  vsum = wave_sum(vsum);
  const bool anyf = __any(any_feas);
  if (lane == 0) mask[0] = !((cur == 0) && anyf);
  return vsum;
}

__global__ __launch_bounds__(256) void cvrp_reset_kernel(int64_t B, int N, const float2* depot,
                                                         const float2* locs_in,
                                                         const float* demand, float vcap,
                                                         float2* locs_out, int64_t* cur,
                                                         float* used, float* vcap_out,
                                                         uint8_t* visited, uint8_t* mask) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    float2* lo = locs_out + b * (N + 1);
    const float2* li = locs_in + b * (int64_t)N;
    for (int c = lane; c <= N; c += 64) lo[c] = (c == 0) ? depot[b] : li[c - 1];
    uint8_t* vrow = visited + b * (N + 1);
    for (int c = lane; c <= N; c += 64) vrow[c] = 0;
    if (lane == 0) {
      cur[b] = 0;
      used[b] = 0.f;
      vcap_out[b] = vcap;
    }
    // mask from the fresh state: visited == 0, used == 0, current == 0
    const float* dem = demand + b * (int64_t)N;
    uint8_t* mrow = mask + b * (N + 1);
    bool any_feas = false;
    for (int c = lane + 1; c <= N; c += 64) {
      const bool masked = dem[c - 1] + 0.f > vcap;
      mrow[c] = !masked;
      any_feas |= !masked;
    }
    const bool anyf = __any(any_feas);
    if (lane == 0) mrow[0] = !anyf;
  }
}

__global__ __launch_bounds__(256) void cvrp_step_kernel(
    int64_t B, int N, const int64_t* action, const float* demand, const float* used_in,
    float* used_out, const float* vcap, const uint8_t* vis_in, uint8_t* vis_out, int64_t* cur_out,
    uint8_t* done, uint8_t* reward, uint8_t* mask, int32_t* status) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const int64_t a = action[b];
    const bool bad = a < 0 || a > N;
    if (bad && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    const float* dem = demand + b * (int64_t)N;
    int64_t di = a - 1;
    di = di < 0 ? 0 : (di > N - 1 ? N - 1 : di);
    const float d = dem[di];
    const float u = (used_in[b] + d) * ((a != 0) ? 1.0f : 0.0f);
    const float cap = vcap[b];
    const int vsum = cvrp_row(N, dem, u, cap, vis_in + b * (N + 1), vis_out + b * (N + 1),
                              bad ? -1 : a, a, mask + b * (N + 1));
    if (lane == 0) {
      used_out[b] = u;
      if (cur_out) cur_out[b] = a;
      done[b] = vsum == N + 1;
      reward[b] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void cvrp_mask_kernel(int64_t B, int N, const float* demand,
                                                        const float* used, const float* vcap,
                                                        const uint8_t* visited,
                                                        const int64_t* cur, uint8_t* mask) {
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    cvrp_row(N, demand + b * (int64_t)N, used[b], vcap[b], visited + b * (N + 1), nullptr, -1,
             cur[b], mask + b * (N + 1));
  }
}

// Reward: ordered = [depot] + locs[actions] (T+1 points, closed tour).
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void cvrp_reward_kernel(
    int64_t B, int N, int T, const float2* locs, const int64_t* actions, int64_t sb, int64_t st,
    const float* demand, const float* vcap, int check, float* reward, int32_t* status) {
  extern __shared__ uint32_t s_mem[];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int words = (N + 32) >> 5;  // bits for values 0..N
  uint32_t* bits = s_mem + w * (words + T);
  float* dseq = reinterpret_cast<float*>(bits + words);
  for (int64_t b = (int64_t)blockIdx.x * WAVES + w; b < B; b += (int64_t)gridDim.x * WAVES) {
    const int64_t* arow = actions + b * sb;
    const float2* lrow = locs + b * (int64_t)(N + 1);
    if (check) {
      for (int k = lane; k < words; k += 64) bits[k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const float cap = check ? vcap[b] : 0.f;
    double acc = 0.0;
    bool bad = false, range = false;
    int nonzero = 0;
    const int M = T + 1;
    for (int m = lane; m < M; m += 64) {
      const int64_t a_from = (m == 0) ? 0 : arow[(int64_t)(m - 1) * st];
      const int64_t a_to = (m + 1 == M) ? 0 : arow[(int64_t)m * st];
      if (a_from < 0 || a_from > N || a_to < 0 || a_to > N) {
        range = true;
      } else {
        const float2 p = lrow[a_from], q = lrow[a_to];
        acc += (double)edge_len(p.x, p.y, q.x, q.y);
      }
      if (check && m < T) {
        const int64_t a = a_to;  // = actions[m]
        if (a < 0 || a > N) {
          bad = true;
          dseq[m] = 0.f;
        } else {
          if (a != 0) {
            ++nonzero;
            const uint32_t bit = 1u << (a & 31);
            if (atomicOr(&bits[a >> 5], bit) & bit) bad = true;
          }
          dseq[m] = (a == 0) ? -cap : demand[b * (int64_t)N + a - 1];
        }
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) reward[b] = -(float)acc;
    if (__any(range) && lane == 0) set_status(status, CO_ST_INDEX_RANGE);
    if (check) {
      nonzero = wave_sum(nonzero);
      const bool invalid = __any(bad) || nonzero != N;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        if (invalid) {
          set_status(status, CO_ST_INVALID_TOUR);
        } else {
          // cvrp/env.py:181-190, sequential f32 scan
          const float lim = cap + 1e-5f;
          float used = 0.f;
          bool over = false;
          for (int t = 0; t < T; ++t) {
            used += dseq[t];
            if (used < 0.f) used = 0.f;
            if (!(used <= lim)) over = true;
          }
          if (over) set_status(status, CO_ST_OVER_CAPACITY);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void cvrp_nearest_kernel(int64_t B, int N, const float2* locs,
                                                           const uint8_t* mask,
                                                           const int64_t* cur, int64_t* out) {
  const int lane = lane_id();
  const int64_t wpb = blockDim.x >> 6;
  for (int64_t b = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); b < B;
       b += (int64_t)gridDim.x * wpb) {
    const float2* lrow = locs + b * (int64_t)(N + 1);
    const uint8_t* mrow = mask + b * (int64_t)(N + 1);
    int64_t c0 = cur[b];
    c0 = (c0 < 0 || c0 > N) ? 0 : c0;
    const float2 p = lrow[c0];
    float best = __builtin_inff();
    int bi = 0x7fffffff;
    bool any = false;
    for (int c = lane + 1; c <= N; c += 64) {
      if (mrow[c]) {
        any = true;
        const float2 q = lrow[c];
        const float d = edge_len(p.x, p.y, q.x, q.y);
        if (d < best || (d == best && c < bi)) { best = d; bi = c; }
      }
    }
    wave_argmin(best, bi);
    const bool anyf = __any(any);
    if (lane == 0) out[b] = anyf ? bi : 0;
  }
}

}  // namespace

extern "C" int co_cvrp_reset(int64_t B, int64_t N, const float* depot, const float* locs_in,
                             const float* demand, float vcap, float* locs_out, int64_t* cur,
                             float* used, float* vcap_out, uint8_t* visited, uint8_t* mask,
                             void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!depot || !locs_in || !demand || !locs_out || !cur || !used || !vcap_out || !visited ||
      !mask)
    return CO_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(depot) | reinterpret_cast<uintptr_t>(locs_in) |
       reinterpret_cast<uintptr_t>(locs_out)) & 7)
    return CO_E_ALIGN;
  hipLaunchKernelGGL(cvrp_reset_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, reinterpret_cast<const float2*>(depot),
                     reinterpret_cast<const float2*>(locs_in), demand, vcap,
                     reinterpret_cast<float2*>(locs_out), cur, used, vcap_out, visited, mask);
  return launch_status();
}

extern "C" int co_cvrp_step(int64_t B, int64_t N, const int64_t* action, const float* demand,
                            const float* used_in, float* used_out, const float* vcap,
                            const uint8_t* vis_in, uint8_t* vis_out, int64_t* cur_out,
                            uint8_t* done, uint8_t* reward, uint8_t* mask, int32_t* status,
                            void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!action || !demand || !used_in || !used_out || !vcap || !vis_in || !vis_out || !done ||
      !reward || !mask)
    return CO_E_INVAL;
  hipLaunchKernelGGL(cvrp_step_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, action, demand, used_in, used_out, vcap,
                     vis_in, vis_out, cur_out, done, reward, mask, status);
  return launch_status();
}

extern "C" int co_cvrp_action_mask(int64_t B, int64_t N, const float* demand, const float* used,
                                   const float* vcap, const uint8_t* visited, const int64_t* cur,
                                   uint8_t* mask, void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!demand || !used || !vcap || !visited || !cur || !mask) return CO_E_INVAL;
  hipLaunchKernelGGL(cvrp_mask_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, demand, used, vcap, visited, cur, mask);
  return launch_status();
}

extern "C" int co_cvrp_reward(int64_t B, int64_t N, int64_t T, const float* locs,
                              const int64_t* actions, int64_t sb, int64_t st,
                              const float* demand, const float* vcap, int check, float* reward,
                              int32_t* status, void* stream) {
  if (B < 0 || N <= 0 || T <= 0 || T > (1 << 20)) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !actions || !reward) return CO_E_INVAL;
  if (check && (!demand || !vcap || !status)) return CO_E_INVAL;
  if (reinterpret_cast<uintptr_t>(locs) & 7) return CO_E_ALIGN;
  const size_t per_wave = check ? (size_t)((N + 32) / 32 + T) * 4 : 0;
  int waves = 4;
  while (waves > 1 && per_wave * waves > 64 * 1024) waves >>= 1;
  if (per_wave > 64 * 1024) return CO_E_INVAL;
  const size_t shmem = per_wave * waves;
  const dim3 grid(grid_for(B, waves, 256 * 32));
  const float2* l2 = reinterpret_cast<const float2*>(locs);
  switch (waves) {
    case 4:
      hipLaunchKernelGGL(cvrp_reward_kernel<4>, grid, dim3(256), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
    case 2:
      hipLaunchKernelGGL(cvrp_reward_kernel<2>, grid, dim3(128), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
      break;
    default:
      hipLaunchKernelGGL(cvrp_reward_kernel<1>, grid, dim3(64), shmem, (hipStream_t)stream, B,
                         (int)N, (int)T, l2, actions, sb, st, demand, vcap, check, reward,
                         status);
  }
  return launch_status();
}

extern "C" int co_cvrp_nearest_action(int64_t B, int64_t N, const float* locs,
                                      const uint8_t* mask, const int64_t* cur, int64_t* out,
                                      void* stream) {
  if (B < 0 || N <= 0) return CO_E_INVAL;
  if (B == 0) return CO_OK;
  if (!locs || !mask || !cur || !out) return CO_E_INVAL;
  hipLaunchKernelGGL(cvrp_nearest_kernel, dim3(grid_for(B, 4, 256 * 32)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)N, reinterpret_cast<const float2*>(locs), mask,
                     cur, out);
  return launch_status();
}
