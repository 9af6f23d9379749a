/*
 * co_env.h -- C ABI of the MI355X (gfx950) batched CO-environment engine.
 *
 * Drop-in boundary for the rl4co-slap hot path: the per-step env functions of
 * TSP / CVRP / SLAP, the episode-end rewards + validity checks, the fused
 * decode step and utils.ops.gather_by_index.  Each entry point replaces the
 * ATen op sequence the reference issues at the cited file:line of
 * j4n1k/rl4co-slap (reference @ 2025-02-02).
 *
 * Conventions (all entry points):
 *  - plain device pointers + sizes; no torch / HIP types in the signatures;
 *    `stream` is a hipStream_t passed as void* (NULL = default stream);
 *  - every call is stream-ordered and asynchronous: no allocation, no host
 *    synchronisation, graph-capturable; the library never owns user memory;
 *  - the caller allocates every output; outputs may alias their matching input
 *    only where a parameter comment says so ("in-place allowed");
 *  - return 0 on success, CO_E_* (< 0) for invalid arguments, or the positive
 *    hipError_t of a failed launch.  Nothing throws across the ABI;
 *  - data-dependent failures (invalid tour, capacity overflow, infeasible or
 *    out-of-range index) are OR-ed into a caller-provided device word
 *    `status` (bits CO_ST_*); the host maps them to the reference's
 *    AssertionError / IndexError messages;
 *  - dtypes are the reference TensorDict dtypes: bool/uint8 masks as bytes,
 *    int64 indices, float32 coordinates/demands/rewards, int32 assignment.
 */
#ifndef CO_ENV_H
#define CO_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CO_OK 0
#define CO_E_INVAL (-1)     /* bad size / null pointer */
#define CO_E_ALIGN (-2)     /* pointer misaligned for its dtype */
#define CO_E_MODE (-3)      /* unknown mode */

/* status bits (device int32, OR-ed atomically) */
#define CO_ST_INVALID_TOUR 1      /* "Invalid tour"              tsp/env.py:173, cvrp/env.py:175 */
#define CO_ST_OVER_CAPACITY 2     /* "Used more than capacity"   cvrp/env.py:188-190 */
#define CO_ST_INFEASIBLE 4        /* "infeasible action selected" decoding.py:376-379 */
#define CO_ST_INDEX_RANGE 8       /* index out of range (torch raises IndexError/RuntimeError) */
#define CO_ST_TRUNCATED 16        /* an episode hit max_steps before done (rollout max_steps) */
#define CO_ST_LOGP_NEG_INF 32     /* "Logprobs should not be -inf, ..."  decoding.py:57-58 */

/* Library identification: returns the gfx target string compiled in. */
const char* co_build_info(void);

/* ------------------------------------------------------------------ TSP */

/* TSPEnv._reset (rl4co/envs/routing/tsp/env.py:95-120):
 * action_mask[B,N] = 1, first_node[B] = current_node[B] = 0, i[B,1] = 0,
 * reward[B,1] = 0.  first_node and current_node may be the same buffer
 * (the reference aliases them). */
int co_tsp_reset(int64_t batch, int64_t num_loc, uint8_t* action_mask, int64_t* first_node,
                 int64_t* current_node, int64_t* i, float* reward, void* stream);

/* TSPEnv._step (tsp/env.py:67-93):
 *   first_out = (first_mode says the batch has an i == 0) ? action : first_in
 *   mask_out  = mask_in with mask_out[b, action[b]] = 0       (in-place allowed)
 *   done[b]   = sum(mask_out[b]) == 0 ; reward[b] = 0 (bool)
 *   i_out     = i_in + 1 (in-place allowed); current_out = action (may be NULL)
 * first_mode: 0 = keep first_in, 1 = take action, 2 = read *first_flag (device
 * int32, nonzero = take action; produced by co_any_eq_i64).  This is the
 * batch-wide `td["i"].all() == 0` test of tsp/env.py:70. */
int co_tsp_step(int64_t batch, int64_t num_loc, const int64_t* action, const uint8_t* mask_in,
                uint8_t* mask_out, const int64_t* i_in, int64_t* i_out, const int64_t* first_in,
                int64_t* first_out, int64_t* current_out, uint8_t* done, uint8_t* reward,
                int first_mode, const int32_t* first_flag, int32_t* status, void* stream);

/* K consecutive TSPEnv._step calls (tsp/env.py:67-93) in one launch (round 6): exactly the
 * K co_tsp_step launches t = 0..K-1 with action row t at action + t*act_stride and the
 * state ping-ponging between buffers A and B (step t reads A and writes B for even t, the
 * reverse for odd t; current_out / done / reward written by every step), so every step's
 * state is stored as its own launch would store it and the final contents are
 * bit-identical.  first_mode (step 0 only): 0 = keep first_a, 1 = take action (the
 * episode's first step).  Rows the lane-group kernel does not take (N % 4 != 0, tiny N)
 * run as the K single-step launches.  Replaces K env.step() calls of a loop whose actions
 * are known in advance (teacher forcing, the stepwise engine). */
int co_tsp_steps(int64_t batch, int64_t num_loc, int64_t steps, const int64_t* action,
                 int64_t act_stride, uint8_t* mask_a, int64_t* i_a, int64_t* first_a,
                 uint8_t* mask_b, int64_t* i_b, int64_t* first_b, int64_t* current_out,
                 uint8_t* done, uint8_t* reward, int first_mode, int32_t* status, void* stream);

/* TSPEnv.get_reward (envs/common/base.py:182-188 + tsp/env.py:157-173):
 * reward[b] = -closed tour length of locs[b % locs_batch, actions[b, 0..T-1]]
 * (locs_batch = batch normally; = instances for the POMO [S, B] multistart layout,
 * which then reads each instance's coordinates without batchify's copy, ops.py:16).
 * actions element (b, t) lives at actions[b*act_stride_b + t*act_stride_t].
 * check != 0: a row that is not a permutation of 0..T-1 sets CO_ST_INVALID_TOUR
 * (the reference's sort(1) == arange(T) test). */
int co_tsp_reward(int64_t batch, int64_t num_loc, int64_t steps, const float* locs,
                  int64_t locs_batch, const int64_t* actions, int64_t act_stride_b, int64_t act_stride_t, int check,
                  float* reward, int32_t* status, void* stream);

/* ----------------------------------------------------------------- CVRP */

/* CVRPEnv._reset + get_action_mask (cvrp/env.py:107-149).  N = customers.
 * locs_out[B,N+1,2] = cat(depot[B,2], locs_in[B,N,2]); current_node[B,1] = 0;
 * used_capacity[B,1] = 0; vehicle_capacity_out[B,1] = vehicle_capacity;
 * visited[B,N+1] = 0; action_mask[B,N+1] per get_action_mask. */
int co_cvrp_reset(int64_t batch, int64_t num_loc, const float* depot, const float* locs_in,
                  const float* demand, float vehicle_capacity, float* locs_out,
                  int64_t* current_node, float* used_capacity, float* vehicle_capacity_out,
                  uint8_t* visited, uint8_t* action_mask, void* stream);

/* CVRPEnv._step fused with get_action_mask (cvrp/env.py:73-105,137-149):
 *   d = demand[b, clamp(a-1, 0, N-1)]; used_out = (used_in + d) * (a != 0)
 *   visited_out = visited_in with [a] = 1 (in-place allowed); current_out = a
 *   done = sum(visited_out) == N+1 ; reward = 0 (bool); action_mask recomputed.
 * not_done (optional) is atomically incremented by the number of rows not done
 * (the `while not td["done"].all()` poll of constructive/base.py:245 without a second
 * pass over `done`); the caller zeroes it. */
int co_cvrp_step(int64_t batch, int64_t num_loc, const int64_t* action, const float* demand,
                 const float* used_in, float* used_out, const float* vehicle_capacity,
                 const uint8_t* visited_in, uint8_t* visited_out, int64_t* current_out,
                 uint8_t* done, uint8_t* reward, uint8_t* action_mask, int32_t* status,
                 int32_t* not_done, void* stream);

/* CVRPEnv.get_action_mask alone (cvrp/env.py:137-149). current_node is [B,1]. */
int co_cvrp_action_mask(int64_t batch, int64_t num_loc, const float* demand, const float* used,
                        const float* vehicle_capacity, const uint8_t* visited,
                        const int64_t* current_node, uint8_t* action_mask, void* stream);

/* CVRPEnv.get_reward (cvrp/env.py:151-190): reward = -tour length of
 * [depot] + locs[actions] (closed).  check != 0 also runs
 * check_solution_validity: customers 1..N exactly once, every other entry 0
 * (CO_ST_INVALID_TOUR), then the per-step capacity scan
 * used = max(used + d, 0) <= vehicle_capacity + 1e-5 (CO_ST_OVER_CAPACITY). */
int co_cvrp_reward(int64_t batch, int64_t num_loc, int64_t steps, const float* locs,
                   const int64_t* actions, int64_t act_stride_b, int64_t act_stride_t,
                   const float* demand, const float* vehicle_capacity, int check, float* reward,
                   int32_t* status, void* stream);

/* ----------------------------------------------------------------- SLAP */

/* SLAPEnv._reset (rl4co/envs/warehousing/slap/env.py:95-129). L = n_aisles*n_locs,
 * P = products: action_mask[B,L] = 1 except column 0 (depot); to_choose[B,P] =
 * 0..P-1 (float); i[B,1] = 0; reward[B,1] = 0; ratio[B,L] = 0 (ratio may be NULL); and
 * the zero done[B,1] / terminated[B,1] that RL4COEnvBase.reset adds (envs/common/base.py:
 * 138-143 via TorchRL; each may be NULL), so a reset is one launch. */
int co_slap_reset(int64_t batch, int64_t num_slots, int64_t n_products, uint8_t* action_mask,
                  float* to_choose, int64_t* i, float* reward, float* ratio, uint8_t* done,
                  uint8_t* terminated, void* stream);

/* SLAPEnv._step (slap/env.py:38-93): product p = (int)to_choose[b*tc_stride];
 * assign_out = assign_in with [b, p] = (int)action[b] (in-place allowed:
 * then only that element is written); mask_out = mask_in with [b, action] = 0
 * (in-place allowed); done[b] = (i_in[b] == P-1); reward[b] = 0 (bool);
 * i_out = i_in + 1.  Negative indices wrap like torch advanced indexing.
 * to_choose may be NULL when every row's to_choose[b, 0] holds one value k (the env's
 * untouched arange to_choose at step k, slap/env.py:105-108): tc_stride then carries k
 * (0 <= k < P) and no to_choose column is read (the same for co_slap_decode_step and
 * co_slap_closest_step). */
int co_slap_step(int64_t batch, int64_t num_slots, int64_t n_products, const int64_t* action,
                 const float* to_choose, int64_t tc_stride, const int32_t* assign_in,
                 int32_t* assign_out, const uint8_t* mask_in, uint8_t* mask_out,
                 const int64_t* i_in, int64_t* i_out, uint8_t* done, uint8_t* reward,
                 int32_t* status, void* stream);

/* SLAPEnv._get_reward (slap/env.py:131-143): for each order o (in order),
 * total -= closed Euclidean tour over locs[assignment[picklist[b, o, :]]]. */
int co_slap_reward(int64_t batch, int64_t num_slots, int64_t n_products, int64_t n_orders,
                   int64_t order_size, const int32_t* assignment, const int64_t* picklist,
                   const float* locs, float* reward, int32_t* status, void* stream);

/* ------------------------------------------------------------ utilities */

/* utils.ops.gather_by_index (rl4co/utils/ops.py:65-77), gather along one dim:
 * src element (o, j, :) at src + o*src_stride_outer + j*src_stride_len (bytes),
 * `inner_bytes` contiguous bytes each; idx (o, m) at idx[o*idx_stride_outer +
 * m*idx_stride_len]; dst[o, m, :] contiguous [outer, idx_len, inner_bytes].
 * Out-of-range index: CO_ST_INDEX_RANGE and a zero-filled output element. */
int co_gather_by_index(const void* src, int64_t outer, int64_t src_len, int64_t inner_bytes,
                       int64_t src_stride_outer, int64_t src_stride_len, const int64_t* idx,
                       int64_t idx_len, int64_t idx_stride_outer, int64_t idx_stride_len,
                       void* dst, int32_t* status, void* stream);

/* The batch-wide test of tsp/env.py:70: *flag = any(x[0..n) == value). */
int co_any_eq_i64(const int64_t* x, int64_t n, int64_t value, int32_t* flag, void* stream);

/* ---------------------------------------------------------- decode step */

#define CO_DECODE_GREEDY 0
#define CO_DECODE_SAMPLING 1
#define CO_DECODE_EVALUATE 2
/* mode flag (OR-ed into `mode`), opt-in: hardware v_exp tanh / exp and lane-order sums.
 * Without it the step is ATen-exact: logp bit-identical to F.log_softmax of the processed
 * logits (SLEEF expf/logf and vec::map_reduce_all's 16-lane order), tanh correctly
 * rounded; with it logp is within ~1e-6 and greedy picks may differ on near-ties. */
#define CO_DECODE_FAST 0x100
/* mode flag, opt-in: greedy picks computed with the fast math and certified per row by
 * its error bound (the runner-up must trail the pick by more than the fast tanh error
 * times the clip plus two ulps of the log-sum-exp); any wave holding an uncertified row
 * is recomputed with the exact math.  Greedy actions are therefore the exact path's;
 * the selected logp is the fast one (within ~1e-6).  Other modes run exact under it. */
#define CO_DECODE_CERTIFIED 0x200

/* DecodingStrategy.step (rl4co/utils/decoding.py:141-191,327-399,489-499):
 * x = logits[b*logits_stride + c]; tanh clip (tanh_clipping > 0); masked
 * (mask != NULL and mask[b*n+c] == 0) -> -inf; x /= temperature;
 * logp = (x - max) - log(sum(exp(x - max))) (ATen's CPU evaluation, bit-exact; see
 * CO_DECODE_FAST);
 * greedy: first argmax of logp (torch tie-break); sampling: inverse CDF of
 * exp(logp) with a Philox draw keyed by (seed, offset, b); evaluate: action_in.
 * action_out[b], logp_sel[b] = logp[b, action]; logprobs_full (nullable)
 * receives the whole row.  Greedy/sampling picking a masked action sets
 * CO_ST_INFEASIBLE.  Rows of n_actions > 2048 run a workgroup-per-row kernel in the
 * exact math whatever the math flags (top-p filtering is not offered there: CO_E_INVAL). */
int co_decode_step(int64_t batch, int64_t n_actions, const float* logits, int64_t logits_stride,
                   const uint8_t* mask, float tanh_clipping, float temperature, int mode,
                   const int64_t* action_in, int64_t* action_out, float* logp_sel,
                   float* logprobs_full, uint64_t seed, uint64_t offset, int32_t* status,
                   void* stream);

/* co_decode_step with the top-k / top-p filters of process_logits (decoding.py:112-138,
 * 183-187) applied after the temperature: top_k > 0 keeps values >= the k-th largest
 * (torch.topk, multiplicity counted); 0 < top_p < 1 drops elements whose ascending
 * cumulative softmax probability (ties by index) is <= 1 - top_p.  top_k = 0 / top_p = 0
 * disable them (co_decode_step == this with 0, 0). */
int co_decode_step_ex(int64_t batch, int64_t n_actions, const float* logits,
                      int64_t logits_row_stride, const uint8_t* mask, float tanh_clipping,
                      float temperature, int top_k, double top_p, int mode,
                      const int64_t* action_in, int64_t* action_out, float* logp_selected,
                      float* logp_full, uint64_t seed, uint64_t offset, int32_t* status,
                      void* stream);

/* co_decode_step fused with TSPEnv._step (tsp/env.py:67-93) for the selected action:
 * mask_out = mask_in minus the action (in-place NOT allowed), i_out = i_in + 1,
 * first_out = first_mode ? action : first_in, done = nothing left, step_reward = 0,
 * action_out / logp_sel as co_decode_step (action_out must not alias action_in);
 * ll_accum (nullable) += logp_sel: get_log_likelihood's sum (decoding.py:39-65).
 * The decode-fused env-step of SURVEY.md 8d (4N + 4 B on top of co_tsp_step). */
int co_tsp_decode_step(int64_t batch, int64_t num_loc, const float* logits,
                       int64_t logits_stride, const uint8_t* mask_in, float tanh_clipping,
                       float temperature, int mode, const int64_t* action_in,
                       int64_t* action_out, float* logp_sel, uint64_t seed, uint64_t offset,
                       uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                       const int64_t* first_in, int64_t* first_out, int first_mode,
                       uint8_t* done, uint8_t* step_reward, float* ll_accum, int32_t* status,
                       void* stream);

/* co_decode_step fused with SLAPEnv._step (slap/env.py:38-93) for the selected action
 * (replaces DecodingStrategy.step + env.step of constructive/base.py:245-251 on the fork's
 * examples/slap.py policy path).  L = locations (the row length of logits / masks),
 * P = products.  Decode as co_decode_step; then, with a = the selected action (evaluate:
 * action_in, negative values index from the end as python indexing):
 *   assign_out = assign_in with [b, (int)to_choose[b*tc_stride]] = (int)a (out of place:
 *   the row is copied; in place: that element only); mask_out = mask_in minus a
 *   (in place allowed, as i_out = i_in); done[b] = i_in[b] == P-1; i_out = i_in + 1; step_reward = 0;
 *   ll_accum (nullable) += logp_sel.  Same bits as co_decode_step + co_slap_step. */
int co_slap_decode_step(int64_t batch, int64_t num_slots, int64_t n_products,
                        const float* logits, int64_t logits_stride, const uint8_t* mask_in,
                        float tanh_clipping, float temperature, int mode,
                        const int64_t* action_in, int64_t* action_out, float* logp_sel,
                        uint64_t seed, uint64_t offset, const float* to_choose,
                        int64_t tc_stride, const int32_t* assign_in, int32_t* assign_out,
                        uint8_t* mask_out, const int64_t* i_in, int64_t* i_out, uint8_t* done,
                        uint8_t* step_reward, float* ll_accum, int32_t* status, void* stream);

/* co_decode_step fused with CVRPEnv._step + get_action_mask (cvrp/env.py:73-149):
 * N = customers, rows of logits / masks / visited are N+1 wide.  Decode as
 * co_decode_step; then the co_cvrp_step transition for the selected action (evaluate:
 * action_in): used_out, visited_out (separate buffer), current_out (nullable) = a,
 * done, step_reward = 0, action_mask recomputed into mask_out (separate buffer);
 * ll_accum (nullable) += logp_sel.  Same bits as co_decode_step + co_cvrp_step. */
int co_cvrp_decode_step(int64_t batch, int64_t num_loc, const float* logits,
                        int64_t logits_stride, const uint8_t* mask_in, float tanh_clipping,
                        float temperature, int mode, const int64_t* action_in,
                        int64_t* action_out, float* logp_sel, uint64_t seed, uint64_t offset,
                        const float* demand, const float* used_in, float* used_out,
                        const float* vehicle_capacity, const uint8_t* visited_in,
                        uint8_t* visited_out, int64_t* current_out, uint8_t* done,
                        uint8_t* step_reward, uint8_t* mask_out, float* ll_accum,
                        int32_t* status, void* stream);

/* ------------------------------------------- bench policies (in-kernel) */

/* Deterministic cheap policies for the env-throughput benchmark
 * (SURVEY.md 8d); they are the "policy" half of a rollout, not reference code.
 * TSP: step0 -> 0, then nearest unvisited to current_node (ties lowest index).
 * CVRP: nearest feasible customer, else depot.  SLAP: free location with the
 * lowest depot_loc_dist.  first_step != 0 selects the TSP step-0 branch. */
int co_tsp_nearest_action(int64_t batch, int64_t num_loc, const float* locs,
                          const uint8_t* action_mask, const int64_t* current_node, int first_step,
                          int64_t* action_out, void* stream);
int co_cvrp_nearest_action(int64_t batch, int64_t num_loc, const float* locs,
                           const uint8_t* action_mask, const int64_t* current_node,
                           int64_t* action_out, void* stream);
int co_slap_closest_free_action(int64_t batch, int64_t num_slots, const float* depot_loc_dist,
                                const uint8_t* action_mask, int64_t* action_out, void* stream);
/* The nearest-feasible bench policy fused with CVRPEnv._step + get_action_mask
 * (cvrp/env.py:73-149): the action co_cvrp_nearest_action would pick from (mask_in,
 * cur_in) is written to action_out and applied as co_cvrp_step does, in one launch.
 * In place (visited_out == visited_in, mask_out == mask_in) is allowed.  Results are
 * identical to the two calls (which it falls back to for N + 1 > 128). */
int co_cvrp_nearest_step(int64_t batch, int64_t num_loc, const float* locs, const float* demand,
                         const float* used_in, float* used_out, const float* vehicle_capacity,
                         const uint8_t* visited_in, uint8_t* visited_out,
                         const uint8_t* mask_in, const int64_t* current_in, int64_t* action_out,
                         int64_t* current_out, uint8_t* done, uint8_t* reward, uint8_t* mask_out,
                         int32_t* status, int32_t* not_done, void* stream);
/* The closest-free bench policy fused with SLAPEnv._step (slap/env.py:38-93): the
 * action co_slap_closest_free_action would pick is written to action_out and applied
 * as co_slap_step does (assign_out = assign_in with [b, p] = action; in-place allowed),
 * in one launch.  Results identical to the two calls (which it falls back to when
 * num_slots % 4 != 0, num_slots > 256 or the buffers are misaligned). */
int co_slap_closest_step(int64_t batch, int64_t num_slots, int64_t n_products,
                         const float* depot_loc_dist, const float* to_choose, int64_t tc_stride,
                         const int32_t* assign_in, int32_t* assign_out, const uint8_t* mask_in,
                         uint8_t* mask_out,
                         int64_t* action_out, const int64_t* i_in, int64_t* i_out, uint8_t* done,
                         uint8_t* reward, int32_t* status, void* stream);

/* K consecutive co_slap_closest_step calls in one launch (round 6): the state ping-pongs
 * between buffers A and B (step k reads mask / i from A for even k, from B for odd k, and
 * writes the other), step k's action to action_out + k*act_stride, its product from
 * to_choose column k (row stride tc_stride; with to_choose NULL the uniform product
 * tc_stride + k), the assignment of step 0 written out of place from assign_in when it
 * differs from assign_out and in place after; done / reward written by every step.  Each
 * step stores its whole state as its own launch would; the final contents are
 * bit-identical to the K calls.  For the stepwise engine's closest-free bench policy. */
int co_slap_closest_steps(int64_t batch, int64_t num_slots, int64_t n_products, int64_t steps,
                          const float* depot_loc_dist, const float* to_choose, int64_t tc_stride,
                          const int32_t* assign_in, int32_t* assign_out, uint8_t* mask_a,
                          int64_t* i_a, uint8_t* mask_b, int64_t* i_b, int64_t* action_out,
                          int64_t act_stride, uint8_t* done, uint8_t* reward, int32_t* status,
                          void* stream);

/* -------------------------------------------- fused episode rollouts */

/* One launch per episode (reset + N steps + reward) for the env-only rollout of
 * rl4co/utils/decoding.py:88-109 with the policy in-kernel.  Each step applies
 * TSPEnv._step (tsp/env.py:67-93) to register state; only what a caller can
 * observe after rollout() is written: the final action_mask[B,N], first_node[B],
 * current_node[B], i[B,1] (= N), done[B], the last step's bool reward[B], the
 * episode reward[B] (= -closed tour length, TSPEnv.get_reward) and, for the
 * in-kernel policy, the actions.  Actions are step-major [N, B] (row t = the [B]
 * action tensor of step t).  acts_in != NULL: teacher-forced (Evaluate mode);
 * acts_in == NULL: nearest-unvisited policy (co_tsp_nearest_action) writing
 * acts_out.  check != 0: a non-permutation sets CO_ST_INVALID_TOUR.  One launch for
 * N <= 256 (teacher) / N <= 1024 (nearest); longer episodes run the same steps as a
 * sequence of the stepwise kernels (co_tsp_reset, co_tsp_step in place, co_tsp_reward),
 * with identical outputs. */
int co_tsp_rollout(int64_t batch, int64_t num_loc, const float* locs, const int64_t* acts_in,
                   int64_t* acts_out, uint8_t* action_mask, int64_t* first_node,
                   int64_t* current_node, int64_t* i, uint8_t* done, uint8_t* step_reward,
                   float* reward, int check, int32_t* status, void* stream);

/* co_tsp_rollout with the teacher actions' layout given by strides: element (b, t) at
 * acts_in[b*act_stride_b + t*act_stride_t].  (1, batch) is co_tsp_rollout's step-major
 * [N, B]; (>= num_loc, 1) is row-major [B, N] -- the reference's [B, T] layout
 * (ConstructivePolicy's `actions`, rl4co/models/common/constructive/base.py:223-230): one
 * lane group per instance reads the instance's contiguous action and coordinate rows
 * (num_loc <= 1024).  acts_in == NULL: the nearest policy as co_tsp_rollout (strides
 * unused).  Same outputs as co_tsp_rollout. */
int co_tsp_rollout_ex(int64_t batch, int64_t num_loc, const float* locs, const int64_t* acts_in,
                      int64_t act_stride_b, int64_t act_stride_t, int64_t* acts_out,
                      uint8_t* action_mask, int64_t* first_node, int64_t* current_node,
                      int64_t* i, uint8_t* done, uint8_t* step_reward, float* reward, int check,
                      int32_t* status, void* stream);

/* CVRP episode in one launch (cvrp/env.py:73-190 under decoding.py:88-109 rollout):
 * reset from the generator columns (depot[B,2], locs[B,N,2], demand[B,N] already
 * divided by the capacity, vehicle capacity vcap), then the nearest-feasible policy
 * (co_cvrp_nearest_action's rule) until every instance is done, then the closed-tour
 * reward.  Actions are step-major [max_steps, B]; *steps_out (device int32) receives
 * the batch-wide episode length T (the reference's number of loop iterations); rows
 * [len_b, T) of a shorter episode hold the depot steps the reference applies to
 * finished instances, and their state reflects them.  Writes locs_out[B,N+1,2]
 * (nullable), current_node[B], used_capacity[B], vehicle_capacity[B], visited[B,N+1],
 * action_mask[B,N+1], done[B], step_reward[B] (bool 0), reward[B], len_out[B] (own
 * episode length).  An instance not done after max_steps sets CO_ST_TRUNCATED.
 * N <= 1023. */
int co_cvrp_rollout(int64_t batch, int64_t num_loc, const float* depot, const float* locs,
                    const float* demand, float vehicle_capacity, int64_t max_steps,
                    int64_t* acts_out, float* locs_out, int64_t* current_node,
                    float* used_capacity, float* vehicle_capacity_out, uint8_t* visited,
                    uint8_t* action_mask, uint8_t* done, uint8_t* step_reward, float* reward,
                    int32_t* len_out, int32_t* steps_out, int32_t* status, void* stream);

/* SLAP episode in one launch (slap/env.py:38-143): P steps (product t <- the
 * step-t location; locations masked; done at i == P-1) then the per-order pick
 * tour reward.  Writes action_mask[B,L], assignment[B,P] (from assign_in, the
 * generator's -1s), i[B,1] (= P), done[B,1], step_reward[B,1], reward[B] and
 * ratio[B,L] = 0 (nullable).  acts_in != NULL: teacher-forced step-major [P,B];
 * acts_in == NULL: closest-free policy on depot_dist, written to acts_out.  L <= 256. */
int co_slap_rollout(int64_t batch, int64_t num_slots, int64_t n_products, int64_t n_orders,
                    int64_t order_size, const float* locs, const int64_t* picklist,
                    const float* depot_dist, const int32_t* assign_in, const int64_t* acts_in,
                    int64_t* acts_out, uint8_t* action_mask, int32_t* assignment, int64_t* i,
                    uint8_t* done, uint8_t* step_reward, float* reward, float* ratio,
                    int32_t* status, void* stream);

/* POMO shared baseline (rl4co/models/rl/reinforce/baselines.py:57-61,
 * reinforce.py:97-115, zoo/pomo/model.py:105-114) over the multistart layout
 * env e = s*instances + b: bl[b] = mean_s reward, max_reward[b] / best_start[b] =
 * max / first argmax over s, adv[e] = reward[e] - bl[b] and
 * loss_terms[b] = sum_s adv * log_likelihood (loss = -sum_b loss_terms / (S*B)).
 * log_likelihood / adv / loss_terms may be NULL. */
int co_pomo_shared_baseline(int64_t instances, int64_t starts, const float* reward,
                            const float* log_likelihood, float* bl, float* max_reward,
                            int64_t* best_start, float* adv, float* loss_terms, void* stream);

/* The deterministic part of SLAPGenerator._generate (slap/generator.py:51-81,137-155):
 * locs[B,L,2] aisle grid (x = aisle * inter_aisle_dist, y = loc * inter_loc_dist, products
 * in double rounded to f32), depot_loc_dist[B,L] and dist_mat[B,L,L] (nullable;
 * Manhattan, f32) and assignment[B,P] = -1 (nullable); L = n_aisles * n_locs.  freq and
 * the picklists stay on the host RNG streams. */
int co_slap_generate(int64_t batch, int64_t n_aisles, int64_t n_locs, double inter_aisle_dist,
                     double inter_loc_dist, int64_t n_products, float* locs,
                     float* depot_loc_dist, float* dist_mat, int32_t* assignment,
                     void* stream);

/* dihedral_8_augmentation (rl4co/data/transforms.py:15-37): out[8B, N, 2], row r*B + b
 * = transform r of instance b, r in the reference's order (x,y) (1-x,y) (x,1-y)
 * (1-x,1-y) (y,x) (1-y,x) (y,1-x) (1-y,1-x). */
int co_dihedral8_augment(int64_t batch, int64_t num_loc, const float* xy, float* out,
                         void* stream);

/* symmetric_transform (rl4co/data/transforms.py:49-71) given the per-row angles phi[B]
 * (drawn by the caller exactly as symmetric_augmentation does, transforms.py:74-93):
 * rotate (x,y) - offset by phi, swap the axes where phi > 2*pi, add the offset. */
int co_symmetric_augment(int64_t batch, int64_t num_loc, const float* xy, const float* phi,
                         float offset, float* out, void* stream);

/* BeamSearch._make_beam_step (rl4co/utils/decoding.py:611-641): rows e = s*B + b of
 * logp[BW*B, N] (full log-probabilities of the beams) plus parent[e] are ranked per
 * instance over the BW*N (beam, node) candidates; the BW best (descending; equal scores
 * -> lower candidate index s*N + c) are written to rows j*B + b: selected node,
 * beam_parent s, beam_row = b + s*B (the state row to continue from) and the new parent
 * score.  mask != NULL: a selected node with mask 0 sets CO_ST_INFEASIBLE
 * (decoding.py:519-522).  BW*N <= 36864. */
int co_beam_select(int64_t batch, int64_t beam_width, int64_t n_actions, const float* logp,
                   int64_t logp_row_stride, const float* parent, const uint8_t* mask,
                   int64_t* selected, int32_t* beam_parent, int64_t* beam_row,
                   float* score_out, int32_t* status, void* stream);

/* get_distance_matrix (rl4co/utils/ops.py:104-111): out[B, N, N] = Euclidean distances
 * between the instance's coordinates, f32 sqrt(dx*dx + dy*dy).  out 16-byte aligned. */
int co_distance_matrix(int64_t batch, int64_t num_loc, const float* locs, float* out,
                       void* stream);

/* Number of rows with done[b] == 0 written to *count (device int32). */
int co_count_not_done(const uint8_t* done, int64_t n, int32_t* count, void* stream);

/* *out (device int32) = max(0, max over rows b of (width - sum of rows[b*row_stride + c],
 * c < width)).  The decode loop's `while not td["done"].all()` poll for CVRP
 * (constructive/base.py:245, cvrp/env.py:92 done = visited.sum(-1) == N+1): a positive
 * deficit d means no instance set can be all done within the next d - 1 steps, so those
 * host syncs are skipped without changing the stopping step. */
int co_row_deficit_max(const uint8_t* rows, int64_t n_rows, int64_t width, int64_t row_stride,
                       int32_t* out, void* stream);

/* Device instance generation for throughput runs: the Uniform
 * samplers of tsp/generator.py:51-60 and cvrp/generator.py:116-143 on a Philox-4x32-10
 * stream (key = seed, block counter offset + i/4) instead of torch's CPU generator, so the
 * values follow torch's f32 uniform grid and transform but not its stream (parity
 * instances keep the host generators).  demand == 0: out[i] = low + u*(high-low);
 * demand != 0: out[i] = ((int)(low + u*(high-low)) + 1) / capacity. */
int co_uniform_fill(float* out, int64_t n, float low, float high, float capacity, int demand,
                    uint64_t seed, uint64_t offset, void* stream);

/* Integers in [low, high) on the same Philox stream layout, for SLAP picklists in
 * throughput runs (slap/generator.py:137-155 draws them with numpy's randint):
 * out[i] = low + ((uint64)x_i * (high - low)) >> 32, 0 < high - low < 2^32. */
int co_randint_fill(int64_t* out, int64_t n, int64_t low, int64_t high, uint64_t seed,
                    uint64_t offset, void* stream);

/* ------------------------------------------------ measurement utility (no reference
 * counterpart): dst[0:nbytes) = src[0:nbytes), one 16-byte load/store per thread over a
 * full grid -- the streaming ceiling the bench quotes beside each kernel's roofline.
 * src/dst 16-byte aligned, nbytes a multiple of 16. */
int co_probe_copy(const void* src, void* dst, int64_t nbytes, void* stream);

/* The decode loop's epilogue (DecodingStrategy.post_decoder_hook, decoding.py:315-325, and
 * get_log_likelihood, decoding.py:39-65) in one launch.  The T per-step [B] actions and
 * log-probabilities are rows of step-major slabs (act_sm[t * act_rs + b], logp_sm[t *
 * logp_rs + b]: the tensors the per-step calls returned); writes torch.stack(..., 1) =
 * actions[B, T] / logprobs[B, T], ll[B] = logprobs.sum(1) (summed in step order in f64,
 * rounded once; may be NULL), and ORs CO_ST_LOGP_NEG_INF into status when any log-
 * probability is not > -1000 (the assert of decoding.py:57-58).  act_sm or logp_sm may be
 * NULL (that half is skipped). */
int co_episode_stack(int64_t batch, int64_t steps, const int64_t* act_sm, int64_t act_rs,
                     const float* logp_sm, int64_t logp_rs, int64_t* actions, float* logprobs,
                     float* ll, int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CO_ENV_H */
