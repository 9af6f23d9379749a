// Host cost of a kernel launch by argument shape (diagnostic, not part of the product):
// 19 scalar arguments as co_tsp_decode_step's greedy kernel has, against the same bytes as
// one by-value struct.  The kernels do nothing (grid of 1).
#include <hip/hip_runtime.h>
#include <cstdint>

struct P19 {
  int64_t B;
  int N;
  const float* logits;
  int64_t lstride;
  const uint8_t* mask_in;
  float clip, temp;
  int64_t* action_out;
  float* logp_sel;
  uint8_t* mask_out;
  const int64_t* i_in;
  int64_t* i_out;
  const int64_t* first_in;
  int64_t* first_out;
  int take_first;
  uint8_t* done;
  uint8_t* step_reward;
  float* ll_accum;
  int32_t* status;
};

__global__ void k19(int64_t B, int N, const float* logits, int64_t lstride, const uint8_t* mask_in,
                    float clip, float temp, int64_t* action_out, float* logp_sel,
                    uint8_t* mask_out, const int64_t* i_in, int64_t* i_out,
                    const int64_t* first_in, int64_t* first_out, int take_first, uint8_t* done,
                    uint8_t* step_reward, float* ll_accum, int32_t* status) {
  if (B < 0 && status) status[0] = N + take_first;
}
__global__ void kstruct(const P19 p) {
  if (p.B < 0 && p.status) p.status[0] = p.N + p.take_first;
}

extern "C" int launch19(void* stream, int reps) {
  hipStream_t s = (hipStream_t)stream;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k19, dim3(1), dim3(64), 0, s, (int64_t)1, 100, nullptr, (int64_t)100,
                       nullptr, 0.f, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, 0, nullptr, nullptr, nullptr, nullptr);
  return (int)hipGetLastError();
}
extern "C" int launch_struct(void* stream, int reps) {
  hipStream_t s = (hipStream_t)stream;
  P19 p{};
  p.B = 1;
  p.N = 100;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kstruct, dim3(1), dim3(64), 0, s, p);
  return (int)hipGetLastError();
}
extern "C" int launch_module(void* stream, int reps) {
  hipStream_t s = (hipStream_t)stream;
  static hipFunction_t f = nullptr;
  if (!f && hipGetFuncBySymbol(&f, (const void*)kstruct) != hipSuccess) return -1;
  P19 p{};
  p.B = 1;
  p.N = 100;
  size_t sz = sizeof(p);
  for (int r = 0; r < reps; ++r) {
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &p, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                   HIP_LAUNCH_PARAM_END};
    hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, s, nullptr, cfg);
  }
  return (int)hipGetLastError();
}

extern "C" int launch19_err(void* stream, int reps) {
  hipStream_t s = (hipStream_t)stream;
  int rc = 0;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k19, dim3(1), dim3(64), 0, s, (int64_t)1, 100, nullptr, (int64_t)100,
                       nullptr, 0.f, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, 0, nullptr, nullptr, nullptr, nullptr);
    rc |= (int)hipGetLastError();
  }
  return rc;
}
extern "C" int get_error_only(void* stream, int reps) {
  int rc = 0;
  for (int r = 0; r < reps; ++r) rc |= (int)hipGetLastError();
  return rc;
}
// the product entry point called from C in a loop (no Python in between)
typedef int (*TspDecodeStep)(int64_t, int64_t, const float*, int64_t, const uint8_t*, float, float,
                             int, const int64_t*, int64_t*, float*, uint64_t, uint64_t, uint8_t*,
                             const int64_t*, int64_t*, const int64_t*, int64_t*, int, uint8_t*,
                             uint8_t*, float*, int32_t*, void*);
extern "C" int call_tsp_decode_step(void* fn, int reps, int64_t B, int64_t N, const float* logits,
                                    const uint8_t* mask, int64_t* act, float* lp, uint8_t* mo,
                                    const int64_t* i, int64_t* io, const int64_t* first,
                                    int64_t* fo, uint8_t* done, uint8_t* rew, int32_t* st,
                                    void* stream) {
  TspDecodeStep f = (TspDecodeStep)fn;
  int rc = 0;
  for (int r = 0; r < reps; ++r)
    rc |= f(B, N, logits, N, mask, 0.f, 1.f, 0x200, nullptr, act, lp, 0, 0, mo, i, io, first, fo,
            0, done, rew, nullptr, st, stream);
  return rc;
}
