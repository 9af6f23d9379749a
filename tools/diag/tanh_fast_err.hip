// Measures the absolute error of decode.hip's CO_DECODE_FAST tanh (co_tanh_fast: v_exp_f32
// + v_rcp_f32) against the f64 tanh over every f32 in [-9.1, 9.1] (the clip range where
// tanh is not saturated).  The certified decode's bound (decode.hip, GreedyRow::certify)
// assumes <= 1.5e-6.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/diag/tanh_fast_err
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float tanh_fast(float x) {  // = decode.hip co_tanh_fast
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

__global__ void err_kernel(uint32_t lo, uint32_t n, unsigned long long* worst) {
  double w = 0.0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t bits = lo + k;
    const float x = __uint_as_float(bits);
    if (!(fabsf(x) <= 9.1f)) continue;
    const double e = fabs((double)tanh_fast(x) - tanh((double)x));
    w = e > w ? e : w;
  }
  atomicMax(worst, (unsigned long long)__double_as_longlong(w));  // non-negative doubles
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 8);
  hipMemset(d, 0, 8);
  // positive and negative f32 up to 9.1 (bit patterns are monotone within a sign)
  const uint32_t top = 0x4111999au;  // 9.1f
  hipLaunchKernelGGL(err_kernel, dim3(4096), dim3(256), 0, 0, 0u, top + 1u, d);
  hipLaunchKernelGGL(err_kernel, dim3(4096), dim3(256), 0, 0, 0x80000000u, top + 1u, d);
  unsigned long long h = 0;
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  double w;
  std::memcpy(&w, &h, 8);
  std::printf("{\"max_abs_err_fast_tanh\": %.6e}\n", w);
  return 0;
}
