// Launch ceiling of the one-round step kernels (diagnostic, not part of the product): a
// kernel with the step kernels' grid (2,048 workgroups of 256 threads; and the same 512K
// threads in other workgroup sizes) and (a) an empty body, (b) one 4-byte load + store per thread (the smallest memory round trip every wave
// of a step kernel makes).  tools/launch_ceiling.py times them beside co_tsp_step /
// co_cvrp_step and the same-byte co_probe_copy, under a rocprofv3 kernel trace.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void __launch_bounds__(1024) ceiling_empty_kernel(int32_t* sink, int flag) {
  if (flag == 12345 && sink) sink[threadIdx.x] = 0;  // never taken: keeps the arguments live
}

__global__ void __launch_bounds__(1024) ceiling_touch_kernel(const int32_t* src, int32_t* dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  dst[t] = src[t] + 1;
}

extern "C" int ceiling_empty(int blocks, int threads, int reps, int32_t* sink, void* stream) {
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(ceiling_empty_kernel, dim3(blocks), dim3(threads), 0,
                       (hipStream_t)stream, sink, 0);
  return (int)hipGetLastError();
}

extern "C" int ceiling_touch(int blocks, int threads, int reps, const int32_t* src, int32_t* dst,
                             void* stream) {
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(ceiling_touch_kernel, dim3(blocks), dim3(threads), 0,
                       (hipStream_t)stream, src, dst);
  return (int)hipGetLastError();
}
