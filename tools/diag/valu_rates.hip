// VALU throughput probes (diagnostic, not part of the product): each lane runs ITERS
// iterations of 8 independent chains of one instruction (inline asm, so the compiler neither
// folds nor reorders them); tools/valu_rates.py times the grid with HIP events and reports
// SIMD cycles per wave-instruction at W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>

#define CHAINS(OP)                                                                      \
  for (int i = 0; i < iters; ++i) {                                                     \
    OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)                             \
  }

#define K(NAME, DECL, OP, OUT)                                                          \
  __global__ void __launch_bounds__(256) NAME(int iters, float* sink, float seed) {      \
    DECL                                                                                \
    CHAINS(OP)                                                                          \
    if (seed == 12345.f) sink[threadIdx.x] = OUT;                                       \
  }

#define F8 float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
  a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c = seed * 0.5f;
#define OUTF (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7)
#define OP_SUB(x) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MUL(x) asm volatile("v_mul_f32 %0, %0, %0" : "+v"(x));
#define OP_FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(c));
K(k_sub, F8, OP_SUB, OUTF)
K(k_mul, F8, OP_MUL, OUTF)
K(k_fma, F8, OP_FMA, OUTF)

typedef float v2f __attribute__((ext_vector_type(2)));
#define V8 v2f a0 = {seed, seed + 1}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
  a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c = {seed, seed};
#define OUTV (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7)[0]
#define OP_PKADD(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_PKMUL(x) asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(x));
#define OP_PKFMA(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(c));
K(k_pkadd, V8, OP_PKADD, OUTV)
K(k_pkmul, V8, OP_PKMUL, OUTV)
K(k_pkfma, V8, OP_PKFMA, OUTV)

#define U8 uint32_t a0 = (uint32_t)seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, \
  a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c = a0 * 3u, d = a0 * 5u;
#define OUTU (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7)
#define OP_MIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MED3(x) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(d));
#define OP_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(d));
#define OP_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(c));
#define OP_DPP(x) asm volatile("v_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
K(k_min, U8, OP_MIN, OUTU)
K(k_med3, U8, OP_MED3, OUTU)
K(k_andor, U8, OP_ANDOR, OUTU)
K(k_cnd, U8, OP_CND, OUTU)
K(k_dpp, U8, OP_DPP, OUTU)

// one chain only (dependent latency)
#define CHAIN1(OP)                                                                      \
  for (int i = 0; i < iters; ++i) {                                                     \
    OP(a0) OP(a0) OP(a0) OP(a0) OP(a0) OP(a0) OP(a0) OP(a0)                             \
  }
#define K1(NAME, DECL, OP, OUT)                                                         \
  __global__ void __launch_bounds__(256) NAME(int iters, float* sink, float seed) {      \
    DECL                                                                                \
    CHAIN1(OP)                                                                          \
    if (seed == 12345.f) sink[threadIdx.x] = OUT;                                       \
  }
K1(k_min_dep, U8, OP_MIN, OUTU)
K1(k_med3_dep, U8, OP_MED3, OUTU)
K1(k_pkadd_dep, V8, OP_PKADD, OUTV)
K1(k_sub_dep, F8, OP_SUB, OUTF)
K1(k_dpp_dep, U8, OP_DPP, OUTU)

extern "C" int valu_probe(int which, int blocks, int threads, int iters, float* sink,
                          void* stream) {
  void (*ks[])(int, float*, float) = {k_sub, k_mul, k_fma, k_pkadd, k_pkmul, k_pkfma,
                                      k_min, k_med3, k_andor, k_cnd, k_dpp, k_min_dep,
                                      k_med3_dep, k_pkadd_dep, k_sub_dep, k_dpp_dep};
  if (which < 0 || which >= (int)(sizeof(ks) / sizeof(ks[0]))) return -1;
  hipLaunchKernelGGL(ks[which], dim3(blocks), dim3(threads), 0, (hipStream_t)stream, iters,
                     sink, 1.0f);
  return (int)hipGetLastError();
}
