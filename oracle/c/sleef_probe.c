/* TEST INFRASTRUCTURE: direct calls into the SLEEF functions torch itself bundles and calls
 * from ATen's vectorised CPU kernels (libtorch_cpu exports Sleef_expf16_u10 /
 * Sleef_logf16_u10), so tests/test_aten_math.py can compare oracle/c/aten_math.c with the
 * very code ATen runs.  Needs an AVX512F host; never part of the product. */
#include <immintrin.h>

__m512 Sleef_expf16_u10(__m512);
__m512 Sleef_logf16_u10(__m512);

void probe_sleef_expf(const float* x, float* y, long n) {
  for (long i = 0; i + 16 <= n; i += 16) _mm512_storeu_ps(y + i, Sleef_expf16_u10(_mm512_loadu_ps(x + i)));
}
void probe_sleef_logf(const float* x, float* y, long n) {
  for (long i = 0; i + 16 <= n; i += 16) _mm512_storeu_ps(y + i, Sleef_logf16_u10(_mm512_loadu_ps(x + i)));
}
