// Diagnostic builds: the -DCO_DIAG_* switches of the measurement tools, in one place.
//
// The product library (csrc/build.py) defines none of them; every hook below is then a
// compile-time false and the compiler drops the code it guards.  Tools build variants of
// the library with one switch set (tools/build_variants.sh, tools/diag_cert_count.py) to
// time or count one part of a kernel; such a library exports co_variant_timing_cut_decode
// (decode_step.hip, for any of the switches below), and _native.load() refuses it in the
// product's slot (_lib/libco_env.so) and only warns when a tool points LIB_PATH at it.
#pragma once

namespace co {

#ifdef CO_DIAG_FASTTANH  // timing: the fast tanh inside the exact decode math
constexpr bool kDiagFastTanh = true;
#else
constexpr bool kDiagFastTanh = false;
#endif

#ifdef CO_DIAG_FASTEXP  // timing: the fast exp-sum inside the exact decode math
constexpr bool kDiagFastExp = true;
#else
constexpr bool kDiagFastExp = false;
#endif

#ifdef CO_DIAG_CERT_COUNT  // counting: certified-decode rows resolved by tier 1 get
constexpr bool kDiagCertCount = true;  // logp -23456, rows of tier 2 -12345
#else
constexpr bool kDiagCertCount = false;
#endif

#ifdef CO_DIAG_CVRP_CUT  // timing: co_cvrp_decode_step without its transition (1) or decode (2)
constexpr int kDiagCvrpCut = CO_DIAG_CVRP_CUT;
#else
constexpr int kDiagCvrpCut = 0;
#endif

// a build whose "exact" decode is not exact
constexpr bool kDiagTimingCut = kDiagFastTanh || kDiagFastExp || kDiagCvrpCut != 0;

}  // namespace co
