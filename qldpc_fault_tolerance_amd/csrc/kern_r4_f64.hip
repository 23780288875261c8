// kern_r4_f64.hip — double kernels of engine 4 (c2v computed by the check phase, column degree <= 4):
// the 1024-thread family and the <= 256-thread family (3 workgroups per CU: <= 168 VGPRs).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
#if QLDPC_EXPERIMENTAL
SVariant get_r4variant_f64(int vpl) { return pick_rvpl<double, 4>(vpl); }
SVariant get_r4variant_f64_w(int vpl) {
  switch (vpl) {
    case 4: return make_rvariant<double, 4, 4, 0, 4, 256>();
    case 5: return make_rvariant<double, 5, 4, 0, 4, 256>();
    case 6: return make_rvariant<double, 6, 4, 0, 4, 256>();
    case 7: return make_rvariant<double, 7, 4, 0, 4, 256>();
    case 8: return make_rvariant<double, 8, 4, 0, 4, 256>();
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
#else
// measured-and-not-kept family: built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)
SVariant get_r4variant_f64(int vpl) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
SVariant get_r4variant_f64_w(int vpl) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
#endif
}  // namespace qldpc
