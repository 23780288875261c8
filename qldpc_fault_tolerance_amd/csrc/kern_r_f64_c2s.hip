// kern_r_f64_c2s.hip — double kernels of engine 3, "c2v in slot" family (engine id 31103,
// bp_reg.h eng_c2s): the check phase writes every edge's c2v into the row's slots (alpha * m1 with
// the edge's sign, one xor turning the argmin's into alpha * m2), so the variable phase reads one
// word per edge and keeps no previous v2c in VGPRs.  No check-state array: the n1600 image is
// 46.2 KB, rows of 7 edges as 3 16-byte chunks + a tail slot, 3 workgroups per CU.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
#if QLDPC_EXPERIMENTAL
SVariant get_rvariant_f64_c2s(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 31103, 4, 256, 3>(d3k);
    case 5: return pick_rd3k<double, 5, 31103, 4, 256, 3>(d3k);
    case 6: return pick_rd3k<double, 6, 31103, 4, 256, 3>(d3k);
    case 7: return pick_rd3k<double, 7, 31103, 4, 256, 3>(d3k);
    case 8: return pick_rd3k<double, 8, 31103, 4, 256, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
#else
// measured-and-not-kept family: built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)
SVariant get_rvariant_f64_c2s(int vpl, int d3k) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
#endif
}  // namespace qldpc
