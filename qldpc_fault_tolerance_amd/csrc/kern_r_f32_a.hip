// kern_r_f32_a.hip — float kernels of engine 3 (register-resident variables,
// column degree <= 4) for VPL 1,2,3,4, every compile-time D3K (degree-3 slots) in 0..VPL.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_a(int vpl, int d3k) {
  switch (vpl) {
    case 1: return pick_rd3k<float, 1, 3>(d3k);
    case 2: return pick_rd3k<float, 2, 3>(d3k);
    case 3: return pick_rd3k<float, 3, 3>(d3k);
    case 4: return pick_rd3k<float, 4, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
SVariant get_rvariant_f32(int vpl, int d3k) {
  return vpl <= 4 ? get_rvariant_f32_a(vpl, d3k) : vpl <= 6 ? get_rvariant_f32_b(vpl, d3k) : get_rvariant_f32_c(vpl, d3k);
}
}  // namespace qldpc
