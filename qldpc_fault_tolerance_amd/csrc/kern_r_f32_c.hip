// kern_r_f32_c.hip — float kernels of engine 3 (register-resident variables,
// column degree <= 4) for VPL 7,8, every compile-time D3K (degree-3 slots) in 0..VPL.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_c(int vpl, int d3k) {
  switch (vpl) {
    case 7: return pick_rd3k<float, 7, 3>(d3k);
    case 8: return pick_rd3k<float, 8, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
