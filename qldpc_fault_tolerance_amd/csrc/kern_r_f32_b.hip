// kern_r_f32_b.hip — float kernels of engine 3 (register-resident variables,
// column degree <= 4) for VPL 5,6, every compile-time D3K (degree-3 slots) in 0..VPL.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_b(int vpl, int d3k) {
  switch (vpl) {
    case 5: return pick_rd3k<float, 5, 3>(d3k);
    case 6: return pick_rd3k<float, 6, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
