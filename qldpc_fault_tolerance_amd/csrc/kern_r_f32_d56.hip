// kern_r_f32_d56.hip — float kernels of engine 3 for column degree 5 and 6
// (e.g. the lifted-product codes: degrees 3 and 5), VPL 1-5, every D3K.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
template <int DM>
SVariant pick_d56(int vpl, int d3k) {
  switch (vpl) {
    case 1: return pick_rd3k<float, 1, 3, DM>(d3k);
    case 2: return pick_rd3k<float, 2, 3, DM>(d3k);
    case 3: return pick_rd3k<float, 3, 3, DM>(d3k);
    case 4: return pick_rd3k<float, 4, 3, DM>(d3k);
    case 5: return pick_rd3k<float, 5, 3, DM>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
SVariant get_rvariant_f32_d5(int vpl, int d3k) { return pick_d56<5>(vpl, d3k); }
SVariant get_rvariant_f32_d6(int vpl, int d3k) { return pick_d56<6>(vpl, d3k); }
}  // namespace qldpc
