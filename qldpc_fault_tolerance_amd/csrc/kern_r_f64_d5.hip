// kern_r_f64_d5.hip — double kernels of engine 3 with 5 edge slots per variable (column degree
// 5: the lifted-product codes) for <= 256-thread workgroups (engine id 103: own v2c in VGPRs,
// unpacked absolute addresses), rows of 3 or 4 16-byte chunks, VPL 4-5, every D3K in 0..VPL.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
template <int NCH>
static SVariant pick_d5(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 103, 5, 256, NCH>(d3k);
    case 5: return pick_rd3k<double, 5, 103, 5, 256, NCH>(d3k);
    // 6 variables (rows of 9-10 only: LP_Matg8_L30's [h | I], 1470 columns at 256 threads; <= 212 VGPRs)
    case 6:
      if constexpr (NCH == 5) return pick_rd3k<double, 6, 103, 5, 256, NCH>(d3k);
      return SVariant{nullptr, nullptr, nullptr, nullptr};
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
SVariant get_rvariant_f64_w_d5(int vpl, int d3k, int nch) {
  // (nch 5: rows of 9-10, the lifted-product [h | I] graphs of CodeSimulator_Phenon's decoder1, round 6)
  return nch == 4 ? pick_d5<4>(vpl, d3k) : nch == 3 ? pick_d5<3>(vpl, d3k) : nch == 5 ? pick_d5<5>(vpl, d3k)
                                                                           : SVariant{nullptr, nullptr, nullptr, nullptr};
}
}  // namespace qldpc
