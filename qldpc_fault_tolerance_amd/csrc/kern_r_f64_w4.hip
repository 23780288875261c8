// kern_r_f64_w4.hip — double kernels of engine 3 for workgroups of <= 256 threads
// (engine id 103) with rows of 4 16-byte chunks (compile-time check-phase width):
// 2 workgroups per CU, so a 256-VGPR budget that holds each thread's own
// previous v2c messages; every compile-time D3K in 0..VPL.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_w4(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 103, 4, 256, 4>(d3k);
    case 5: return pick_rd3k<double, 5, 103, 4, 256, 4>(d3k);
    case 6: return pick_rd3k<double, 6, 103, 4, 256, 4>(d3k);
    case 7: return pick_rd3k<double, 7, 103, 4, 256, 4>(d3k);
    case 8: return pick_rd3k<double, 8, 103, 4, 256, 4>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
SVariant get_rvariant_f64_w(int vpl, int d3k, int nch) {
  return nch == 4 ? get_rvariant_f64_w4(vpl, d3k) : nch == 3 ? get_rvariant_f64_w3(vpl, d3k)
                                                             : SVariant{nullptr, nullptr, nullptr, nullptr};
}
}  // namespace qldpc
