// kern_r_f64_m2s.hip — double kernels of engine 3, "m2 in slot" family (engine id 11103,
// bp_reg.h eng_m2s): <= 256-thread workgroups, rows of 3 16-byte chunks + a tail slot (rows
// of up to 7 edges), one-word check state; 3 workgroups per CU (168 VGPRs).  The headline
// hgp_34_n1600 graphs: 256 threads x 7 variables, D3K 4, a 52.3 KB image.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_m2s(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 11103, 4, 256, 3>(d3k);
    case 5: return pick_rd3k<double, 5, 11103, 4, 256, 3>(d3k);
    case 6: return pick_rd3k<double, 6, 11103, 4, 256, 3>(d3k);
    case 7: return pick_rd3k<double, 7, 11103, 4, 256, 3>(d3k);
    case 8: return pick_rd3k<double, 8, 11103, 4, 256, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
