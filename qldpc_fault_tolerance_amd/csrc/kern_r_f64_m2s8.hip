// kern_r_f64_m2s8.hip — double kernels of the "m2 in slot" family for rows of 8 edges and column
// degree 5 (engine id 10103, bp_reg.h eng_m2s without the tail array): rows of 4 16-byte chunks,
// one-word check state, 256-thread workgroups.  The lifted-product codes (LP_Matg8_L30: 750
// degree-3 and 270 degree-5 columns, rows of 8, VPL 4, D3K 2): the degree-3 variables of the slot
// shared with the degree-5 class keep private dummy V slots for their two missing edges
// (qldpc_hip.hip build_slot_edges).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_m2s8(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 10103, 5, 256, 4>(d3k);
    case 5: return pick_rd3k<double, 5, 10103, 5, 256, 4>(d3k);
    case 6: return pick_rd3k<double, 6, 10103, 5, 256, 4>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
// packed absolute edge addresses (engine id 10203, bp_reg.h RState::kPk): 4 workgroups per CU
SVariant get_rvariant_f64_m2s8pk(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 10203, 5, 256, 4>(d3k);
    case 5: return pick_rd3k<double, 5, 10203, 5, 256, 4>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
