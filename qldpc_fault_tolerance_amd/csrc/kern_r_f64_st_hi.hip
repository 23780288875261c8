// kern_r_f64_st_hi.hip — engine id 1013 (see kern_r_f64_st.hip) for VPL 7-8.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_st_hi(int vpl, int d3k) {
  switch (vpl) {
    case 7: return pick_rd3k<double, 7, 1013, 4, 1024, 4>(d3k);
    case 8: return pick_rd3k<double, 8, 1013, 4, 1024, 4>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
