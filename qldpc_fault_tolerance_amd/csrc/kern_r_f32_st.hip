// kern_r_f32_st.hip — float kernels of engine 3 for the tail layout (engine id 1013):
// rows of 2 16-byte chunks plus one tail slot per row, dword-scaled edge addresses,
// 1024-thread workgroups (the space-time graphs' rows of 9: the check phase reads 36
// instead of 48 bytes per row, with the compile-time-width loop).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_st(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<float, 4, 1013, 4, 1024, 2>(d3k);
    case 5: return pick_rd3k<float, 5, 1013, 4, 1024, 2>(d3k);
    case 6: return pick_rd3k<float, 6, 1013, 4, 1024, 2>(d3k);
    case 7: return pick_rd3k<float, 7, 1013, 4, 1024, 2>(d3k);
    case 8: return pick_rd3k<float, 8, 1013, 4, 1024, 2>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
