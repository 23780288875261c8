// kern_r_f32_w.hip — float kernels of engine 3 with the compile-time 2-chunk check phase
// (rows of <= 8 edges: prefetched rows, no chunk loop) for VPL 5-8, every compile-time D3K.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_w(int vpl, int d3k) {
  switch (vpl) {
    case 5: return pick_rd3k<float, 5, 3, 4, kMaxThreadsS, 2>(d3k);
    case 6: return pick_rd3k<float, 6, 3, 4, kMaxThreadsS, 2>(d3k);
    case 7: return pick_rd3k<float, 7, 3, 4, kMaxThreadsS, 2>(d3k);
    case 8: return pick_rd3k<float, 8, 3, 4, kMaxThreadsS, 2>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
