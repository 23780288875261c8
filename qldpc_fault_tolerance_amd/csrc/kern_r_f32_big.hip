// kern_r_f32_big.hip — float kernels of engine 3 with dword-scaled edge
// addresses (kernel id 13): LDS images of 64-256 KiB, e.g. the space-time graphs
// (hgp_34_n1225_q3, num_rep 3: 1764 x 5439, one 1024-thread workgroup per CU).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_big(int vpl, int d3k) {
  switch (vpl) {
    case 3: return pick_rd3k<float, 3, 13>(d3k);
    case 4: return pick_rd3k<float, 4, 13>(d3k);
    case 5: return pick_rd3k<float, 5, 13>(d3k);
    case 6: return pick_rd3k<float, 6, 13>(d3k);
    case 7: return pick_rd3k<float, 7, 13>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
