// kern_r_f32_stfb.hip — float kernels of engine 3 for the tail layout with byte F words (engine
// id 21013, bp_reg.h eng_fb): rows of 2 16-byte chunks plus a tail slot, dword-scaled edge
// addresses, 512-thread workgroups with 9-12 variables per thread, 128 VGPRs.  Config 5's fp32
// space-time graphs (1764 x 5439) fit a 79.6 KB image this way: two decodes share a CU instead
// of one 1024-thread decode per CU.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32_stfb(int vpl, int d3k) {
  switch (vpl) {
    case 9: return pick_rd3k<float, 9, 21013, 4, 512, 2>(d3k);
    case 10: return pick_rd3k<float, 10, 21013, 4, 512, 2>(d3k);
    case 11: return pick_rd3k<float, 11, 21013, 4, 512, 2>(d3k);
    case 12: return pick_rd3k<float, 12, 21013, 4, 512, 2>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
