// kern_r_f32_stfb.hip — float kernels of engine 3 for the tail layout with byte F words (engine
// id 21013, bp_reg.h eng_fb): rows of 2 16-byte chunks plus a tail slot, dword-scaled edge
// addresses, 512-thread workgroups with 9-12 variables per thread, 128 VGPRs.  Config 5's fp32
// space-time graphs (1764 x 5439) fit a 79.6 KB image this way: two decodes share a CU instead
// of one 1024-thread decode per CU.  D2K (engine id + 100000 * D2K, 1-4 with D3K = 8): the first
// slots hold the degree-2 measurement variables with two edge slots (host degree sort).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
template <int VPL>
SVariant stfb_d2k(int d3k, int d2k) {
  if (d3k >= 8 && VPL >= 8) {
    switch (d2k) {
      case 1: return make_rvariant<float, VPL, 121013, (8 <= VPL ? 8 : 0), 4, 512, 2>();
      case 2: return make_rvariant<float, VPL, 221013, (8 <= VPL ? 8 : 0), 4, 512, 2>();
      case 3: return make_rvariant<float, VPL, 321013, (8 <= VPL ? 8 : 0), 4, 512, 2>();
      case 4: return make_rvariant<float, VPL, 421013, (8 <= VPL ? 8 : 0), 4, 512, 2>();
      default: break;
    }
  }
  return pick_rd3k<float, VPL, 21013, 4, 512, 2>(d3k);
}
SVariant get_rvariant_f32_stfb(int vpl, int d3k, int d2k) {
  if (d2k > 4) d2k = 4;
  switch (vpl) {
    case 9: return stfb_d2k<9>(d3k, d2k);
    case 10: return stfb_d2k<10>(d3k, d2k);
    case 11: return stfb_d2k<11>(d3k, d2k);
    case 12: return stfb_d2k<12>(d3k, d2k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
