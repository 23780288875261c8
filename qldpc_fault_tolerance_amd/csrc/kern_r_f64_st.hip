// kern_r_f64_st.hip — double kernels of engine 3 for the tail layout (engine id 1013):
// rows of 4 16-byte chunks plus one tail slot per row, dword-scaled edge addresses,
// 1024-thread workgroups.  The fp64 space-time graphs (hgp_34_n1225_q3, num_rep 3:
// 1764 x 5439, rows of 8 / 9 edges) fit one CU's LDS this way (162 KB image instead
// of 176 KB with 5-chunk rows).  VPL 4-6 here, 7-8 in kern_r_f64_st_hi.hip.  VPL 6 (config 5) also
// with D2K = 1 (engine id 101013): its first slot holds 1024 of the degree-2 measurement variables
// with two edge slots instead of three.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_st(int vpl, int d3k, int d2k) {
  if (vpl == 6 && d2k >= 1 && d3k >= 1) return pick_rd3k<double, 6, 101013, 4, 1024, 4>(d3k);
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 1013, 4, 1024, 4>(d3k);
    case 5: return pick_rd3k<double, 5, 1013, 4, 1024, 4>(d3k);
    case 6: return pick_rd3k<double, 6, 1013, 4, 1024, 4>(d3k);
    default: return get_rvariant_f64_st_hi(vpl, d3k);
  }
}
}  // namespace qldpc
