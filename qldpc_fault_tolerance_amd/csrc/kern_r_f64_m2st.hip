// kern_r_f64_m2st.hip — double kernels of engine 3 for the fp64 space-time graphs with the one-word
// "m2 in slot" check state (engine id 11313, + 100000 with D2K = 1; bp_reg.h eng_m2s): rows of 4
// 16-byte chunks + a tail slot, dword-scaled packed edge addresses, 1024-thread workgroups (128
// VGPRs), the own previous v2c in VGPRs instead of re-read from LDS, m1 | parity as the check
// state (8 B) and m2 | parity in the argmin edge's slot.  BASELINE config 5 (hgp_34_n1225_q3,
// num_rep 3: 1764 x 5439, rows of 8 / 9) is VPL 6, D2K 1, D3K 4: a 159.1 KB image with 1,348
// private dummy slots for the measurement / degree-3 variables in wider slots (round 6).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64_m2st(int vpl, int d3k, int d2k) {
  if (d2k < 1 || d3k < 1) return SVariant{nullptr, nullptr, nullptr, nullptr};
  switch (vpl) {
    case 5: return pick_rd3k<double, 5, 111313, 4, 1024, 4>(d3k);
    case 6: return pick_rd3k<double, 6, 111313, 4, 1024, 4>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
}  // namespace qldpc
