// kern_r_f64_m2v.hip — double kernels of engine 3, "m2 in slot" with variable-major V slots
// (engine id 40103, bp_reg.h eng_m2v): 256-thread workgroups, one-word check state, m2 | parity in
// the argmin edge's V slot as m2s, but the V slots laid out [variable slot][edge][lane] so the
// variable phase's slot reads and v2c stores are lane-linear; the check phase gathers its rows
// through a per-thread register table.  3 workgroups per CU (168 VGPRs).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
#if QLDPC_EXPERIMENTAL
SVariant get_rvariant_f64_m2v(int vpl, int d3k) {
  switch (vpl) {
    case 4: return pick_rd3k<double, 4, 40103, 4, 256, 3>(d3k);
    case 5: return pick_rd3k<double, 5, 40103, 4, 256, 3>(d3k);
    case 6: return pick_rd3k<double, 6, 40103, 4, 256, 3>(d3k);
    case 7: return pick_rd3k<double, 7, 40103, 4, 256, 3>(d3k);
    case 8: return pick_rd3k<double, 8, 40103, 4, 256, 3>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
#else
// measured-and-not-kept family: built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)
SVariant get_rvariant_f64_m2v(int vpl, int d3k) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
#endif
}  // namespace qldpc
