// kern_r_f64_x.hip — double kernels of engine 3 for workgroups of 257-512 threads (engine id 303:
// own previous v2c in VGPRs, packed edge words, runtime-width check phase): 2 workgroups of
// 8 waves per CU within 128 VGPRs; every compile-time D3K in 0..VPL.  Opt-in (QLDPC_F64X=1).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
#if QLDPC_EXPERIMENTAL
SVariant get_rvariant_f64_x(int vpl, int d3k) {
  switch (vpl) {
    case 3: return pick_rd3k<double, 3, 303, 4, 512, 0>(d3k);
    case 4: return pick_rd3k<double, 4, 303, 4, 512, 0>(d3k);
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
#else
// measured-and-not-kept family: built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)
SVariant get_rvariant_f64_x(int vpl, int d3k) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
#endif
}  // namespace qldpc
