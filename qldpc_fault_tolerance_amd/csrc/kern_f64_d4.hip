// kern_f64_d4.hip — double kernels, max column degree 4 (v1 atomic and v4 slot families).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f64_d4(int vpl) { return pick_vpl<double, 4>(vpl); }
SVariant get_svariant_f64_d4(int ns) { return pick_sns<double, 4>(ns); }
}  // namespace qldpc
