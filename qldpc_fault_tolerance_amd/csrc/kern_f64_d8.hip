// kern_f64_d8.hip — double kernels, max column degree 8 (v1 atomic and v4 slot families).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f64_d8(int vpl) { return pick_vpl<double, 8>(vpl); }
SVariant get_svariant_f64_d8(int ns) { return pick_sns<double, 8>(ns); }
}  // namespace qldpc
