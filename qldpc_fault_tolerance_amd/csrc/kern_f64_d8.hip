// kern_f64_d8.hip — double kernels, max column degree 8.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f64_d8(int vpl) { return pick_vpl<double, 8>(vpl); }
}  // namespace qldpc
