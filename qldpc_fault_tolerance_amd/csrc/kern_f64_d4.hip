// kern_f64_d4.hip — double kernels, max column degree 4.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f64_d4(int vpl) { return pick_vpl<double, 4>(vpl); }
}  // namespace qldpc
