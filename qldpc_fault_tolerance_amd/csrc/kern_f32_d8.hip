// kern_f32_d8.hip — float kernels, max column degree 8.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f32_d8(int vpl) { return pick_vpl<float, 8>(vpl); }
}  // namespace qldpc
