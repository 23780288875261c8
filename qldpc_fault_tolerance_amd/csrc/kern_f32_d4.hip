// kern_f32_d4.hip — float kernels, max column degree 4.
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f32_d4(int vpl) { return pick_vpl<float, 4>(vpl); }
}  // namespace qldpc
