// kern_f32_d8.hip — float kernels, max column degree 8 (v1 atomic and v4 slot families).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
Variant get_variant_f32_d8(int vpl) { return pick_vpl<float, 8>(vpl); }
SVariant get_svariant_f32_d8(int ns) { return pick_sns<float, 8>(ns); }
}  // namespace qldpc
