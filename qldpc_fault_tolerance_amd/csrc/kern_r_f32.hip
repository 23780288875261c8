// kern_r_f32.hip — float kernels of engine 3 (register-resident variables, column degree <= 4).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f32(int vpl) { return pick_rvpl<float, 3>(vpl); }
}  // namespace qldpc
