// kern_r4_f64.hip — double kernels of engine 4 (c2v computed by the check phase, column degree <= 4).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_r4variant_f64(int vpl) { return pick_rvpl<double, 4>(vpl); }
}  // namespace qldpc
