// kern_r_f64.hip — double kernels of engine 3 (register-resident variables, column degree <= 4).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
SVariant get_rvariant_f64(int vpl) { return pick_rvpl<double, 3>(vpl); }
}  // namespace qldpc
