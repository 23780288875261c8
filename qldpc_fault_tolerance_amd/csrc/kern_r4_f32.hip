// kern_r4_f32.hip — float kernels of engine 4 (c2v computed by the check phase, column degree <= 4).
#define QLDPC_VARIANT_TU 1
#include "variants.h"

namespace qldpc {
#if QLDPC_EXPERIMENTAL
SVariant get_r4variant_f32(int vpl) { return pick_rvpl<float, 4>(vpl); }
#else
// measured-and-not-kept family: built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)
SVariant get_r4variant_f32(int vpl) { return SVariant{nullptr, nullptr, nullptr, nullptr}; }
#endif
}  // namespace qldpc
