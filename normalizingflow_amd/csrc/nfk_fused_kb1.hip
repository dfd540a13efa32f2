// nfk_fused_kb1.hip -- fused NSF layer kernel instances with 1 hidden k-blocks of 32 (H <= 32).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 1)
}  // namespace nfk_fused
