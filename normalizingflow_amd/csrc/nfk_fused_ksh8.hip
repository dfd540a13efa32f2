// nfk_fused_ksh8.hip -- fused NSF layer kernel instances with 8 hidden k-steps (H <= 32).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 8)
}  // namespace nfk_fused
