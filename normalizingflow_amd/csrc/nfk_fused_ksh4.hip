// nfk_fused_ksh4.hip -- fused NSF layer kernel instances with 4 hidden k-steps (H <= 16).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 4)
}  // namespace nfk_fused
