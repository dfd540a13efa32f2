// nfk_fused_ksh16.hip -- fused NSF layer kernel instances with 16 hidden k-steps (H <= 64).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 16)
}  // namespace nfk_fused
