// nfk_fused_ksh25.hip -- fused NSF layer kernel instances with 25 hidden k-steps (H <= 100).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 25)
}  // namespace nfk_fused
