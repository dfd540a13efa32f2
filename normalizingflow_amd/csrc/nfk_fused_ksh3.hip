// nfk_fused_ksh3.hip -- fused NSF layer kernel instances with 3 hidden k-steps (H <= 12).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 3)
}  // namespace nfk_fused
