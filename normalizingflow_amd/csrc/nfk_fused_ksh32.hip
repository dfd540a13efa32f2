// nfk_fused_ksh32.hip -- fused NSF layer kernel instances with 32 hidden k-steps (H <= 128).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 32)
}  // namespace nfk_fused
