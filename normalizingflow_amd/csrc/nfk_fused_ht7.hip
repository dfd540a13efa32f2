// nfk_fused_ht7.hip -- fused NSF layer kernel instances with 7 hidden tiles (H <= 112).
#include "nfk_fused_impl.h"

namespace nfk_fused {
#ifndef NFK_FUSED_DEV
NFK_FUSED_K(NFK_FUSED_INSTANCE, 7)
#elif 7 == 7
NFK_FUSED_INSTANCE(7, 8)
#endif
}  // namespace nfk_fused
