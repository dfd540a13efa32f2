// nfk_fused_ht2.hip -- fused NSF layer kernel instances with 2 hidden tiles (H <= 32).
#include "nfk_fused_impl.h"

namespace nfk_fused {
#ifndef NFK_FUSED_DEV
NFK_FUSED_K(NFK_FUSED_INSTANCE, 2)
#elif 2 == 7
NFK_FUSED_INSTANCE(7, 8)
#endif
}  // namespace nfk_fused
