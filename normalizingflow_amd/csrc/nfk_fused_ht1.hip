// nfk_fused_ht1.hip -- fused NSF layer kernel instances with 1 hidden tiles (H <= 16).
#include "nfk_fused_impl.h"

namespace nfk_fused {
#ifndef NFK_FUSED_DEV
NFK_FUSED_K(NFK_FUSED_INSTANCE, 1)
#elif 1 == 7
NFK_FUSED_INSTANCE(7, 8)
#endif
}  // namespace nfk_fused
