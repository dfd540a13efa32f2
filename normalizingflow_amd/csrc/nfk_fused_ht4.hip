// nfk_fused_ht4.hip -- fused NSF layer kernel instances with 4 hidden tiles (H <= 64).
#include "nfk_fused_impl.h"

namespace nfk_fused {
#ifndef NFK_FUSED_DEV
NFK_FUSED_K(NFK_FUSED_INSTANCE, 4)
#elif 4 == 7
NFK_FUSED_INSTANCE(7, 8)
#endif
}  // namespace nfk_fused
