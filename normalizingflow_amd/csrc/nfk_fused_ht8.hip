// nfk_fused_ht8.hip -- fused NSF layer kernel instances with 8 hidden tiles (H <= 128).
#include "nfk_fused_impl.h"

namespace nfk_fused {
#ifndef NFK_FUSED_DEV
NFK_FUSED_K(NFK_FUSED_INSTANCE, 8)
#elif 8 == 7
NFK_FUSED_INSTANCE(7, 8)
#endif
}  // namespace nfk_fused
