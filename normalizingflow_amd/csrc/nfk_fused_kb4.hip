// nfk_fused_kb4.hip -- fused NSF layer kernel instances with 4 hidden k-blocks of 32 (H <= 128).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 4)
}  // namespace nfk_fused
