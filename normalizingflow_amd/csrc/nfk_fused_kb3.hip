// nfk_fused_kb3.hip -- fused NSF layer kernel instances with 3 hidden k-blocks of 32 (H <= 96).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 3)
}  // namespace nfk_fused
