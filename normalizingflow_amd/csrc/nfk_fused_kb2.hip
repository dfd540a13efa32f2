// nfk_fused_kb2.hip -- fused NSF layer kernel instances with 2 hidden k-blocks of 32 (H <= 64).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 2)
}  // namespace nfk_fused
