// nfk_fused_kb3.hip -- fused NSF layer kernel instances with 3 fp16 hidden k-blocks of 32
// (H = 96, or H = 97..100 with an f16 tail step).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 3, 0)
NFK_FUSED_K(NFK_FUSED_INSTANCE, 3, 1)
}  // namespace nfk_fused
