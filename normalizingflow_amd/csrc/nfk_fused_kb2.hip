// nfk_fused_kb2.hip -- fused NSF layer kernel instances with 2 fp16 hidden k-blocks of 32
// (H = 64, or H = 65..68 with an f16 tail step).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 2, 0)
NFK_FUSED_K(NFK_FUSED_INSTANCE, 2, 1)
}  // namespace nfk_fused
