// nfk_fused_kb4.hip -- fused NSF layer kernel instances with 4 fp16 hidden k-blocks of 32
// (H = 128, or H = 129..132 with an f16 tail step).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 4, 0)
NFK_FUSED_K(NFK_FUSED_INSTANCE, 4, 1)
}  // namespace nfk_fused
