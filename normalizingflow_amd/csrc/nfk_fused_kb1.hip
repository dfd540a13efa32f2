// nfk_fused_kb1.hip -- fused NSF layer kernel instances with 1 fp16 hidden k-blocks of 32
// (H = 32, or H = 33..36 with an f16 tail step).
#include "nfk_fused_impl.h"

namespace nfk_fused {
NFK_FUSED_K(NFK_FUSED_INSTANCE, 1, 0)
NFK_FUSED_K(NFK_FUSED_INSTANCE, 1, 1)
}  // namespace nfk_fused
