// nfk_fused_wide_kb8.hip -- wide fused NSF layer kernel instances with H = 256
// (8 fp16 hidden k-blocks of 32); one TU per hidden width so make -j compiles them in parallel.
#include "nfk_fused_wide.h"

namespace nfk_fused {
NFK_WIDE_K(NFK_WIDE_INSTANCE, 8)
}  // namespace nfk_fused
