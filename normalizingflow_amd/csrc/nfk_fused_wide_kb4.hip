// nfk_fused_wide_kb4.hip -- wide fused NSF layer kernel instances with H = 128
// (4 fp16 hidden k-blocks of 32); one TU per hidden width so make -j compiles them in parallel.
#include "nfk_fused_wide.h"

namespace nfk_fused {
NFK_WIDE_K(NFK_WIDE_INSTANCE, 4)
}  // namespace nfk_fused
