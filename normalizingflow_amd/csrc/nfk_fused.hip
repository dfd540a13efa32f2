// nfk_fused.hip -- fused NSF coupling layer (MLP conditioner on fp32 MFMA +
// spline epilogue).  Placeholder until the MFMA kernel lands: reports every
// shape as unsupported so the host layer takes the streaming path.
#include <hip/hip_runtime.h>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);

extern "C" int nfk_fused_nsf_supported(int32_t, int32_t, int32_t, int32_t) { return 0; }
extern "C" int64_t nfk_fused_nsf_pack_elems(int32_t, int32_t, int32_t, int32_t) { return 0; }
extern "C" int nfk_fused_nsf_pack(const float*, const float*, const float*, const float*,
                                  const float*, const float*, int32_t, int32_t, int32_t, int32_t,
                                  float*, nfk_stream_t) {
    return nfk_set_error("nfk_fused_nsf_pack: shape not supported");
}
extern "C" int nfk_fused_nsf(const float*, int64_t, const float*, const int32_t*, const int32_t*,
                             int32_t, const int32_t*, const int32_t*, int32_t, int32_t, float*,
                             int64_t, float*, int32_t, int64_t, int32_t, double, int32_t, int32_t*,
                             nfk_stream_t) {
    return nfk_set_error("nfk_fused_nsf: shape not supported");
}
