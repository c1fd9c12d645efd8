// join.hip -- placeholder until the cell-pair join kernels land.
#include "join.h"

namespace geohip {
int join_pp_impl(geohip_ctx* ctx, const geohip_grid*, const geohip_grid*, const double*, const double*, uint64_t,
                 const double*, const double*, uint64_t, double, int, uint32_t*, uint64_t, uint64_t*, bool) {
    return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "join not built yet");
}
}  // namespace geohip
