// ppoly.hip -- placeholder until the point-polygon kernels land.
#include "join.h"
#include "ppoly.h"

namespace geohip {
int ppoly_impl(geohip_ctx* ctx, const geohip_grid*, const double*, const double*, uint64_t, const uint32_t*,
               const double*, const double*, uint32_t, double, int, uint32_t*, uint64_t, uint64_t*) {
    return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "point-polygon range not built yet");
}
}  // namespace geohip
