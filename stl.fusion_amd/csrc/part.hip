// part.hip — multi-GPU 1-D vertex-range partition with an RCCL all-to-all frontier exchange.
// (Filled in after the single-device path; until then the entry points report FGI_ENOTSUP.)
#include <hip/hip_runtime.h>

#include "fgi_internal.h"

namespace fgi {
fgi_status part_destroy(fgi_graph* g) {
    (void)g;
    return FGI_OK;
}
}  // namespace fgi

using namespace fgi;

extern "C" {

fgi_status fgi_part_unique_id(uint8_t* id128) {
    (void)id128;
    return FGI_ENOTSUP;
}
fgi_status fgi_part_init(fgi_graph* g, uint32_t n_global, const uint8_t* id128) {
    (void)n_global;
    (void)id128;
    return set_err(g, FGI_ENOTSUP, "multi-GPU partition not built");
}
fgi_status fgi_part_synth_rmat(fgi_graph* g, uint32_t, uint32_t, uint64_t, uint32_t, uint64_t) {
    return set_err(g, FGI_ENOTSUP, "multi-GPU partition not built");
}
fgi_status fgi_part_invalidate(fgi_graph* g, uint32_t, const uint32_t*, const uint8_t*, uint64_t*, fgi_wave_stats*) {
    return set_err(g, FGI_ENOTSUP, "multi-GPU partition not built");
}
fgi_status fgi_part_export_ids(fgi_graph* g, uint32_t*, uint64_t, uint64_t*) {
    return set_err(g, FGI_ENOTSUP, "multi-GPU partition not built");
}

}  // extern "C"
