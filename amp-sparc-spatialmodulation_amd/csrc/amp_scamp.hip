// amp_scamp.hip — SCAMP detector (placeholder until the fused kernels land).
#include "amp_host.h"
using namespace amp;
extern "C" {
size_t amp_scamp_workspace_bytes(const amp_dims* d, int32_t max_iter) { return (d && max_iter > 0) ? 256 : 0; }
int amp_scamp_run(const amp_dims*, const amp_constellation*, const amp_scamp_args*, void*) {
    set_error("amp_scamp_run: not implemented yet");
    return AMP_E_ARG;
}
}
