// amp_scamp_persist_h2.hip — the persistent SCAMP engine with both per-iteration GEMMs in the
// split-precision fp16x2 form (amp_persist.h gemm_h2); its own translation unit so the
// instantiations compile in parallel.
#include "amp_scamp_persist_kernel.h"

namespace amp {

int scamp_persist_launch_h2(const ScampK& P, const DecConst& c64, hipStream_t st) {
    const int twoN = 2 * P.N, twon = 2 * P.n;
    if (twoN == 128 && twon == 256) return spersist_launch_s<4, 8, 2, 16, true, true>(P, c64, st);
    if (twoN == 256 && twon == 512) return spersist_launch_s<8, 16, 4, 32, true, true>(P, c64, st);
    if (twoN == 256 && twon == 256) return spersist_launch_s<4, 16, 4, 16, true, true>(P, c64, st);
    set_error("scamp_persist (fp16x2): (2N, 2n) = (%d, %d) not supported", twoN, twon);
    return AMP_E_ARG;
}

}  // namespace amp
