// amp_scamp_persist_x3.hip — the persistent SCAMP engine with both per-iteration GEMMs on the
// split-precision bf16x3 engine (amp_persist.h gemm_x3); its own translation unit so the f32 and
// bf16x3 instantiations compile in parallel.
#include "amp_scamp_persist_kernel.h"

namespace amp {

static bool scamp_waves8() {
    static const bool v = [] {
        const char* e = diag_env("AMP_SCAMP_X3_WAVES");
        return !(e && atoi(e) == 4);
    }();
    return v;
}

int scamp_persist_launch_x3(const ScampK& P, const DecConst& c64, hipStream_t st) {
    const int twoN = 2 * P.N, twon = 2 * P.n;
    if (twoN == 128 && twon == 256) return spersist_launch_s<4, 8, 2, 16, true>(P, c64, st);
    // cfg3's shape: eight waves (two per SIMD) unless AMP_SCAMP_X3_WAVES=4 (A/B runs)
    if (twoN == 256 && twon == 512)
        return scamp_waves8() ? spersist_launch_s<4, 16, 2, 32, true, false, 8>(P, c64, st)
                              : AMP_DIAG_ONLY(spersist_launch_s<8, 16, 4, 32, true>(P, c64, st));
    if (twoN == 256 && twon == 256) return spersist_launch_s<4, 16, 4, 16, true>(P, c64, st);
    set_error("scamp_persist (bf16x3): (2N, 2n) = (%d, %d) not supported", twoN, twon);
    return AMP_E_ARG;
}

}  // namespace amp
