// amp_vamp_persist_i8.hip — the persistent VAMP engine with both per-iteration GEMMs in the
// split-precision int8x4 form (amp_persist.h gemm_i8: block fixed point on the integer matrix
// cores, per-row / per-column exponents); its own translation unit so that it compiles in parallel
// with the other instantiations.  One workgroup per CU at every N.
#include "amp_vamp_persist_kernel.h"

namespace amp {

static bool i8_waves8() {
    static const bool v = [] {
        const char* e = diag_env("AMP_VAMP_X3_WAVES");
        return !(e && atoi(e) == 4);
    }();
    return v;
}

int persist_dispatch_i8(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.N) {
    case 64: return persist_launch_nt<2, 4, true, 1, false, true>(P, dc, st);
    case 128: return persist_launch_nt<4, 4, true, 1, false, true>(P, dc, st);
    case 256:   // eight waves (two per SIMD) unless AMP_VAMP_X3_WAVES=4, as the bf16x3 engine
        return i8_waves8() ? persist_launch_nt<4, 8, true, 1, false, true>(P, dc, st)
                           : AMP_DIAG_ONLY(persist_launch_nt<8, 4, true, 1, false, true>(P, dc, st));
    default: break;
    }
    set_error("vamp_persist (int8x4): N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp
