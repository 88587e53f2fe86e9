// amp_vamp_persist_h2.hip — the persistent VAMP engine with both per-iteration GEMMs in the
// split-precision fp16x2 form (amp_persist.h gemm_h2: per-row power-of-two scaled A operand,
// three fp16 MFMA products per product); its own translation unit so that it compiles in
// parallel with the f32 and bf16x3 instantiations.
#include "amp_vamp_persist_kernel.h"

namespace amp {

int persist_dispatch_h2(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.N) {
    case 64:   // as in the bf16x3 unit: the two-per-CU build for every N = 64 launch
        return persist_wg2() ? persist_launch_nt<2, 4, true, 2, true>(P, dc, st)
                             : AMP_DIAG_ONLY(persist_launch_nt<2, 4, true, 1, true>(P, dc, st));
    case 128: return persist_launch_nt<4, 4, true, 1, true>(P, dc, st);
    case 256: return persist_launch_nt<8, 4, true, 1, true>(P, dc, st);
    default: break;
    }
    set_error("vamp_persist (fp16x2): N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp
