// amp_vamp_persist_x3f.hip — the persistent VAMP engine on the bf16x3 arithmetic with the operators
// streamed as plain f32 and split in registers (amp_persist.h gemm_x3f), eight waves per workgroup
// (two per SIMD); its own translation unit so that it compiles beside the other instantiations.
#include "amp_vamp_persist_kernel.h"

namespace amp {

// AMP_VAMP_X3F_WAVES = 4 | 8 (default 4): waves per workgroup (one or two per SIMD)
static int x3f_waves() {
    static const int w = [] {
        const char* e = getenv("AMP_VAMP_X3F_WAVES");
        return (e && atoi(e) == 8) ? 8 : 4;
    }();
    return w;
}

int persist_dispatch_x3f(const VampK& P, const DecConst& dc, hipStream_t st) {
    if (x3f_waves() == 8) {
        switch (P.N) {
        case 128: return persist_launch_nt<2, 8, true, 1, false, true>(P, dc, st);
        case 256: return persist_launch_nt<4, 8, true, 1, false, true>(P, dc, st);
        default: break;
        }
    } else {
        switch (P.N) {
        case 128: return persist_launch_nt<4, 4, true, 1, false, true>(P, dc, st);
        case 256: return persist_launch_nt<8, 4, true, 1, false, true>(P, dc, st);
        default: break;
        }
    }
    set_error("vamp_persist (bf16x3, f32-streamed operators): N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp
