// amp_vamp_persist_x3.hip — the persistent VAMP engine with both per-iteration GEMMs on the
// split-precision bf16x3 engine (amp_persist.h gemm_x3); its own translation unit so that the
// f32 and bf16x3 instantiations of vamp_persist compile in parallel.  One wave per SIMD.
#include "amp_vamp_persist_kernel.h"

namespace amp {

int persist_dispatch_x3(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.N) {
    case 64:   // the two-per-CU build for every N = 64 launch, so that one epoch and side-by-side
               // epochs run the same arithmetic (bit-identical results, tests/test_gpu_epochs.py)
        return persist_wg2() ? persist_launch_nt<2, 4, true, 2>(P, dc, st) : persist_launch_nt<2, 4, true>(P, dc, st);
    case 128: return persist_launch_nt<4, 4, true>(P, dc, st);
    case 256: return persist_launch_nt<8, 4, true>(P, dc, st);
    default: break;
    }
    set_error("vamp_persist (bf16x3): N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp
