// amp_scamp_persist.hip — persistent SCAMP engine: the whole iteration loop of SCAMP.forward
// (scamp.py:77-107) in ONE launch.
//
// Each workgroup (256 threads, one wave per SIMD, one workgroup per CU) owns PB = 16 trials for
// the whole forward; their state lives in LDS across iterations: xmmse (x), xmap, z, the GEMM2
// operand s = z / phi, psi (this and the previous iteration), phi, and the per-row coupling
// scalars.  Per iteration t (same arithmetic, element by element, as amp_scamp.hip):
//   1. per (trial, row block lo): gamma = W psi / Lc, b = gamma / phi_old, phi = sigma2 + gamma
//      (scamp.py:45-51); per (trial, column block lc): tau = L / (W^T (1/phi)) / Mr (scamp.py:53)
//   2. GEMM1 A x on v_mfma_f32_16x16x4_f32 (A 16x16x4-packed, streamed from L2) with the
//      epilogue z = y - A x + b z, s = z / phi  (scamp.py:47-49, 57)
//   3. GEMM2 A^H s, epilogue xmap = x + tau (A^H s)  (scamp.py:55-57)
//   4. the mean-only section denoiser on xmap (tau/2, scamp.py:61-68) -> x, and
//      psi = 1 - sum_block |x|^2 / Na with its allclose count (scamp.py:59, 105)
//   5. the batch-global exchange (amp_persist.h granules): max|xi|, the danger test of the
//      float64 softmax, and the allclose count; the rare exact float64 path (amp_denoise.h) takes
//      two bounded grid barriers, uniformly in every workgroup.
// Launch-engine parity: the same f32 operations in the same order per element, so the only
// differences are the GEMM summation order (16x16x4 vs 32x32x2 MFMA) and psi's float64 sum
// order — the summation-order noise the curve tests accept.
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "amp_scamp_persist_kernel.h"

namespace amp {

bool scamp_persist_x3_fits(const amp_dims* d) {
    return (size_t)slayout(d->N, d->n, d->L, d->Lin, d->Lout, true).total * 4 + 1024 <= 160 * 1024;
}

bool scamp_persist_eligible(const amp_dims* d, int ncu) {
    const int twoN = 2 * d->N, twon = 2 * d->n;
    const bool shape = (twoN == 128 && twon == 256) || (twoN == 256 && twon == 512) || (twoN == 256 && twon == 256);
    if (!shape || d->M > 64 || d->Lin > SMAXLIN || d->Lout > SMAXLIN || !is_pow2(d->N / d->M)) return false;
    if (ncu <= 0 || cdiv(d->B, SPB) > ncu) return false;
    return (size_t)slayout(d->N, d->n, d->L, d->Lin, d->Lout).total * 4 + 1024 <= 160 * 1024;
}

// NT1 = 2n / 64 column tiles per wave (GEMM1, K = 2N = 16 G1); NT2 = 2N / 64 (GEMM2, K = 2n)
int scamp_persist_launch_x3(const ScampK& P, const DecConst& c64, hipStream_t st);   // amp_scamp_persist_x3.hip
int scamp_persist_launch_h2(const ScampK& P, const DecConst& c64, hipStream_t st);   // amp_scamp_persist_h2.hip

int scamp_persist_launch(const ScampK& P, const DecConst& c64, hipStream_t st) {
    if (P.x3 == 2) return scamp_persist_launch_h2(P, c64, st);
    if (P.x3) return scamp_persist_launch_x3(P, c64, st);
    const int twoN = 2 * P.N, twon = 2 * P.n;
    if (twoN == 128 && twon == 256) return spersist_launch_s<4, 8, 2, 16, false>(P, c64, st);
    if (twoN == 256 && twon == 512) return spersist_launch_s<8, 16, 4, 32, false>(P, c64, st);
    if (twoN == 256 && twon == 256) return spersist_launch_s<4, 16, 4, 16, false>(P, c64, st);
    set_error("scamp_persist: (2N, 2n) = (%d, %d) not supported", twoN, twon);
    return AMP_E_ARG;
}

}  // namespace amp
