// amp_gemm.h — fp32 MFMA tile engine for the batched complex mat-vecs.
//
// Every per-iteration product of the detectors is   C[B x Nc] = A[B x Ka] . Wt[Nc x Ka]^T
// with A = one trial per row (the reference's [B, len, 1] batch of vectors, complex
// interleaved {re, im}) and Wt a weight matrix expanded ONCE per forward:
//   complex y = X x   ->  Wt[2o][2j] = Re X, Wt[2o][2j+1] = -Im X,
//                         Wt[2o+1][2j] = Im X, Wt[2o+1][2j+1] = Re X
// so the complex GEMM is a real GEMM whose A rows are the c64 vectors as they lie in
// memory and whose output rows come out interleaved re/im again (8 real flops per
// complex MAC: nothing is wasted).  One H/V is shared by all B trials,
// so this is a true GEMM and runs on v_mfma_f32_32x32x2_f32 (exact f32, 64 flop/clk/SIMD).
//
// Tile: BM = 32 trials x BN (128 | 256) output columns, 4 waves side by side in N,
// BK = 32.  Both operand tiles are staged K-contiguous in LDS (row stride 36 floats:
// conflict-free ds_read_b128 for the 16-lane groups), double-buffered with register
// prefetch (one barrier per K step).  K is split between the two wave halves
// (lanes 0-31 take k in [0,16), lanes 32-63 k in [16,32) of each K step) so each lane
// feeds four MFMAs from one ds_read_b128 per operand.
//
// The accumulators are written to an LDS C tile [32][BN+4] that aliases the staging
// buffers, where the caller's fused epilogue (LMMSE step, Onsager update, section
// denoiser, ...) reads whole rows/sections.
#pragma once

#include "amp_common.h"

namespace amp {

constexpr int GBM = 32;
constexpr int GBK = 32;
constexpr int GLDK = GBK + 4;

template <int BN>
struct GemmCfg {
    static_assert(BN == 128 || BN == 256, "BN must be 128 or 256");
    static constexpr int NACC = BN / 128;                 // 32x32 accumulators per wave
    static constexpr int WN = BN / 4;                     // columns per wave
    static constexpr int WLD = BN * (GBK / 4) / AMP_WG;   // W float4 per thread per K step
    static constexpr int LDC = BN + 4;                    // C tile row stride (floats)
    static constexpr int STAGE_FLOATS = 2 * (GBM + BN) * GLDK;
    static constexpr int CTILE_FLOATS = GBM * LDC;
    static constexpr int LDS_FLOATS = STAGE_FLOATS > CTILE_FLOATS ? STAGE_FLOATS : CTILE_FLOATS;
    static constexpr size_t LDS_BYTES = (size_t)LDS_FLOATS * 4;
};

// Plain A operand: rows of `lda` floats, `ka` valid columns (zero beyond, and for rows >= rows).
struct ALoadPlain {
    const float* __restrict__ a;
    int lda, rows, ka;
    __device__ __forceinline__ float4 operator()(int row, int k) const {
        if (row >= rows || k >= ka) return make_float4(0.f, 0.f, 0.f, 0.f);
        return *reinterpret_cast<const float4*>(a + (size_t)row * lda + k);
    }
};

// Computes the C tile of rows [row0, row0+32) x cols [col0, col0+BN) into `lds` (as the C
// tile, row stride GemmCfg<BN>::LDC).  `wt` is [Ncp][kap] with kap % 32 == 0 and col0+BN <= Ncp.
template <int BN, class AL>
__device__ __forceinline__ void gemm_tile(const AL& al, const float* __restrict__ wt, int kap, int row0,
                                          int col0, float* lds) {
    using C = GemmCfg<BN>;
    float* As = lds;
    float* Ws = lds + 2 * GBM * GLDK;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;

    f32x16 acc[C::NACC];
#pragma unroll
    for (int j = 0; j < C::NACC; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    const int ar = tid >> 3, akq = (tid & 7) * 4;
    int woff[C::WLD], wlds[C::WLD];
#pragma unroll
    for (int j = 0; j < C::WLD; ++j) {
        const int idx = tid + j * AMP_WG;
        woff[j] = (col0 + (idx >> 3)) * kap + (idx & 7) * 4;
        wlds[j] = (idx >> 3) * GLDK + (idx & 7) * 4;
    }
    float4 ra = al(row0 + ar, akq);
    float4 rw[C::WLD];
#pragma unroll
    for (int j = 0; j < C::WLD; ++j) rw[j] = *reinterpret_cast<const float4*>(wt + woff[j]);
    *reinterpret_cast<float4*>(As + ar * GLDK + akq) = ra;
#pragma unroll
    for (int j = 0; j < C::WLD; ++j) *reinterpret_cast<float4*>(Ws + wlds[j]) = rw[j];
    __syncthreads();

    const int nk = kap / GBK;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        // prefetch the next K step (the last step re-reads its own tile: no branch, so the
        // prefetch registers stay registers)
        const int k0 = min(kt + 1, nk - 1) * GBK;
        ra = al(row0 + ar, k0 + akq);
#pragma unroll
        for (int j = 0; j < C::WLD; ++j) rw[j] = *reinterpret_cast<const float4*>(wt + woff[j] + k0);
        const float* a_s = As + cur * GBM * GLDK + li * GLDK + lh * 16;
        const float* w_s = Ws + cur * BN * GLDK + (wave * C::WN + li) * GLDK + lh * 16;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const float4 a4 = *reinterpret_cast<const float4*>(a_s + s4 * 4);
#pragma unroll
            for (int j = 0; j < C::NACC; ++j) {
                const float4 b4 = *reinterpret_cast<const float4*>(w_s + j * 32 * GLDK + s4 * 4);
                acc[j] = mfma32x32x2(a4.x, b4.x, acc[j]);
                acc[j] = mfma32x32x2(a4.y, b4.y, acc[j]);
                acc[j] = mfma32x32x2(a4.z, b4.z, acc[j]);
                acc[j] = mfma32x32x2(a4.w, b4.w, acc[j]);
            }
        }
        const int nb = cur ^ 1;
        *reinterpret_cast<float4*>(As + nb * GBM * GLDK + ar * GLDK + akq) = ra;
#pragma unroll
        for (int j = 0; j < C::WLD; ++j) *reinterpret_cast<float4*>(Ws + nb * BN * GLDK + wlds[j]) = rw[j];
        __syncthreads();
    }
    // accumulators -> LDS C tile (aliases the staging buffers; the loop ended on a barrier)
    float* ct = lds;
#pragma unroll
    for (int j = 0; j < C::NACC; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            const int col = wave * C::WN + j * 32 + li;
            ct[row * C::LDC + col] = acc[j][r];
        }
    __syncthreads();
}

}  // namespace amp
