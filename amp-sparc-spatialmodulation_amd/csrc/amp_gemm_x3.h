// amp_gemm_x3.h — the launch engines' split-precision bf16x3 GEMM tile (BAMP's four
// per-iteration products, bamp.py:59-64), the 24-bit counterpart of amp_gemm_h2.h's fp16x2 tile.
//
// Same contract as gemm_tile<BN> / gemm_tile_h2<BN>: C[32 trials x BN real columns] lands in LDS
// as the f32 C tile (row stride GemmCfg<BN>::LDC; complex outputs interleaved re / im), so the
// fused epilogues are unchanged.  The arithmetic is amp_persist.h's bf16x3 form (gemm_x3):
//  * the A operand rows are split ONCE per GEMM by x3_split_rows_kernel into three bf16 pieces per
//    value in global memory ([plane][row][k]; complex: Re x0 x1 x2, Im x0 x1 x2; real: x0 x1 x2) —
//    every column tile then reuses them.  bf16 keeps f32's exponent range: no scaling, so unlike
//    fp16x2 there is no operator magnitude limit;
//  * the operator is packed by x3_index (complex, six planes) / x3r_index (real, three planes);
//  * per product the six terms a0w0 a0w1 a1w0 a0w2 a1w1 a2w0 (every dropped term <= 2^-24 of the
//    product: the reference's c64 operand precision) on v_mfma_f32_16x16x32_bf16, smallest terms
//    first, f32 accumulation; two row blocks of 16 trials per wave share each weight fragment.
// The A planes are staged through LDS in chunks of X3KC elements in the XOR-permuted plane layout
// (pl_col), one chunk ahead; the weights stream from L2 in a two-group register ring.  A block-banded operator
// (the ISI channel) reduces each tile over [kb, ke) only (h2_kband on the packed planes).
#pragma once

#include "amp_gemm.h"
#include "amp_persist.h"

namespace amp {

constexpr int X3KC = 128;           // A elements (complex or real) per staged chunk
constexpr int X3SWM = 15;           // chunk permutation mask (pl_col): rows of 128 bf16

// bytes of LDS gemm_tile_x3<BN, CPX> needs: the staged planes, or the C tile (which aliases them)
// plus `extra` floats of the caller's epilogue scratch past it, whichever is larger
template <int BN, bool CPX>
constexpr size_t x3_tile_lds(size_t extra) {
    constexpr size_t planes = (size_t)(CPX ? 6 : 3) * GBM * X3KC * 2;
    const size_t ct = ((size_t)GemmCfg<BN>::CTILE_FLOATS + extra) * 4;
    return planes > ct ? planes : ct;
}

// Split rows [0, rows_pad) of a (row stride lda floats; rows >= rows are zero) into bf16 planes
// planes[f][row][k] (k < K, plane stride rows_pad * K): wpr wavefronts per row (1: four rows per
// workgroup; 4: a workgroup per row, for long rows); complex rows (CPX) hold K interleaved values,
// real rows K floats.  K % 8 == 0.  `stopped` (optional): the iteration record's stop word, which
// turns the launch into a no-op.
template <bool CPX>
__global__ __launch_bounds__(256) void x3_split_rows_kernel(const float* __restrict__ a, int lda, int rows,
                                                            int rows_pad, int K, unsigned short* __restrict__ planes,
                                                            const int* __restrict__ stopped, int wpr) {
    if (stopped && *stopped) return;                     // the detector's loop has stopped (no-op launch)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row = blockIdx.x * (4 / wpr) + wave / wpr;
    const int t = (wave % wpr) * 64 + lane, nt = 64 * wpr;
    if (row >= rows_pad) return;
    const bool in = row < rows;
    const float* ar = a + (size_t)(in ? row : 0) * lda;
    constexpr int FPE = CPX ? 2 : 1;                   // floats per element
    constexpr int PL = CPX ? 6 : 3;
    const size_t ps = (size_t)rows_pad * K;            // plane stride (elements)
    unsigned short* pr = planes + (size_t)row * K;
    for (int j0 = 8 * t; j0 < K; j0 += 8 * nt) {      // 8 elements per thread and step
        float re[8], im[8];
        float4 v[2 * FPE];
#pragma unroll
        for (int h = 0; h < 2 * FPE; ++h)
            v[h] = in ? *reinterpret_cast<const float4*>(ar + FPE * j0 + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int h = 0; h < 2 * FPE; ++h) {
            if (CPX) {
                re[2 * h] = v[h].x; im[2 * h] = v[h].y; re[2 * h + 1] = v[h].z; im[2 * h + 1] = v[h].w;
            } else {
                re[4 * h] = v[h].x; re[4 * h + 1] = v[h].y; re[4 * h + 2] = v[h].z; re[4 * h + 3] = v[h].w;
            }
        }
        u32x4 q[PL];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            unsigned a0, a1, a2;
            split3x2(re[2 * h], re[2 * h + 1], a0, a1, a2);
            q[0][h] = a0; q[1][h] = a1; q[2][h] = a2;
            if constexpr (CPX) {
                unsigned b0, b1, b2;
                split3x2(im[2 * h], im[2 * h + 1], b0, b1, b2);
                q[3][h] = b0; q[4][h] = b1; q[5][h] = b2;
            }
        }
#pragma unroll
        for (int f = 0; f < PL; ++f) *reinterpret_cast<u32x4*>(pr + f * ps + j0) = q[f];
    }
}

// C tile of rows [row0, row0 + 32) x real columns [col0, col0 + BN) into `lds` (row stride
// GemmCfg<BN>::LDC).  planes: x3_split_rows_kernel's output for K elements per row (rows_pad rows,
// K % 64 == 0); wq: the x3-packed operator (J = K; complex x3_index, real x3r_index).  Each wave
// owns NT output tiles of 16 (complex: BN / 128, real: BN / 64).  [kb, ke): the reduction range
// holding every nonzero weight of this column tile (multiples of 64; h2_kband), default all of it.
template <int BN, bool CPX>
__device__ __forceinline__ void gemm_tile_x3(const unsigned short* __restrict__ planes, int rows_pad, int K,
                                             const void* __restrict__ wq, int row0, int col0, float* lds,
                                             int kb = 0, int ke = -1) {
    using Cg = GemmCfg<BN>;
    constexpr int PL = CPX ? 6 : 3;                  // planes
    constexpr int NT = CPX ? BN / 128 : BN / 64;      // 16-wide output tiles per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned short* sP = reinterpret_cast<unsigned short*>(lds);
    const size_t ps = (size_t)rows_pad * K;
    f32x4 cr[2][NT], ci[2][NT];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int t = 0; t < NT; ++t) { cr[b][t] = f32x4{0.f, 0.f, 0.f, 0.f}; ci[b][t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int ct0 = (CPX ? col0 / 2 : col0) / 16 + wave * NT;
    const int G = K >> 5;                               // groups of 32 reduction elements
    if (ke < 0) ke = K;
    const int gl1 = (ke > kb ? ke >> 5 : 1) - 1;        // last group of the range (refill clamp)
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * PL * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    const u32x4 sgn = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
    u32x4 wA[NT][PL], wB[NT][PL];
    auto wload = [&](u32x4 (&w)[NT][PL], int gg) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < PL; ++f)
#ifdef AMP_X3T_NOWLOAD   // diagnostic builds only (wrong results): the tile without its operator stream
                w[t][f] = u32x4{(unsigned)gg, (unsigned)f, (unsigned)t, 0x3f803f80u};
#else
                w[t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + gg) * PL + f) * 1024, 0);
#endif
    };
    // one group's MFMAs: both row blocks of 16 trials against this wave's NT tiles (gl: the group
    // within the staged chunk)
    auto mma_group = [&](int gl, const u32x4 (&w)[NT][PL]) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            // chunk 4 gl + (lane >> 4) of row lane & 15, permuted (pl_col, m = 15)
            const int sw = lane & 15 & X3SWM;
            const unsigned short* ap = sP + (16 * b + (lane & 15)) * X3KC + 8 * ((lane >> 4) ^ (sw & 3)) +
                                       ((32 * gl) ^ (32 * (sw >> 2)));
            u32x4 a[PL];
#pragma unroll
            for (int f = 0; f < PL; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * GBM * X3KC);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const u32x4* x = w[t];
#ifdef AMP_X3T_NOMMA   // diagnostic builds only (wrong results): the tile without its MFMAs
#define AMP_MB(acc, p, q) acc[0] += __builtin_bit_cast(float, (p)[0] ^ (q)[0])
#else
#define AMP_MB(acc, p, q) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(p), as_bf16x8(q), acc, 0, 0, 0)
#endif
                if constexpr (CPX) {
                    // Cr = Ar.Xr - Ai.Xi, Ci = Ar.Xi + Ai.Xr, smallest terms first (gemm_x3's order)
                    u32x4 na[3];
#pragma unroll
                    for (int f = 0; f < 3; ++f) na[f] = a[3 + f] ^ sgn;
                    AMP_MB(cr[b][t], a[0], x[2]);  AMP_MB(ci[b][t], a[0], x[5]);
                    AMP_MB(cr[b][t], a[1], x[1]);  AMP_MB(ci[b][t], a[1], x[4]);
                    AMP_MB(cr[b][t], a[2], x[0]);  AMP_MB(ci[b][t], a[2], x[3]);
                    AMP_MB(cr[b][t], na[0], x[5]); AMP_MB(ci[b][t], a[3], x[2]);
                    AMP_MB(cr[b][t], na[1], x[4]); AMP_MB(ci[b][t], a[4], x[1]);
                    AMP_MB(cr[b][t], na[2], x[3]); AMP_MB(ci[b][t], a[5], x[0]);
                    AMP_MB(cr[b][t], a[0], x[1]);  AMP_MB(ci[b][t], a[0], x[4]);
                    AMP_MB(cr[b][t], a[1], x[0]);  AMP_MB(ci[b][t], a[1], x[3]);
                    AMP_MB(cr[b][t], na[0], x[4]); AMP_MB(ci[b][t], a[3], x[1]);
                    AMP_MB(cr[b][t], na[1], x[3]); AMP_MB(ci[b][t], a[4], x[0]);
                    AMP_MB(cr[b][t], a[0], x[0]);  AMP_MB(ci[b][t], a[0], x[3]);
                    AMP_MB(cr[b][t], na[0], x[3]); AMP_MB(ci[b][t], a[3], x[0]);
                } else {
                    AMP_MB(cr[b][t], a[0], x[2]);
                    AMP_MB(cr[b][t], a[1], x[1]);
                    AMP_MB(cr[b][t], a[2], x[0]);
                    AMP_MB(cr[b][t], a[0], x[1]);
                    AMP_MB(cr[b][t], a[1], x[0]);
                    AMP_MB(cr[b][t], a[0], x[0]);
                }
#undef AMP_MB
            }
        }
    };
    if (ke > kb) {
        wload(wA, kb >> 5);
        wload(wB, min((kb >> 5) + 1, gl1));
    }
    // A chunk staging, one chunk ahead: the next chunk's plane loads are in flight (registers)
    // while this chunk's MFMAs issue, and land in LDS after them (the f32 tile's short-chunk
    // scheme, amp_gemm.h).  Every chunk is staged with the full chunk's compile-time geometry (no
    // divisions, no per-element guards: straight-line code keeps every vmcnt wait counted, so the
    // weight ring stays in flight across the stores); a tail chunk's columns past ke are loaded
    // at clamped addresses and never read.
    constexpr int CH = PL * GBM * (X3KC / 8) / AMP_WG;   // 16-byte units per thread
    static_assert(CH * AMP_WG == PL * GBM * (X3KC / 8), "whole chunk per workgroup");
    u32x4 v[CH];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int e = tid + i * AMP_WG;
            const int f = e / (GBM * (X3KC / 8)), rem = e % (GBM * (X3KC / 8)), r = rem / (X3KC / 8), c8 = rem % (X3KC / 8);
            v[i] = *reinterpret_cast<const u32x4*>(planes + f * ps + (size_t)(row0 + r) * K + min(c0 + 8 * c8, K - 8));
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int e = tid + i * AMP_WG;
            const int f = e / (GBM * (X3KC / 8)), rem = e % (GBM * (X3KC / 8)), r = rem / (X3KC / 8), c8 = rem % (X3KC / 8);
            *reinterpret_cast<u32x4*>(sP + (f * GBM + r) * X3KC + pl_col(r, 8 * c8, X3SWM)) = v[i];
        }
    };
    if (ke > kb) {
        load_chunk(kb);
        store_chunk();
    }
    for (int kc0 = kb; kc0 < ke; kc0 += X3KC) {
        const int kc = min(X3KC, ke - kc0);
        const bool more = kc0 + X3KC < ke;
        __syncthreads();                                // this chunk's LDS stores are visible
        if (more) load_chunk(kc0 + X3KC);
        // groups in pairs with two weight register sets: the fragments two groups ahead are in
        // flight while this group's MFMAs issue (K % 64 == 0; the refill index is clamped, so the
        // tail re-reads its last group)
        const int g0 = kc0 >> 5, gc = kc >> 5;
        if (gc == X3KC / 32) {
#pragma unroll
            for (int g = 0; g < X3KC / 32; g += 2) {
                mma_group(g, wA);
                wload(wA, min(g0 + g + 2, gl1));
                __builtin_amdgcn_sched_barrier(0);   // keep the refill behind its group's MFMAs
                mma_group(g + 1, wB);
                wload(wB, min(g0 + g + 3, gl1));
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            for (int g = 0; g < gc; g += 2) {
                mma_group(g, wA);
                wload(wA, min(g0 + g + 2, gl1));
                __builtin_amdgcn_sched_barrier(0);
                mma_group(g + 1, wB);
                wload(wB, min(g0 + g + 3, gl1));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (more) {
            __syncthreads();                            // every wave is done with this chunk
            store_chunk();
        }
    }
    __syncthreads();   // the C tile aliases the staged planes
    float* ct = lds;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * b + 4 * (lane >> 4) + r;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int o = 16 * (wave * NT + t) + (lane & 15);   // tile-local output
                if constexpr (CPX) {
                    ct[row * Cg::LDC + 2 * o] = cr[b][t][r];
                    ct[row * Cg::LDC + 2 * o + 1] = ci[b][t][r];
                } else {
                    ct[row * Cg::LDC + o] = cr[b][t][r];
                }
            }
        }
    __syncthreads();
}

}  // namespace amp
