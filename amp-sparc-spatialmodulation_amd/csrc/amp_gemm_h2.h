// amp_gemm_h2.h — the launch engines' split-precision fp16x2 GEMM tile (BAMP's four
// per-iteration products at the cfg5 shape), the counterpart of amp_gemm.h's f32 gemm_tile.
//
// Same contract as gemm_tile<BN>: C[32 trials x BN real columns] lands in LDS as the f32 C tile
// (row stride GemmCfg<BN>::LDC; complex outputs interleaved re / im), so the fused epilogues are
// unchanged.  The arithmetic is amp_persist.h's fp16x2 form:
//  * the A operand rows are split ONCE per GEMM by h2_split_rows_kernel into fp16 planes in
//    global memory ([plane][row][k]; complex: Re h0, Re h1, Im h0, Im h1; real: h0, h1) after
//    scaling each row by its own power of two (h2_row_exp over the row's max |value|, kept in
//    rexp[row]) — every column tile then reuses them;
//  * the operator is packed by h2_index (complex, four planes) / h2r_index (real, two planes) with
//    scale exponent H2_EX;
//  * products h0g0 + h0g1 + h1g0 on v_mfma_f32_16x16x32_f16 (two row blocks of 16 trials per wave
//    share each weight fragment), f32 accumulation, the scales taken off exactly in the epilogue.
// The A planes are staged through LDS in chunks of H2KC elements, in amp_persist.h's XOR-permuted
// plane layout (pl_col: the fragment reads and the staging stores hit distinct banks); the weights
// stream from L2.  A block-banded operator (the ISI channel) reduces each tile over [kb, ke) only
// (h2_kband).
#pragma once

#include "amp_gemm.h"
#include "amp_persist.h"

namespace amp {

constexpr int H2KC = 256;           // A elements (complex or real) per staged chunk
#ifdef AMP_H2_PAD_LAYOUT
constexpr int H2SWM = 0;            // A/B builds: the 16-byte row pad of the first version
#else
constexpr int H2SWM = 15;           // chunk permutation mask (pl_col)
#endif
constexpr int H2LDK = H2KC + (H2SWM ? 0 : 8);   // LDS row stride of a staged plane (fp16)

// bytes of LDS gemm_tile_h2<BN, CPX> needs (the staged planes; the C tile aliases them)
template <int BN, bool CPX>
constexpr size_t h2_tile_lds() {
    constexpr size_t planes = (size_t)(CPX ? 4 : 2) * GBM * H2LDK * 2;
    return planes > GemmCfg<BN>::LDS_BYTES ? planes : GemmCfg<BN>::LDS_BYTES;
}

// Real operators: two planes (h0, h1) per (tile, group).
__host__ __device__ __forceinline__ size_t h2r_index(int o, int j, int f, int J) {
    const int kk = j & 31;
    const int lane = (o & 15) + 16 * (kk >> 3);
    return ((((size_t)(o >> 4) * (J >> 5) + (j >> 5)) * 2 + f) * 64 + lane) * 8 + (kk & 7);
}

// Split rows [0, rows_pad) of a (row stride lda floats; rows >= rows are zero) into fp16 planes
// planes[f][row][k] (k < K, plane stride rows_pad * K) scaled by 2^rexp[row]: wpr wavefronts per
// row (1: four rows per workgroup; 4: a workgroup per row, the long rows of the ISI shape, where
// one wave per row left half the chip idle), the row max over them through LDS; complex rows
// (CPX) hold K interleaved values, real rows K floats.  K % 8 == 0.  `stopped` (optional): the
// iteration record's stop word, which turns the launch into a no-op.
template <bool CPX>
__global__ __launch_bounds__(256) void h2_split_rows_kernel(const float* __restrict__ a, int lda, int rows,
                                                            int rows_pad, int K, unsigned short* __restrict__ planes,
                                                            int* __restrict__ rexp, const int* __restrict__ stopped,
                                                            int wpr) {
    __shared__ float s_m[4];
    if (stopped && *stopped) return;                     // the detector's loop has stopped (no-op launch)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row = blockIdx.x * (4 / wpr) + wave / wpr;
    const int t = (wave % wpr) * 64 + lane, nt = 64 * wpr;   // this thread within the row's group
    const bool valid = row < rows_pad;
    const bool in = valid && row < rows;
    const float* ar = a + (size_t)(in ? row : 0) * lda;
    constexpr int FPE = CPX ? 2 : 1;                   // floats per element
    float m = 0.f;
    if (in)
        for (int q = t; q < K * FPE / 4; q += nt) {
            const float4 v = *reinterpret_cast<const float4*>(ar + 4 * q);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    m = group_max(m, 64);
    if (wpr > 1) {                                     // workgroup-uniform
        if (lane == 0) s_m[wave] = m;
        __syncthreads();
        for (int w = 0; w < wpr; ++w) m = fmaxf(m, s_m[(wave / wpr) * wpr + w]);
    }
    if (!valid) return;
    const int ex = in ? h2_row_exp(m) : 0;
    if (t == 0) rexp[row] = ex;
    const size_t ps = (size_t)rows_pad * K;          // plane stride (elements)
    unsigned short* pr = planes + (size_t)row * K;
    for (int j0 = 8 * t; j0 < K; j0 += 8 * nt) {      // 8 elements per thread and step
        float re[8], im[8];
#pragma unroll
        for (int h = 0; h < 8 / (4 / FPE); ++h) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (in) v = *reinterpret_cast<const float4*>(ar + FPE * j0 + 4 * h);
            if (CPX) {
                re[2 * h] = v.x; im[2 * h] = v.y; re[2 * h + 1] = v.z; im[2 * h + 1] = v.w;
            } else {
                re[4 * h] = v.x; re[4 * h + 1] = v.y; re[4 * h + 2] = v.z; re[4 * h + 3] = v.w;
            }
        }
        u32x4 q[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            unsigned a0, a1;
            split2x2(__builtin_amdgcn_ldexpf(re[2 * h], ex), __builtin_amdgcn_ldexpf(re[2 * h + 1], ex), a0, a1);
            q[0][h] = a0; q[1][h] = a1;
            if (CPX) {
                unsigned b0, b1;
                split2x2(__builtin_amdgcn_ldexpf(im[2 * h], ex), __builtin_amdgcn_ldexpf(im[2 * h + 1], ex), b0, b1);
                q[2][h] = b0; q[3][h] = b1;
            }
        }
#pragma unroll
        for (int f = 0; f < (CPX ? 4 : 2); ++f) *reinterpret_cast<u32x4*>(pr + f * ps + j0) = q[f];
    }
}

// C tile of rows [row0, row0 + 32) x real columns [col0, col0 + BN) into `lds` (row stride
// GemmCfg<BN>::LDC).  planes / rexp: h2_split_rows_kernel's output for K elements per row
// (rows_pad rows, K % 64 == 0); wq: the h2-packed operator (J = K) with scale exponent wex, ncp
// (complex or real outputs) a multiple of 16.  Each wave owns NT output tiles of 16 (complex: BN / 128, real: BN / 64).
// [kb, ke): the reduction range holding every nonzero weight of this column tile (multiples of
// 64; h2_kband), default all of it.
template <int BN, bool CPX>
__device__ __forceinline__ void gemm_tile_h2(const unsigned short* __restrict__ planes, int rows_pad,
                                             const int* __restrict__ rexp, int K, const void* __restrict__ wq,
                                             int wex, int row0, int col0, float* lds, int kb = 0, int ke = -1) {
    using Cg = GemmCfg<BN>;
    constexpr int PL = CPX ? 4 : 2;                  // planes
    constexpr int NT = CPX ? BN / 128 : BN / 64;      // 16-wide output tiles per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned short* sP = reinterpret_cast<unsigned short*>(lds);
    const size_t ps = (size_t)rows_pad * K;
    f32x4 cr[2][NT], ci[2][NT];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int t = 0; t < NT; ++t) { cr[b][t] = f32x4{0.f, 0.f, 0.f, 0.f}; ci[b][t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    // this wave's first output tile and its weight stream (one buffer resource, SGPR offsets)
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
                w[t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + gg) * PL + f) * 1024, 0);
    };
    // one group's MFMAs: both row blocks of 16 trials against this wave's NT tiles (gl: the group
    // within the staged chunk)
    auto mma_group = [&](int gg, int gl, const u32x4 (&w)[NT][PL]) {
        (void)gg;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            // chunk 4 gl + (lane >> 4) of row lane & 15, permuted (pl_col, m = 15)
            const int sw = lane & 15 & H2SWM;
            const unsigned short* ap = sP + (16 * b + (lane & 15)) * H2LDK + 8 * ((lane >> 4) ^ (sw & 3)) + ((32 * gl) ^ (32 * (sw >> 2)));
            u32x4 a[PL];
#pragma unroll
            for (int f = 0; f < PL; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * GBM * H2LDK);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
#define AMP_MH(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(x), as_f16x8(y), acc, 0, 0, 0)
                if constexpr (CPX) {
                    const u32x4 na0 = a[2] ^ sgn, na1 = a[3] ^ sgn;
                    AMP_MH(cr[b][t], a[0], w[t][1]); AMP_MH(ci[b][t], a[0], w[t][3]);
                    AMP_MH(cr[b][t], a[1], w[t][0]); AMP_MH(ci[b][t], a[1], w[t][2]);
                    AMP_MH(cr[b][t], na0, w[t][3]);  AMP_MH(ci[b][t], a[2], w[t][1]);
                    AMP_MH(cr[b][t], na1, w[t][2]);  AMP_MH(ci[b][t], a[3], w[t][0]);
                    AMP_MH(cr[b][t], a[0], w[t][0]); AMP_MH(ci[b][t], a[0], w[t][2]);
                    AMP_MH(cr[b][t], na0, w[t][2]);  AMP_MH(ci[b][t], a[2], w[t][0]);
                } else {
                    AMP_MH(cr[b][t], a[0], w[t][1]);
                    AMP_MH(cr[b][t], a[1], w[t][0]);
                    AMP_MH(cr[b][t], a[0], w[t][0]);
                }
#undef AMP_MH
            }
        }
    };
    if (ke > kb) {
        wload(wA, kb >> 5);
        wload(wB, min((kb >> 5) + 1, gl1));
    }
    for (int kc0 = kb; kc0 < ke; kc0 += H2KC) {
        const int kc = min(H2KC, ke - kc0);
        if (kc0 > kb) __syncthreads();                  // every wave done with the previous chunk
        // stage PL planes x 32 rows x the chunk (16-byte loads, all in flight before the stores),
        // with the full chunk's compile-time geometry and no branch (amp_gemm_x3.h): a tail chunk's
        // columns past ke are loaded at clamped addresses and never read
        {
            constexpr int Q8 = H2KC / 8;                // 16-byte units per plane row
            constexpr int CH = PL * GBM * Q8 / AMP_WG;
            static_assert(CH * AMP_WG == PL * GBM * Q8, "whole chunk per workgroup");
            u32x4 v[CH];
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                const int e = tid + i * AMP_WG;
                const int f = e / (GBM * Q8), rem = e % (GBM * Q8), r = rem / Q8, c8 = rem % Q8;
                v[i] = *reinterpret_cast<const u32x4*>(planes + f * ps + (size_t)(row0 + r) * K + min(kc0 + 8 * c8, K - 8));
            }
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                const int e = tid + i * AMP_WG;
                const int f = e / (GBM * Q8), rem = e % (GBM * Q8), r = rem / Q8, c8 = rem % Q8;
                *reinterpret_cast<u32x4*>(sP + (f * GBM + r) * H2LDK + pl_col(r, 8 * c8, H2SWM)) = v[i];
            }
        }
        __syncthreads();
        // groups in pairs with two weight register sets: the fragments two groups ahead are in
        // flight while this group's MFMAs issue (K % 64 == 0; the refill index is clamped, so the
        // tail re-reads its last group).  A whole chunk is unrolled so every wait on the weight
        // ring is a counted vmcnt (a rolled loop drained it to vmcnt(0) at its back edge).
        const int g0 = kc0 >> 5, gc = kc >> 5;
        if (gc == H2KC / 32) {
#pragma unroll
            for (int g = 0; g < H2KC / 32; g += 2) {
                mma_group(g0 + g, g, wA);
                wload(wA, min(g0 + g + 2, gl1));
                __builtin_amdgcn_sched_barrier(0);   // keep the refill behind its group's MFMAs
                mma_group(g0 + g + 1, g + 1, wB);
                wload(wB, min(g0 + g + 3, gl1));
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            for (int g = 0; g < gc; g += 2) {
                mma_group(g0 + g, g, wA);
                wload(wA, min(g0 + g + 2, gl1));
                __builtin_amdgcn_sched_barrier(0);   // keep the refill behind its group's MFMAs
                mma_group(g0 + g + 1, g + 1, wB);
                wload(wB, min(g0 + g + 3, gl1));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    __syncthreads();   // the C tile aliases the staged planes
    float* ct = lds;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * b + 4 * (lane >> 4) + r;
            const float sc = __builtin_amdgcn_ldexpf(1.0f, -(rexp[row0 + row] + wex));
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int o = 16 * (wave * NT + t) + (lane & 15);   // tile-local output
                if constexpr (CPX) {
                    ct[row * Cg::LDC + 2 * o] = cr[b][t][r] * sc;
                    ct[row * Cg::LDC + 2 * o + 1] = ci[b][t][r] * sc;
                } else {
                    ct[row * Cg::LDC + o] = cr[b][t][r] * sc;
                }
            }
        }
    __syncthreads();
}

// The reduction range of each column tile of an h2-packed operator (h2_index / h2r_index, PL
// planes, n16 packed 16-output tiles): grid (column tile, slice of 64 groups), the first / last 32-group holding a nonzero
// piece (NaN / inf included), met through atomic min / max in band[] (weight_kband_init before,
// h2_kband_fin after, amp_weights.hip), then widened to whole 64-element pairs: [kb, ke) in reduction elements.
template <int PL>
__global__ __launch_bounds__(256) void h2_kband_kernel(const u32x4* __restrict__ wq, int G, int tpt, int gps, int n16,
                                                       int* __restrict__ band) {
    __shared__ int s_lo, s_hi;
    if (threadIdx.x == 0) { s_lo = G; s_hi = -1; }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ga = blockIdx.y * gps, gn = min(gps, G - ga);
    int lo = G, hi = -1;
    for (int b = wave; b < tpt * gn; b += blockDim.x >> 6) {   // wave-uniform
        const int t16 = blockIdx.x * tpt + b / gn, g = ga + b % gn;
        if (t16 >= n16) continue;                               // past the operator's outputs (tail tile)
        const size_t base = ((size_t)t16 * G + g) * PL * 64 + lane;
        unsigned bits = 0u;
#pragma unroll
        for (int f = 0; f < PL; ++f) {
            const u32x4 v = wq[base + (size_t)f * 64];
            bits |= v.x | v.y | v.z | v.w;
        }
        if (__any((bits & 0x7fff7fffu) != 0u)) { lo = min(lo, g); hi = max(hi, g); }
    }
    if (lane == 0) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
    __syncthreads();
    if (threadIdx.x == 0 && s_hi >= 0) {
        atomicMin(&band[2 * blockIdx.x], s_lo);
        atomicMax(&band[2 * blockIdx.x + 1], s_hi);
    }
}

}  // namespace amp
