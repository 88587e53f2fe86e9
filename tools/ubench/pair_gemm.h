// pair_gemm.h (tools/ubench; not built into the library) — split-K workgroup pairs for the
// persistent bf16x3 engine at N = 256 (cfg4), the round-5 review's item 1, measured and NOT adopted.
//
// The 16-trial engine streams the WHOLE operator (256 x 256 complex, 786 KB at 12 B per entry)
// through every CU for every GEMM, and that per-CU stream was the GEMMs' wall.
// A pair of workgroups on one XCD (blocks b and b + 8 under round-robin placement; placement is a
// speed matter only) shares 32 trials and splits every GEMM's reduction: workgroup h owns the
// complex columns [128 h, 128 h + 128) of every per-trial vector, i.e. its half of the K range of
// both GEMMs and its half of their outputs.  Per GEMM each wave
//   1. forms the partial sums of its PARTNER's output tile (8 (1 - h) + wave) over its own K half
//      (two 16-row A tiles share every operator fragment: half the operator bytes per CU),
//   2. hands them over as data-tagged 16-byte granules (three floats + tag, one write-through
//      store each: MI355X_MICROARCH.md handoff-1to1 / R2 — no flag, no fence),
//   3. forms its OWN tile's partial sums (the hand-off travels meanwhile), and
//   4. adds the partner's partials for its own tile (polling their tags, bounded).
// Every output is then (own half) + (partner half): a pairwise split of the f32 accumulation.
// Measured (tools/ubench/pair_ubench.hip, profiles/r06_pair_ubench.txt, cycles per iteration of the
// two GEMMs): the pair GEMMs alone 23.7k against the engine form's 32.1k (MFMA-bound: the operator
// stream halves), but every hand-off variant 34.3k-37.6k: 12.6 MB of granules per GEMM chip-wide
// (8 MB as raw partials behind a flag) cost ~4.5k cycles per GEMM in the stores alone (all bytes
// leave L2: fabric write bandwidth), and a second ~0.5-1k in the poll.
#pragma once

#include "../../amp-sparc-spatialmodulation_amd/csrc/amp_persist.h"

namespace amp {

// Eight bf16x3 products pairs of one complex tile-group in gemm_x3's order (smallest terms first);
// a: the A fragment's six planes, na: its imaginary planes sign-flipped, w: the operator's.
__device__ __forceinline__ void x3_mf_group(const u32x4 (&a)[6], const u32x4 (&na)[3], const u32x4* w, f32x4& gr,
                                            f32x4& gi) {
#define AMP_MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(x), as_bf16x8(y), acc, 0, 0, 0)
    AMP_MF(gr, a[0], w[2]);  AMP_MF(gi, a[0], w[5]);
    AMP_MF(gr, a[1], w[1]);  AMP_MF(gi, a[1], w[4]);
    AMP_MF(gr, a[2], w[0]);  AMP_MF(gi, a[2], w[3]);
    AMP_MF(gr, na[0], w[5]); AMP_MF(gi, a[3], w[2]);
    AMP_MF(gr, na[1], w[4]); AMP_MF(gi, a[4], w[1]);
    AMP_MF(gr, na[2], w[3]); AMP_MF(gi, a[5], w[0]);
    AMP_MF(gr, a[0], w[1]);  AMP_MF(gi, a[0], w[4]);
    AMP_MF(gr, a[1], w[0]);  AMP_MF(gi, a[1], w[3]);
    AMP_MF(gr, na[0], w[4]); AMP_MF(gi, a[3], w[1]);
    AMP_MF(gr, na[1], w[3]); AMP_MF(gi, a[4], w[0]);
    AMP_MF(gr, a[0], w[0]);  AMP_MF(gi, a[0], w[3]);
    AMP_MF(gr, na[0], w[3]); AMP_MF(gi, a[3], w[0]);
#undef AMP_MF
}

// C[32 x 16] (complex; two 16-row tiles rt = 0 / 1, Re in cr[rt], Im in ci[rt]) = A[32 x 32 GH] .
// X^T over the GH 32-deep groups [gbase, gbase + GH) of the operator tile behind `wr` (x3-packed:
// group g at (g * 6 + f) KB), A as two sets of six bf16 planes (rows 0-15 at sP0, 16-31 at sP1,
// plane row stride ldx = 32 GH, pl_col-permuted).  Each operator group feeds both row tiles; the
// A fragments are read one row tile ahead; D operator groups in flight.
// pre(): called once the first D groups' operator loads are issued; mid(g): after group g's
// MFMAs and the ring refill behind them (the pair hand-off's stores and poll loads go there, so
// the in-order vmcnt waits of the first groups do not wait for them).
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
    __device__ __forceinline__ void operator()(int) const {}
};
template <int GH, int D = 1, class Pre = NoHook, class Mid = NoHook>
__device__ __forceinline__ void gemm_x3_r2(const unsigned short* sP0, const unsigned short* sP1, int ldx,
                                           __amdgpu_buffer_rsrc_t wr, int gbase, f32x4 (&cr)[2], f32x4 (&ci)[2],
                                           Pre&& pre = Pre(), Mid&& mid = Mid()) {
    constexpr int DD = GH < D ? GH : D;
    const int lane = threadIdx.x & 63;
    const int vo = lane * 16;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) { cr[rt] = f32x4{0.f, 0.f, 0.f, 0.f}; ci[rt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    u32x4 ring[DD][6];
#pragma unroll
    for (int d = 0; d < DD; ++d)
#pragma unroll
        for (int f = 0; f < 6; ++f) ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((gbase + d) * 6 + f) * 1024, 0);
    pre();
    const int ln = pl_opaque(lane);
    const int sw = (ln & 15) & pl_mask(ldx);
    const int aoff = (ln & 15) * ldx + 8 * ((ln >> 4) ^ (sw & 3));
    const int s32 = 32 * (sw >> 2);
    const u32x4 sgn = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
    auto lda = [&](int g, int rt, u32x4 (&a)[6]) {
        const unsigned short* ap = (rt ? sP1 : sP0) + aoff + ((32 * g) ^ s32);
#pragma unroll
        for (int f = 0; f < 6; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * ldx);
    };
    u32x4 acur[6];
    lda(0, 0, acur);
#pragma unroll
    for (int g = 0; g < GH; ++g) {
        const u32x4* w = ring[g % DD];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            u32x4 a[6], anx[6], na[3];
#pragma unroll
            for (int f = 0; f < 6; ++f) a[f] = acur[f];
            if (rt == 0) lda(g, 1, anx);
            else if (g + 1 < GH) lda(g + 1, 0, anx);
#pragma unroll
            for (int f = 0; f < 3; ++f) na[f] = a[3 + f] ^ sgn;
            x3_mf_group(a, na, w, cr[rt], ci[rt]);
            if (rt == 0 || g + 1 < GH) {
#pragma unroll
                for (int f = 0; f < 6; ++f) acur[f] = anx[f];
            }
        }
        if (g + DD < GH) {
#pragma unroll
            for (int f = 0; f < 6; ++f)
                ring[g % DD][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((gbase + g + DD) * 6 + f) * 1024, 0);
        }
        mid(g);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- the pair hand-off: one wave's 16 partial sums per lane as six tagged granules ----
// Granule q of lane l holds values 3q .. 3q + 2 of the lane's list (cr[0], ci[0], cr[1], ci[1]
// flattened; the last granule carries one) and the tag in its fourth word.  Slot layout: granule
// q of lane l at byte off + q KB + 16 l (each store instruction writes 1 KB contiguous).
constexpr int PAIR_GRAN = 6;                        // granules per lane
constexpr int PAIR_WAVE_BYTES = PAIR_GRAN * 1024;   // one wave's slot

__device__ __forceinline__ float pair_val(const f32x4 (&cr)[2], const f32x4 (&ci)[2], int i) {
    const int rt = i >> 3, k = (i >> 2) & 1, r = i & 3;
    return k ? ci[rt][r] : cr[rt][r];
}

template <int AUX = 16>
__device__ __forceinline__ void pair_put(__amdgpu_buffer_rsrc_t rs, int off, unsigned tag, const f32x4 (&cr)[2],
                                         const f32x4 (&ci)[2]) {
    const int vo = (threadIdx.x & 63) * 16;
    off = __builtin_amdgcn_readfirstlane(off);   // wave-uniform: an SGPR offset (no waterfall loop)
#pragma unroll
    for (int q = 0; q < PAIR_GRAN; ++q) {
        u32x4 g;
        g.x = __float_as_uint(pair_val(cr, ci, 3 * q));
        g.y = 3 * q + 1 < 16 ? __float_as_uint(pair_val(cr, ci, 3 * q + 1)) : 0u;
        g.z = 3 * q + 2 < 16 ? __float_as_uint(pair_val(cr, ci, 3 * q + 2)) : 0u;
        g.w = tag;
        __builtin_amdgcn_raw_buffer_store_b128(g, rs, vo, off + q * 1024, AUX);   // aux 16 = sc1 (write-through)
    }
}

// The partner wave's granules: pair_issue loads them (early, behind the own tile's operator loads);
// pair_take_add polls until every tag matches (bounded: 2 s, then the abort word is raised, as
// part_gather does) and ADDS the values into cr / ci.  False: aborted (values untouched).
__device__ __forceinline__ void pair_issue(__amdgpu_buffer_rsrc_t rs, int off, u32x4 (&g)[PAIR_GRAN]) {
    const int vo = (threadIdx.x & 63) * 16;
    off = __builtin_amdgcn_readfirstlane(off);
#pragma unroll
    for (int q = 0; q < PAIR_GRAN; ++q) g[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, off + q * 1024, 16);   // sc1
}

__device__ __forceinline__ bool pair_take_add(__amdgpu_buffer_rsrc_t rs, int off, unsigned tag, unsigned* abort_word,
                                              u32x4 (&g)[PAIR_GRAN], f32x4 (&cr)[2], f32x4 (&ci)[2]) {
    bool ok = true;
#pragma unroll
    for (int q = 0; q < PAIR_GRAN; ++q) ok &= g[q].w == tag;
    if (!__all(ok)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            __builtin_amdgcn_s_sleep(1);
            pair_issue(rs, off, g);
            ok = true;
#pragma unroll
            for (int q = 0; q < PAIR_GRAN; ++q) ok &= g[q].w == tag;
            if (__all(ok)) break;
            if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s at 100 MHz
                __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const u32x4& q = g[i / 3];
        const unsigned u = (i % 3) == 0 ? q.x : (i % 3) == 1 ? q.y : q.z;
        const int rt = i >> 3, k = (i >> 2) & 1, r = i & 3;
        if (k) ci[rt][r] += __uint_as_float(u);
        else cr[rt][r] += __uint_as_float(u);
    }
    return true;
}

__device__ __forceinline__ bool pair_get_add(__amdgpu_buffer_rsrc_t rs, int off, unsigned tag, unsigned* abort_word,
                                             f32x4 (&cr)[2], f32x4 (&ci)[2]) {
    u32x4 g[PAIR_GRAN];
    pair_issue(rs, off, g);
    return pair_take_add(rs, off, tag, abort_word, g, cr, ci);
}

}  // namespace amp
