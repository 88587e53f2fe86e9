// amp_persist.h — device building blocks of the persistent engines (amp_vamp_persist.hip,
// amp_scamp_persist.hip): one workgroup per CU keeps 16 trials' state in LDS across the whole
// iteration loop.
//  * gemm16: C[16 x 16 NT] += A[16 x 16 G] (LDS) . Wq^T on v_mfma_f32_16x16x4_f32, the weight
//    streamed from L2 through a buffer-load ring in 16x16x4-packed order (wpack16_index);
//  * the per-iteration batch-global exchange: each workgroup publishes its partial as two
//    sc1 write-through granules tagged with (launch generation, iteration), every workgroup
//    sweeps and reduces all of them in one fixed order (bit-identical scalars everywhere);
//  * grid_sync: a bounded-spin grid barrier for the rare exact-float64 path.
// Every spin is bounded (2 s) and raises an abort word that releases every other workgroup.
#pragma once

#include <cfloat>

#include "amp_common.h"

namespace amp {

constexpr int PRING = 4;   // W groups in flight per wave

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// C[16 x 16*NT] (this wave's columns ct0*16 ...) += A[16 x 16*G] (LDS, row stride lda) . Wq^T,
// Wq packed by wpack16_index.  Accumulator t, register r: row 4*(lane>>4) + r, column
// 16*(ct0 + t) + (lane & 15).  Fully unrolled over the G reduction groups so every wait on the
// weight ring is a counted `s_waitcnt vmcnt(n)` (a rolled loop drained it to vmcnt(0) at the
// back edge: ~25 % of the GEMM time at cfg4, r01 trace); the A row of group g+1 is read from
// LDS one group ahead.
template <int NT, int G>
__device__ __forceinline__ void gemm16(const float* sA, int lda, const float* __restrict__ wq, int ct0,
                                       f32x4 (&acc)[NT]) {
    constexpr int R = G < PRING ? G : PRING;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one buffer resource per wave (base = this wave's first column tile); every load is
    // lane * 16 + a compile-time byte offset (SGPR), so the unrolled ring holds no addresses
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);   // wave-uniform: SGPR resource, no waterfall
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(wq) + (size_t)ct0u * G * 256, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    auto wload = [&](int t, int g) {
        const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, (t * G + g) * 1024, 0);
        return make_float4(v.x, v.y, v.z, v.w);
    };
    float4 ring[R][NT];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t) ring[d][t] = wload(t, d);
    const float* a_s = sA + (lane & 15) * lda + 4 * (lane >> 4);
    float4 acur = *reinterpret_cast<const float4*>(a_s);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % R;
        const float4 anext = *reinterpret_cast<const float4*>(a_s + 16 * (g + 1 < G ? g + 1 : g));
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(acur.x, ring[d][t].x, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(acur.y, ring[d][t].y, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(acur.z, ring[d][t].z, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(acur.w, ring[d][t].w, acc[t]);
        if (g + R < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t) ring[d][t] = wload(t, g + R);
        }
        acur = anext;
        __builtin_amdgcn_sched_barrier(0);   // keep the ring depth: no hoisting of later groups' loads
    }
}

// ---- A-plane layout of the split-precision engines (bf16x3: six planes, fp16x2: four) ----
// Plane f, row r (16 rows per plane), element j at (16 f + r) ldx + (j ^ 8 (r & m)): no row pad
// (ldx = K, pl_ldx), the 16-byte chunks of row r XOR-permuted by r & m, m + 1 = the lowest set bit
// of K / 8 capped at 16 (the permutation stays inside aligned blocks of m + 1 chunks).  The
// 16x16x32 fragment reads (lanes l and l + 16: rows l & 15, chunks c and c + 1), the 8-row
// 16-byte stores and the accumulator word stores then all hit distinct banks for K = 64 ... 512
// (the 16-byte row pad of rounds 1-2 left every fragment read 2-way in half its lane groups:
// tools/ubench/lds_phase_ubench.hip).
__host__ __device__ inline int pl_ldx(int K) { return K; }
__device__ __forceinline__ int pl_mask(int ldx) {
    const int n = ldx >> 3;
    const int b = n & -n;
    return (b < 16 ? b : 16) - 1;
}
__device__ __forceinline__ int pl_col(int row, int j, int m) { return j ^ ((row & m) << 3); }
// The permuted addresses are cheap to form but loop-invariant, so the compiler would hoist every
// one of them out of the persistent engines' iteration loop and keep it live across the denoiser
// (spilling at 512 VGPRs); pl_opaque pins their inputs inside the loop (an empty volatile asm).
__device__ __forceinline__ int pl_opaque(int x) {
#ifndef AMP_PL_HOIST
    asm volatile("" : "+v"(x));
#endif
    return x;
}

// ---- kernel arguments through a laundered kernarg pointer (the persistent engines) ----
// A persistent kernel's loop reads dozens of argument fields; left alone, the compiler hoists all
// of them into SGPRs for the whole launch.  Reading them through the kernarg segment pointer,
// passed through an empty asm at chosen points (karg_launder), makes each phase reload what it uses
// (s_load from the scalar cache).  karg_second_offset: the kernarg offset of a kernel's second
// by-value argument (the first at 0; the amdhsa metadata's .args offsets agree).
typedef const __attribute__((address_space(4))) char* KargPtr;
template <class A, class B>
constexpr int karg_second_offset() {
    return (int)((sizeof(A) + alignof(B) - 1) / alignof(B) * alignof(B));
}
template <class T>
__device__ __forceinline__ const T* karg_at(unsigned long long base, int off) {
    return (const T*)(const __attribute__((address_space(4))) T*)(KargPtr)(base + (unsigned long long)off);
}
__device__ __forceinline__ unsigned long long karg_launder(unsigned long long v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ unsigned long long karg_base() {
    return (unsigned long long)(KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
}

// ---- split-precision complex GEMM (bf16x3) ----
// x = x0 + x1 + x2 with bf16 pieces (round-to-nearest-even; each residual is exact in f32), so
// a product a.b keeps the six terms a0b0 a0b1 a1b0 a0b2 a1b1 a2b0 (dropped terms <= 2^-24 |ab|)
// and sums them on v_mfma_f32_16x16x32_bf16: the f32 products at 2.7x the f32-MFMA rate, with the
// vector ALU free for 8 of every 16 MFMA cycles.  A non-finite x keeps x0 = x and zero residuals.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Two values -> their three packed bf16 pieces (x in the low half): v_cvt_pk_bf16_f32 and
// v_pk_add_f32, ~14 instructions per pair.
__device__ __forceinline__ void split3x2(float x, float y, unsigned& p0, unsigned& p1, unsigned& p2) {
    const f32x2_t v = {x, y};
    const bf16x2_t b0 = __builtin_convertvector(v, bf16x2_t);
    f32x2_t r1 = v - __builtin_convertvector(b0, f32x2_t);
    r1.x = __builtin_isfinite(x) ? r1.x : 0.0f;
    r1.y = __builtin_isfinite(y) ? r1.y : 0.0f;
    const bf16x2_t b1 = __builtin_convertvector(r1, bf16x2_t);
    const f32x2_t r2 = r1 - __builtin_convertvector(b1, f32x2_t);
    const bf16x2_t b2 = __builtin_convertvector(r2, bf16x2_t);
    p0 = __builtin_bit_cast(unsigned, b0);
    p1 = __builtin_bit_cast(unsigned, b1);
    p2 = __builtin_bit_cast(unsigned, b2);
}

// Eight consecutive complex values of one row -> the six bf16 planes (Re x0 x1 x2, Im x0 x1 x2)
// of an x3 A operand: plane f, row `row`, elements j0 .. j0+7 (one 16-byte store each).
__device__ __forceinline__ void x3_store8(unsigned short* sP, int ldx, int row, int j0, const float (&re)[8],
                                          const float (&im)[8]) {
    u32x4 q[6];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        unsigned a0, a1, a2, b0, b1, b2;
        split3x2(re[2 * h], re[2 * h + 1], a0, a1, a2);
        split3x2(im[2 * h], im[2 * h + 1], b0, b1, b2);
        q[0][h] = a0; q[1][h] = a1; q[2][h] = a2; q[3][h] = b0; q[4][h] = b1; q[5][h] = b2;
    }
    const int c = pl_col(pl_opaque(row), j0, pl_mask(ldx));
#pragma unroll
    for (int f = 0; f < 6; ++f) *reinterpret_cast<u32x4*>(sP + (f * 16 + row) * ldx + c) = q[f];
}

__device__ __forceinline__ float dpp_swap_pair(float v) {   // lane l <-> l ^ 1 (quad_perm [1,0,3,2])
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// One accumulator tile's values (this lane: rows 4*(lane>>4) + r, complex column o) -> the six
// planes, as 32-bit words of column pairs: the even lane of each pair writes rows +0 / +1, the
// odd lane rows +2 / +3 (one DPP swap per sent value; no 16-bit LDS stores).
__device__ __forceinline__ void x3_store_acc(unsigned short* sP, int ldx, int o, const float (&vr)[4],
                                             const float (&vi)[4]) {
    const int lane = pl_opaque((int)threadIdx.x) & 63;
    const bool odd = (lane & 1) != 0;
    float gr[2], gi[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        gr[h] = dpp_swap_pair(odd ? vr[h] : vr[2 + h]);
        gi[h] = dpp_swap_pair(odd ? vi[h] : vi[2 + h]);
    }
    const int row0 = 4 * (lane >> 4) + (odd ? 2 : 0);
    const int m = pl_mask(ldx);
    const int pl = 16 * ldx;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        unsigned short* p = sP + (row0 + h) * ldx + pl_col(row0 + h, o & ~1, m);
        const float mr = odd ? vr[2 + h] : vr[h], mi = odd ? vi[2 + h] : vi[h];
        unsigned q[6];
        split3x2(odd ? gr[h] : mr, odd ? mr : gr[h], q[0], q[1], q[2]);
        split3x2(odd ? gi[h] : mi, odd ? mi : gi[h], q[3], q[4], q[5]);
#pragma unroll
        for (int f = 0; f < 6; ++f) *reinterpret_cast<unsigned*>(p + f * pl) = q[f];
    }
}

// Scalar form (weight builder): the three pieces of one value.
__device__ __forceinline__ void split3(float x, unsigned& p0, unsigned& p1, unsigned& p2) {
    unsigned q0, q1, q2;
    split3x2(x, 0.0f, q0, q1, q2);
    p0 = q0 & 0xffffu; p1 = q1 & 0xffffu; p2 = q2 & 0xffffu;
}

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// C[16 x 16 NT] (complex; Re in cr, Im in ci; this wave's complex column tiles ct0 ...) =
// A[16 x 32 G] (complex, six bf16 planes in LDS, plane row stride ldx) . X^T, X packed by
// x3_index (amp_gemm.h) as six planes per (tile, group).  Cr = Ar.Xr - Ai.Xi, Ci = Ar.Xi + Ai.Xr:
// only the operator's unique values are streamed (12 bytes per complex entry, 0.75x the f32
// real expansion).  Accumulator t, register r: row 4*(lane>>4) + r, complex column
// 16*(ct0 + t) + (lane & 15).
// Weight ring: R groups in flight (R = 1 measured best: the MFMA queue of one group covers the
// next group's loads, tools/ubench/gemm_x3_ubench.hip); the A fragments are read one group ahead.
// PIN: keep each ring refill behind the group's MFMAs (a scheduling barrier): the compiler then
// cannot hoist the next group's loads into fresh registers — the ring holds exactly R groups (the
// two-waves-per-SIMD engines, which have 256 registers per wave, use R = 2 with it).
// HL: the two leading-piece products of each group (a0 b0 of Ar.Xr and of Ai.Xi, ~2^0 relative)
// accumulate apart from the ten cross-piece products (<= 2^-8 relative), and the two sums are
// added once at the end: the f32 rounding of the large running sum then happens 2 times per
// group instead of 12 (the VAMP engine's GEMM error against float64: DESIGN.md §4 item 5).
template <int NT, int G, int R = 1, bool PIN = false, bool HL = false>
__device__ __forceinline__ void gemm_x3(const unsigned short* sP, int ldx, const void* __restrict__ wq, int ct0,
                                        f32x4 (&cr)[NT], f32x4 (&ci)[NT]) {
    constexpr int RR = G < R ? G : R;
    constexpr int NL = HL ? NT : 1;
    const int lane = threadIdx.x & 63;
    f32x4 lr[NL], li[NL];
#pragma unroll
    for (int t = 0; t < NT; ++t) { cr[t] = f32x4{0.f, 0.f, 0.f, 0.f}; ci[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
    for (int t = 0; t < NL; ++t) { lr[t] = f32x4{0.f, 0.f, 0.f, 0.f}; li[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 6 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    u32x4 ring[RR][NT][6];
#pragma unroll
    for (int d = 0; d < RR; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < 6; ++f)
                ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + d) * 6 + f) * 1024, 0);
    // A fragment of group g: row lane & 15, chunk 4 g + (lane >> 4), permuted (pl_col): element
    // 8 ((4 g + q) ^ sw) = ((32 g) ^ s32) + 8 (q ^ (sw & 3)), s32 = 32 (sw >> 2) (one v_xad per g)
    const int ln = pl_opaque(lane);
    const int sw = (ln & 15) & pl_mask(ldx);
    const unsigned short* ap = sP + (ln & 15) * ldx + 8 * ((ln >> 4) ^ (sw & 3));
    const int s32 = 32 * (sw >> 2);
    const u32x4 sgn = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
    u32x4 an[6];
    if constexpr (!PIN) {
#pragma unroll
        for (int f = 0; f < 6; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + s32 + f * 16 * ldx);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % RR;
        u32x4 a[6], na[3];
        if constexpr (PIN) {
            // no A prefetch (24 registers): the SIMD's partner wave covers this group's LDS reads
#pragma unroll
            for (int f = 0; f < 6; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + ((32 * g) ^ s32) + f * 16 * ldx);
        } else {
#pragma unroll
            for (int f = 0; f < 6; ++f) a[f] = an[f];
            if (g + 1 < G) {
#pragma unroll
                for (int f = 0; f < 6; ++f)
                    an[f] = *reinterpret_cast<const u32x4*>(ap + ((32 * (g + 1)) ^ s32) + f * 16 * ldx);
            }
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) na[f] = a[3 + f] ^ sgn;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4* w = ring[d][t];
            f32x4 gr = cr[t], gi = ci[t];
            f32x4 sr = HL ? lr[HL ? t : 0] : gr, si = HL ? li[HL ? t : 0] : gi;   // the cross-piece sums
#define AMP_MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(x), as_bf16x8(y), acc, 0, 0, 0)
            // smallest terms first
            AMP_MF(sr, a[0], w[2]);  AMP_MF(si, a[0], w[5]);
            AMP_MF(sr, a[1], w[1]);  AMP_MF(si, a[1], w[4]);
            AMP_MF(sr, a[2], w[0]);  AMP_MF(si, a[2], w[3]);
            AMP_MF(sr, na[0], w[5]); AMP_MF(si, a[3], w[2]);
            AMP_MF(sr, na[1], w[4]); AMP_MF(si, a[4], w[1]);
            AMP_MF(sr, na[2], w[3]); AMP_MF(si, a[5], w[0]);
            AMP_MF(sr, a[0], w[1]);  AMP_MF(si, a[0], w[4]);
            AMP_MF(sr, a[1], w[0]);  AMP_MF(si, a[1], w[3]);
            AMP_MF(sr, na[0], w[4]); AMP_MF(si, a[3], w[1]);
            AMP_MF(sr, na[1], w[3]); AMP_MF(si, a[4], w[0]);
            if constexpr (HL) {
                lr[HL ? t : 0] = sr; li[HL ? t : 0] = si;
            } else {
                gr = sr; gi = si;
            }
            AMP_MF(gr, a[0], w[0]);  AMP_MF(gi, a[0], w[3]);
            AMP_MF(gr, na[0], w[3]); AMP_MF(gi, a[3], w[0]);
#undef AMP_MF
            cr[t] = gr; ci[t] = gi;
        }
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        if (g + RR < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int f = 0; f < 6; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + RR) * 6 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (HL) {
#pragma unroll
        for (int t = 0; t < NT; ++t) { cr[t] += lr[HL ? t : 0]; ci[t] += li[HL ? t : 0]; }
    }
}

// ---- split-precision complex GEMM (fp16x2) ----
// v 2^e = h0 + h1 with fp16 pieces (round-to-nearest-even; 22 significant bits), so a product
// keeps the three terms h0g0 h0g1 h1g0 (the dropped h1g1 is <= 2^-22 of it) on
// v_mfma_f32_16x16x32_f16 with f32 accumulation, and the power-of-two scales come off exactly in
// the epilogue.  fp16's exponent range is the price: the operator is scaled by 2^H2_EX (entries of
// magnitude < 4; the SVD factors of vamp.py have |v| <= 1), every A row by its own 2^e that puts
// the row's max |value| in [2^13, 2^14) (h2_row_exp).  Against bf16x3: 8 bytes per complex
// operator entry instead of 12 and 12 MFMAs per complex tile-group instead of 24
// (tools/ubench/gemm_h2_ubench.hip at cfg4: 10.4k vs 18.6k cycles per GEMM, max |error| 8.8e-7 vs
// a sequential f32 sum's 1.4e-6 and bf16x3's 1.3e-6 on the same data).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
constexpr int H2_EX = 14;   // operator scale exponent (amp_weights.hip WPACKH2)
constexpr int YH2_EX = 10;  // the y~ operator s Uh (entries s_o |U| < 64; the singular values are O(1))

// The exponent e that puts m 2^e (m = a row's max |value|) in [2^13, 2^14); 0 for 0 / inf / NaN.
__device__ __forceinline__ int h2_row_exp(float m) {
    if (!(m > 0.f) || !__builtin_isfinite(m)) return 0;
    return 14 - __builtin_amdgcn_frexp_expf(m);
}

// Two (scaled) values -> their two packed fp16 pieces (x in the low half).  A non-finite first
// piece keeps a zero residual.
__device__ __forceinline__ void split2x2(float x, float y, unsigned& p0, unsigned& p1) {
    const f32x2_t v = {x, y};
    const f16x2_t h0 = __builtin_convertvector(v, f16x2_t);
    const f32x2_t b = __builtin_convertvector(h0, f32x2_t);
    f32x2_t r = v - b;
    r.x = __builtin_isfinite(b.x) ? r.x : 0.0f;
    r.y = __builtin_isfinite(b.y) ? r.y : 0.0f;
    const f16x2_t h1 = __builtin_convertvector(r, f16x2_t);
    p0 = __builtin_bit_cast(unsigned, h0);
    p1 = __builtin_bit_cast(unsigned, h1);
}

// Scalar form (weight builder): the two pieces of x 2^e.
__device__ __forceinline__ void split2(float x, int e, unsigned& p0, unsigned& p1) {
    unsigned q0, q1;
    split2x2(__builtin_amdgcn_ldexpf(x, e), 0.0f, q0, q1);
    p0 = q0 & 0xffffu; p1 = q1 & 0xffffu;
}

// Eight consecutive complex values of one row (already scaled) -> the four fp16 planes
// (Re h0 h1, Im h0 h1) of an h2 A operand: plane f, row `row`, elements j0 .. j0+7.
__device__ __forceinline__ void h2_store8(unsigned short* sP, int ldx, int row, int j0, const float (&re)[8],
                                          const float (&im)[8]) {
    u32x4 q[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        unsigned a0, a1, b0, b1;
        split2x2(re[2 * h], re[2 * h + 1], a0, a1);
        split2x2(im[2 * h], im[2 * h + 1], b0, b1);
        q[0][h] = a0; q[1][h] = a1; q[2][h] = b0; q[3][h] = b1;
    }
    const int c = pl_col(pl_opaque(row), j0, pl_mask(ldx));
#pragma unroll
    for (int f = 0; f < 4; ++f) *reinterpret_cast<u32x4*>(sP + (f * 16 + row) * ldx + c) = q[f];
}

// x3_store_acc for the h2 planes (values already scaled).
__device__ __forceinline__ void h2_store_acc(unsigned short* sP, int ldx, int o, const float (&vr)[4],
                                             const float (&vi)[4]) {
    const int lane = pl_opaque((int)threadIdx.x) & 63;
    const bool odd = (lane & 1) != 0;
    float gr[2], gi[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        gr[h] = dpp_swap_pair(odd ? vr[h] : vr[2 + h]);
        gi[h] = dpp_swap_pair(odd ? vi[h] : vi[2 + h]);
    }
    const int row0 = 4 * (lane >> 4) + (odd ? 2 : 0);
    const int m = pl_mask(ldx);
    const int pl = 16 * ldx;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        unsigned short* p = sP + (row0 + h) * ldx + pl_col(row0 + h, o & ~1, m);
        const float mr = odd ? vr[2 + h] : vr[h], mi = odd ? vi[2 + h] : vi[h];
        unsigned q[4];
        split2x2(odd ? gr[h] : mr, odd ? mr : gr[h], q[0], q[1]);
        split2x2(odd ? gi[h] : mi, odd ? mi : gi[h], q[2], q[3]);
#pragma unroll
        for (int f = 0; f < 4; ++f) *reinterpret_cast<unsigned*>(p + f * pl) = q[f];
    }
}

__device__ __forceinline__ f16x8 as_f16x8(u32x4 v) { return __builtin_bit_cast(f16x8, v); }

// gemm_x3's contract on the h2 planes: A = four fp16 planes in LDS (Re h0 h1, Im h0 h1), X packed
// by h2_index (amp_gemm.h) as four planes per (tile, group).  The accumulators hold the product
// of the SCALED operands (A 2^e_row, X 2^H2_EX): the caller takes the scales off.
template <int NT, int G, int R = 1>
__device__ __forceinline__ void gemm_h2(const unsigned short* sP, int ldx, const void* __restrict__ wq, int ct0,
                                        f32x4 (&cr)[NT], f32x4 (&ci)[NT]) {
    constexpr int RR = G < R ? G : R;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < NT; ++t) { cr[t] = f32x4{0.f, 0.f, 0.f, 0.f}; ci[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 4 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    u32x4 ring[RR][NT][4];
#pragma unroll
    for (int d = 0; d < RR; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < 4; ++f)
                ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + d) * 4 + f) * 1024, 0);
    // A fragment of group g: row lane & 15, chunk 4 g + (lane >> 4), permuted (pl_col): element
    // 8 ((4 g + q) ^ sw) = ((32 g) ^ s32) + 8 (q ^ (sw & 3)), s32 = 32 (sw >> 2) (one v_xad per g)
    const int ln = pl_opaque(lane);
    const int sw = (ln & 15) & pl_mask(ldx);
    const unsigned short* ap = sP + (ln & 15) * ldx + 8 * ((ln >> 4) ^ (sw & 3));
    const int s32 = 32 * (sw >> 2);
    const u32x4 sgn = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
    u32x4 an[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + s32 + f * 16 * ldx);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % RR;
        u32x4 a[4], na[2];
#pragma unroll
        for (int f = 0; f < 4; ++f) a[f] = an[f];
        if (g + 1 < G) {
#pragma unroll
            for (int f = 0; f < 4; ++f)
                an[f] = *reinterpret_cast<const u32x4*>(ap + ((32 * (g + 1)) ^ s32) + f * 16 * ldx);
        }
#pragma unroll
        for (int f = 0; f < 2; ++f) na[f] = a[2 + f] ^ sgn;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4* w = ring[d][t];   // w[0] / w[1]: Re h0 / h1, w[2] / w[3]: Im h0 / h1
#define AMP_MH(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(x), as_f16x8(y), acc, 0, 0, 0)
            // smallest terms first: Cr = Ar.Xr - Ai.Xi, Ci = Ar.Xi + Ai.Xr
            AMP_MH(cr[t], a[0], w[1]);  AMP_MH(ci[t], a[0], w[3]);
            AMP_MH(cr[t], a[1], w[0]);  AMP_MH(ci[t], a[1], w[2]);
            AMP_MH(cr[t], na[0], w[3]); AMP_MH(ci[t], a[2], w[1]);
            AMP_MH(cr[t], na[1], w[2]); AMP_MH(ci[t], a[3], w[0]);
            AMP_MH(cr[t], a[0], w[0]);  AMP_MH(ci[t], a[0], w[2]);
            AMP_MH(cr[t], na[0], w[2]); AMP_MH(ci[t], a[2], w[0]);
#undef AMP_MH
        }
        if (g + RR < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + RR) * 4 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---- split-precision complex GEMM (int8x4: block fixed point on the integer matrix cores) ----
// Every A row (r~, then w) carries its own power-of-two scale, every operator column its own:
// with e the smallest exponent such that the row's (column's) max |value| < 2^e, a value v becomes
// the 31-bit integer V = rint(v 2^(30 - e)) (|V| < 2^30), written as four balanced base-256 digits
// d0 .. d3 (V = d0 2^24 + d1 2^16 + d2 2^8 + d3; |d0| <= 64, the others in [-128, 127]): byte k of
// digit plane s is the low byte of (V + c_s) >> 8 (3 - s), c = 0x808080, 0x8080, 0x80, 0.  A
// product keeps the digit pairs i + j <= 3 (ten of the sixteen), summed per level s = i + j on
// v_mfma_i32_16x16x64_i8 — exact in int32 (a level sum is below 2^25 for K <= 512) — and the levels
// are combined in f32 at the end (smallest first), then scaled by 2^(e_row + e_col - 12).
// Operands: 31 significant bits relative to the row / column maximum, i.e. at least 24 bits for
// every element down to 2^-7 of its row's (column's) largest; the dropped pairs (i + j >= 4) are
// below 2^-30 of (row max . column max).  Measured on the cfg4 GEMM shape against a float64 sum
// (tools/ubench/gemm_i8_ubench.hip): max |error| 6.0e-8, a sequential f32 sum's 1.4e-6, bf16x3's
// 1.3e-6.  8 bytes per complex operator entry (bf16x3: 12) and 40 i8 MFMAs per complex tile and
// 64-deep group (bf16x3: 48 bf16 MFMAs of the same cycles for the same depth).
// A non-finite value anywhere in an A row makes the whole row's result NaN (the row's factor is
// NaN; its digits are zero).  The reference's matmul gives NaN there for a NaN input (every output
// of the row sums over it) and +-inf or NaN for an infinite one.
typedef int i32x4 __attribute__((ext_vector_type(4)));
#ifndef AMP_I8_APF
#define AMP_I8_APF 1   // gemm_i8: A fragments read one step ahead
#endif
// byte offset of the column exponents behind an i8-packed [O][J] operator's planes
__host__ __device__ __forceinline__ size_t i8_exp_offset(int O, int J) { return (size_t)O * J * 8; }

// bytes per LDS row of one digit plane: N + 16 (rows 16 bytes apart in bank order: the
// 16-row fragment reads and the 8-byte row stores are conflict-free for N % 64 == 0)
__host__ __device__ __forceinline__ int i8_ldb(int N) { return N + 16; }
__host__ __device__ __forceinline__ int i8_plane_floats(int N) { return 8 * 16 * i8_ldb(N) / 4; }

// The exponent e with m < 2^e for a finite m > 0 (0 for m == 0); INT_MAX for a non-finite m.
__device__ __forceinline__ int i8_row_exp(float m) {
    if (!(m <= FLT_MAX)) return 0x7fffffff;
    if (!(m > 0.f)) return 0;
    return __builtin_amdgcn_frexp_expf(m);
}
// |v| as the row maximum's contribution: a NaN counts as +inf (fmaxf would drop it)
__device__ __forceinline__ float i8_absmax(float m, float v) {
    const float a = fabsf(v);
    return fmaxf(m, a <= FLT_MAX ? a : INFINITY);
}
// 2^(e - 12) as the row factor of gemm_i8's epilogue (NaN for a non-finite row)
__device__ __forceinline__ float i8_row_factor(int e) {
    return e == 0x7fffffff ? __int_as_float(0x7fc00000) : __builtin_amdgcn_ldexpf(1.0f, e - 12);
}
// v -> V = rint(v 2^(30 - e)) (0 for a non-finite row)
__device__ __forceinline__ int i8_fix(float v, int e) {
    return e == 0x7fffffff ? 0 : (int)__builtin_rintf(__builtin_amdgcn_ldexpf(v, 30 - e));
}
// four integers -> one dword of digit plane s (byte i = digit s of V_i)
template <int S>
__device__ __forceinline__ unsigned i8_digits4(int v0, int v1, int v2, int v3) {
    constexpr int sh = 8 * (3 - S);
    constexpr int c = S == 0 ? 0x808080 : S == 1 ? 0x8080 : S == 2 ? 0x80 : 0;
    const unsigned y0 = (unsigned)((v0 + c) >> sh), y1 = (unsigned)((v1 + c) >> sh);
    const unsigned y2 = (unsigned)((v2 + c) >> sh), y3 = (unsigned)((v3 + c) >> sh);
    const unsigned lo = __builtin_amdgcn_perm(y1, y0, 0x0c0c0400u);   // [y0.b0, y1.b0, 0, 0]
    const unsigned hi = __builtin_amdgcn_perm(y3, y2, 0x0c0c0400u);
    return lo | (hi << 16);
}
// two integers -> one 16-bit word of digit plane s
template <int S>
__device__ __forceinline__ unsigned short i8_digits2(int v0, int v1) {
    constexpr int sh = 8 * (3 - S);
    constexpr int c = S == 0 ? 0x808080 : S == 1 ? 0x8080 : S == 2 ? 0x80 : 0;
    return (unsigned short)__builtin_amdgcn_perm((unsigned)((v1 + c) >> sh), (unsigned)((v0 + c) >> sh), 0x0c0c0400u);
}

// Eight consecutive complex values of one row -> the eight digit planes (Re d0..d3, Im d0..d3) of
// an i8 A operand: plane f, row `row`, bytes j0 .. j0+7 (one 8-byte store each).  e: the row's
// exponent (i8_row_exp).
__device__ __forceinline__ void i8_store8(signed char* sB, int ldb, int row, int j0, const float (&re)[8],
                                          const float (&im)[8], int e) {
    int vr[8], vi[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) { vr[h] = i8_fix(re[h], e); vi[h] = i8_fix(im[h], e); }
    signed char* p = sB + pl_opaque(row) * ldb + j0;
    const int pl = 16 * ldb;
#define AMP_I8ST(S)                                                                                          \
    *reinterpret_cast<uint2*>(p + (S) * pl) =                                                                \
        make_uint2(i8_digits4<S>(vr[0], vr[1], vr[2], vr[3]), i8_digits4<S>(vr[4], vr[5], vr[6], vr[7]));     \
    *reinterpret_cast<uint2*>(p + (4 + (S)) * pl) =                                                          \
        make_uint2(i8_digits4<S>(vi[0], vi[1], vi[2], vi[3]), i8_digits4<S>(vi[4], vi[5], vi[6], vi[7]));
    AMP_I8ST(0) AMP_I8ST(1) AMP_I8ST(2) AMP_I8ST(3)
#undef AMP_I8ST
}

// One accumulator tile's values (this lane: rows 4*(lane>>4) + r, complex column o; already
// fixed-point integers) -> the eight digit planes as 16-bit words of column pairs: the even lane
// of each pair writes rows +0 / +1, the odd lane rows +2 / +3 (one DPP swap per sent value).
__device__ __forceinline__ void i8_store_acc(signed char* sB, int ldb, int o, const int (&vr)[4], const int (&vi)[4]) {
    const int lane = pl_opaque((int)threadIdx.x) & 63;
    const bool odd = (lane & 1) != 0;
    int gr[2], gi[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        gr[h] = __builtin_amdgcn_update_dpp(0, odd ? vr[h] : vr[2 + h], 0xB1, 0xF, 0xF, false);
        gi[h] = __builtin_amdgcn_update_dpp(0, odd ? vi[h] : vi[2 + h], 0xB1, 0xF, 0xF, false);
    }
    const int row0 = 4 * (lane >> 4) + (odd ? 2 : 0);
    const int pl = 16 * ldb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        signed char* p = sB + (row0 + h) * ldb + (o & ~1);
        const int mr = odd ? vr[2 + h] : vr[h], mi = odd ? vi[2 + h] : vi[h];
        const int r0 = odd ? gr[h] : mr, r1 = odd ? mr : gr[h];
        const int i0 = odd ? gi[h] : mi, i1 = odd ? mi : gi[h];
        *reinterpret_cast<unsigned short*>(p + 0 * pl) = i8_digits2<0>(r0, r1);
        *reinterpret_cast<unsigned short*>(p + 1 * pl) = i8_digits2<1>(r0, r1);
        *reinterpret_cast<unsigned short*>(p + 2 * pl) = i8_digits2<2>(r0, r1);
        *reinterpret_cast<unsigned short*>(p + 3 * pl) = i8_digits2<3>(r0, r1);
        *reinterpret_cast<unsigned short*>(p + 4 * pl) = i8_digits2<0>(i0, i1);
        *reinterpret_cast<unsigned short*>(p + 5 * pl) = i8_digits2<1>(i0, i1);
        *reinterpret_cast<unsigned short*>(p + 6 * pl) = i8_digits2<2>(i0, i1);
        *reinterpret_cast<unsigned short*>(p + 7 * pl) = i8_digits2<3>(i0, i1);
    }
}

// C[16 x 16 NT] (complex, f32, fully scaled) = A[16 x 64 G] (complex, eight int8 digit planes in
// LDS, row stride ldb bytes) . X^T, X packed by i8_index with its column exponents behind the
// planes.  Tile-outer: complex column tile t runs all G groups before tile t + 1, so one tile's
// level sums are live (P = Ar.Xr, Q = Ai.Xi, C = Ar.Xi + Ai.Xr, four levels each; Re = P - Q in
// int32, exact) and leave as f32; the A fragments are re-read from LDS per tile (one group ahead),
// the operator streams through a ring of D (tile, group) slots in (t, g) order.
// rowf[r]: this lane's rows' factors (i8_row_factor).  Accumulator t, register r: row
// 4*(lane>>4) + r, complex column 16*(ct0 + t) + (lane & 15).
template <int NT, int G, int D = 2, bool APF = AMP_I8_APF>
__device__ __forceinline__ void gemm_i8(const signed char* sB, int ldb, const void* __restrict__ wq, int O, int ct0,
                                        const float (&rowf)[4], f32x4 (&cr)[NT], f32x4 (&ci)[NT]) {
    constexpr int NS = NT * G;
    constexpr int DD = NS < D ? NS : D;
    const int lane = threadIdx.x & 63;
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 8 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = pl_opaque(lane * 16);   // opaque: the first ring loads stay inside the caller's loop
    const int* ecol = reinterpret_cast<const int*>((const char*)wq + i8_exp_offset(O, 64 * G));
    u32x4 ring[DD][8];
#pragma unroll
    for (int d = 0; d < DD; ++d)
#pragma unroll
        for (int f = 0; f < 8; ++f) ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, (d * 8 + f) * 1024, 0);
    const int ln = pl_opaque(lane);
    // this lane's column factors, loaded up front (they arrive during the first tile's MFMAs)
    float cf[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) cf[t] = __builtin_amdgcn_ldexpf(1.0f, ecol[16 * (ct0 + t) + (ln & 15)]);
    const signed char* ap = sB + (ln & 15) * ldb + 16 * (ln >> 4);
    u32x4 an[8];
    if constexpr (APF) {
#pragma unroll
        for (int f = 0; f < 8; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * ldb);
    }
    i32x4 P[4], Q[4], C[4];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
        const int t = st / G, g = st % G, d = st % DD;
        __builtin_amdgcn_sched_barrier(0);   // no motion across steps: one tile's sums live at a time
        if (g == 0) {
#pragma unroll
            for (int s = 0; s < 4; ++s) { P[s] = i32x4{0, 0, 0, 0}; Q[s] = P[s]; C[s] = P[s]; }
        }
        // the same group's fragments are re-read for every tile: the offsets are pinned (opaque)
        // so that the compiler does not keep all G groups' fragments live across the tiles
        u32x4 a[8];
        if constexpr (APF) {
#pragma unroll
            for (int f = 0; f < 8; ++f) a[f] = an[f];
            if (st + 1 < NS) {
                const int off = pl_opaque(64 * ((st + 1) % G));
#pragma unroll
                for (int f = 0; f < 8; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * ldb + off);
            }
        } else {
            const int off = pl_opaque(64 * g);
#pragma unroll
            for (int f = 0; f < 8; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * ldb + off);
        }
        const u32x4* w = ring[d];   // w[0..3]: Re digits, w[4..7]: Im digits
#define AMP_MI(acc_, x, y) \
    acc_ = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, x), __builtin_bit_cast(i32x4, y), acc_, 0, 0, 0)
#pragma unroll
        for (int s = 3; s >= 0; --s)
#pragma unroll
            for (int i = 0; i <= s; ++i) {
                AMP_MI(P[s], a[i], w[s - i]);          // Ar Xr
                AMP_MI(Q[s], a[4 + i], w[4 + s - i]);  // Ai Xi
                AMP_MI(C[s], a[i], w[4 + s - i]);      // Ar Xi
                AMP_MI(C[s], a[4 + i], w[s - i]);      // Ai Xr
            }
#undef AMP_MI
        __builtin_amdgcn_sched_barrier(0);
        if (st + DD < NS) {
#pragma unroll
            for (int f = 0; f < 8; ++f)
                ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((st + DD) * 8 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (g == G - 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float vr = (float)(P[3][r] - Q[3][r]), vi = (float)C[3][r];
                vr = fmaf(vr, 0x1p-8f, (float)(P[2][r] - Q[2][r]));
                vi = fmaf(vi, 0x1p-8f, (float)C[2][r]);
                vr = fmaf(vr, 0x1p-8f, (float)(P[1][r] - Q[1][r]));
                vi = fmaf(vi, 0x1p-8f, (float)C[1][r]);
                vr = fmaf(vr, 0x1p-8f, (float)(P[0][r] - Q[0][r]));
                vi = fmaf(vi, 0x1p-8f, (float)C[0][r]);
                cr[t][r] = vr * rowf[r] * cf[t];
                ci[t][r] = vi * rowf[r] * cf[t];
            }
        }
    }
}

// Grid barrier: arrival counter + abort word in pbar (zeroed before the launch).  The
// workgroup's payload stores precede it in program order (thread 0 stores them or the
// barrier below orders them); agent-scope release on arrival, acquire after the wait.
// grid_sync_on: the same over a group of workgroups with its own arrival counter `cnt` (the
// persistent VAMP engine's side-by-side epochs); `abort_w` is shared by the whole grid.
__device__ inline bool grid_sync_on(unsigned* cnt, unsigned* abort_w, unsigned target, int* s_flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s at 100 MHz
                __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        *s_flag = ok;
    }
    __syncthreads();
    return *s_flag != 0;
}

__device__ inline bool grid_sync(unsigned* pbar, unsigned target, int* s_flag) {
    return grid_sync_on(pbar, pbar + 1, target, s_flag);
}

// ---- per-iteration partials: data-tagged granules (no fences, no counter) ----
// Each workgroup publishes its block partial as two 16-byte granules, each ONE write-through
// (`sc1`) buffer store carrying the tag t + 1 in its last word:
//   g0 = {sumvar lo, sumvar hi, notclose, tag},  g1 = {maxabs (f32 bits), minsecmax (f32 bits), 0, tag}
// (maxabs / minsecmax are float32 values or NaN / inf: exact in f32).  Every workgroup then
// sweeps all nwg granule pairs with `sc1` loads (L2/fabric-served, never a stale L1 line)
// until every tag matches, and reduces them in one fixed order, so every workgroup derives
// bit-identical batch scalars.  The granule block is zeroed before every launch (tag 0 never
// matches).  MI355X_MICROARCH.md § visibility (R2 granules, allgather).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gran_rsrc(void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void part_publish(PartAcc p, __amdgpu_buffer_rsrc_t rs, unsigned off, unsigned tag,
                                             void* lds_scratch) {
    part_wave_reduce(p);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Partial* s = reinterpret_cast<Partial*>(lds_scratch);
    __syncthreads();
    if (lane == 0) {
        s[wave].sumvar = p.sumvar; s[wave].maxabs = p.maxabs;
        s[wave].minsecmax = p.minsecmax; s[wave].notclose = p.notclose;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double sv = s[0].sumvar, mx = s[0].maxabs, mn = s[0].minsecmax;
        uint32_t nc = s[0].notclose;
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) {
            sv += s[w].sumvar; mx = nan_max(mx, s[w].maxabs); mn = nan_min(mn, s[w].minsecmax); nc += s[w].notclose;
        }
        const unsigned long long b = (unsigned long long)__double_as_longlong(sv);
        const u32x4 g0 = {(unsigned)b, (unsigned)(b >> 32), nc, tag};
        const u32x4 g1 = {__float_as_uint((float)mx), __float_as_uint((float)mn), 0u, tag};
        __builtin_amdgcn_raw_buffer_store_b128(g0, rs, (int)off, 0, 16);        // aux 16 = sc1
        __builtin_amdgcn_raw_buffer_store_b128(g1, rs, (int)off + 16, 0, 16);
    }
}

// Wave 0 sweeps the nwg (<= 256) granule pairs of one iteration; the result lands in every
// thread.  A bounded spin (2 s) raises the abort word, as grid_sync does.
__device__ __forceinline__ bool part_gather(__amdgpu_buffer_rsrc_t rs, unsigned off0, int nwg, unsigned tag,
                                            unsigned* abort_word, PartAcc& out, void* lds_scratch, int* s_flag) {
    Partial* s = reinterpret_cast<Partial*>(lds_scratch);
    if ((threadIdx.x >> 6) == 0) {
        const int lane = threadIdx.x & 63;
        u32x4 a[4], b[4];
        int ok_all = 1;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int w = lane + 64 * q;
                if (w < nwg) {
                    a[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off0 + 32u * w), 0, 16);
                    b[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off0 + 32u * w + 16), 0, 16);
                    ok &= (a[q].w == tag) & (b[q].w == tag);
                }
            }
            if (__all(ok)) break;
            if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s at 100 MHz
                __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok_all = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        PartAcc p;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (lane + 64 * q < nwg) {
                p.sumvar += __longlong_as_double((long long)(((unsigned long long)a[q].y << 32) | a[q].x));
                p.maxabs = nan_max(p.maxabs, (double)__uint_as_float(b[q].x));
                p.minsecmax = nan_min(p.minsecmax, (double)__uint_as_float(b[q].y));
                p.notclose += a[q].z;
            }
        }
        part_wave_reduce(p);
        if (lane == 0) {
            s[0].sumvar = p.sumvar; s[0].maxabs = p.maxabs; s[0].minsecmax = p.minsecmax; s[0].notclose = p.notclose;
            *s_flag = ok_all;
        }
    }
    __syncthreads();
    out.sumvar = s[0].sumvar; out.maxabs = s[0].maxabs; out.minsecmax = s[0].minsecmax; out.notclose = s[0].notclose;
    const bool ok = *s_flag != 0;
    __syncthreads();
    return ok;
}

}  // namespace amp
