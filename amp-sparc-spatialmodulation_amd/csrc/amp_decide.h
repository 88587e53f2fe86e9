// amp_decide.h — the MAP hard decision of one section and its error-counter contributions,
// shared by the stand-alone decision kernel (amp_decide.hip) and the persistent VAMP
// engine's epilogue (amp_vamp_persist.hip), so both produce identical decisions and counts.
//
// Restates Loss.error_rate (loss.py:67-103) for generator_mode='sparc':
//   MAP_decision (loss.py:282-302): per section of M entries, argmax over the flattened
//     (m, k) grid of Re(x_m conj(a_k)) in float64.  The value is formed exactly as numpy's
//     complex multiply forms it (measured: fma(xr, ar, xi*ai)), first index wins ties,
//     an all/partly-NaN section picks its first NaN (np.argmax semantics).
//   mean_square_error / vector_error_rate / frame_error_rate / bit_error_rate
//     (loss.py:105-179) as integer counters and float64 sums.
#pragma once

#include <float.h>

#include "amp_common.h"

namespace amp {

// The decision's constellation: the float64 points (a Const64, shared with the exact rare path
// of the fused kernels, so a kernel needs only this one table), their complex64 casts and the
// gray labels.  Passed by value (kernel arguments, read through the scalar cache).
struct DecConst : Const64 {
    int sbits;
    float amax;                                // max_k max(|re_k|, |im_k|) (prefilter bound)
    float re32[AMP_MAX_K], im32[AMP_MAX_K];   // complex64 casts of the points (xhat values)
    unsigned char gray[AMP_MAX_K];            // gray label of point k (< 64)
};

// Unroll factor of the loops over the constellation: complete for K <= 16; chunks of 8 for
// 64-QAM, whose 128 uniform operands would not fit the scalar register file at once.
template <int KK>
struct KUnroll {
    static constexpr int value = KK > 16 ? 8 : KK;
};

struct alignas(16) DecPart {
    long long ier, ser, iber, sber;
    double mse, msef, msem, mseL;
};

// Per-workgroup record of the fused path: the section partials plus the channel-use / trial
// "any mismatch" counts of that workgroup's whole trials.
struct alignas(16) DecWG {
    DecPart p;
    long long ver, verf, verm, verL, fer, pad[3];
};

__device__ __forceinline__ bool dec_better(double v, int i, bool n, double bv, int bi, bool bn) {
    // does candidate (v, i, n) beat the incumbent (bv, bi, bn)?  NaN first, then larger value,
    // then smaller flat index (np.argmax: first occurrence of the maximum; NaN counts as maximum)
    if (n) return !bn || i < bi;
    if (bn) return false;
    return v > bv || (v == bv && i < bi);
}

__device__ __forceinline__ DecPart decpart_zero() { return DecPart{0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0}; }

__device__ __forceinline__ void decpart_add(DecPart& a, const DecPart& b) {
    a.ier += b.ier; a.ser += b.ser; a.iber += b.iber; a.sber += b.sber;
    a.mse += b.mse; a.msef += b.msef; a.msem += b.msem; a.mseL += b.mseL;
}

// One section decided by a group of G = min(M, 64) lanes (g = lane in group, PPL = M / G
// positions per lane).  ld(m, xmap, x, xmmse) loads position m of the section.  Every lane of
// the group returns the decision bi = m * K + k, the mismatch flag (xhat != x anywhere in the
// section, loss.py:133) and the float64 sum |xmmse - x|^2 over the section (loss.py:116).
// Reductions over a group of G consecutive lanes (G a power of two <= 64).
template <int G, class T, class OP>
__device__ __forceinline__ T dec_group_reduce(T v, OP op) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v = op(v, __shfl_xor(v, o, 64));
    return v;
}

// The decided section's xhat (a_k at position m, 0 elsewhere; bi = m * K + k) against the truth:
// mismatch flag (loss.py:133) and float64 sum |xmmse - x|^2 (loss.py:116), group-reduced.
template <int KK, int G, class LD>
__device__ __forceinline__ void section_tail(const DecConst& c, int M, int g, const LD& ld, int bi, int& bi_out,
                                             int& mm_out, double& se_out) {
    constexpr int K = KK;
    const int mh = bi / K, kh = bi - mh * K;
    float ar = 0.f, ai = 0.f;
    constexpr int KU = KUnroll<KK>::value;
#pragma unroll KU
    for (int k = 0; k < K; ++k)
        if (k == kh) { ar = c.re32[k]; ai = c.im32[k]; }
    int mm = 0;
    double se = 0.0;
    for (int m = g; m < M; m += G) {
        float2 xv, xt, xe;
        ld(m, xv, xt, xe);
        const float hr = (m == mh) ? ar : 0.f, hi = (m == mh) ? ai : 0.f;
        mm |= (hr - xt.x != 0.f || hi - xt.y != 0.f) ? 1 : 0;
        const float dr = xe.x - xt.x, di = xe.y - xt.y;
        se += (double)dr * dr + (double)di * di;
    }
    mm = dec_group_reduce<G>(mm, [](int a, int b) { return a | b; });
    se = dec_group_reduce<G>(se, [](double a, double b) { return a + b; });
    bi_out = bi;
    mm_out = mm;
    se_out = se;
}

// Segmented decision (Loss.segmented_decision, loss.py:222-250; generator_mode='segmented'):
// per section, the position of the largest |x_m| (np.abs of complex64 = float32 hypot;
// np.argsort()[-1]: NaN sorts last; among exactly equal magnitudes numpy's SIMD quicksort order
// is implementation-defined, and this kernel takes the last such position),
// then the nearest constellation point |x_m - a_k| in float64 (strict <: first minimum).  A
// NaN x_m has no nearest point in the reference (its section stays empty and the counting
// arrays no longer line up); here it decides k = 0.
template <int KK, int G, class LD>
__device__ __forceinline__ void decide_section_seg(const DecConst& c, int M, int g, const LD& ld, int& bi_out,
                                                   int& mm_out, double& se_out) {
    constexpr int K = KK;
    float bv = -1.f;
    int bm = -1;
    bool bn = false;
    for (int m = g; m < M; m += G) {
        float2 xv, xt, xe;
        ld(m, xv, xt, xe);
        const float a = hypotf(xv.x, xv.y);
        const bool an = a != a;
        // (a, m) beats (bv, bm): NaN largest, then larger value, then larger index
        const bool win = an ? (!bn || m > bm) : (!bn && (a > bv || (a == bv && m > bm)));
        if (win) { bv = a; bm = m; bn = an; }
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int om = __shfl_xor(bm, o, 64);
        const bool on = __shfl_xor((int)bn, o, 64) != 0;
        const bool win = on ? (!bn || om > bm) : (!bn && (ov > bv || (ov == bv && om > bm)));
        if (win) { bv = ov; bm = om; bn = on; }
    }
    float2 xs, xt, xe;
    ld(bm, xs, xt, xe);
    double d = INFINITY;
    int kh = 0;
    constexpr int KU = KUnroll<KK>::value;
#pragma unroll KU
    for (int k = 0; k < K; ++k) {
        const double ds = hypot((double)xs.x - c.re[k], (double)xs.y - c.im[k]);
        if (ds < d) { d = ds; kh = k; }
    }
    section_tail<KK, G>(c, M, g, ld, bm * K + kh, bi_out, mm_out, se_out);
}

// One section decided by a group of G lanes (g = lane in group; lane g owns positions
// g, g + G, ...).  ld(m, xmap, x, xmmse) loads position m of the section.  Every lane of the
// group returns the decision bi = m * K + k, the mismatch flag (xhat != x anywhere in the
// section, loss.py:133) and the float64 sum |xmmse - x|^2 over the section (loss.py:116).
// KK: the constellation size as a compile-time constant.
//
// PF = false: every (m, k) in float64 (the value formed as numpy forms it), np.argmax's rule.
// PF = true: exact float64 argmax behind a float32 prefilter: the float32 value v32 of every
// (m, k) is within eps = 2^-20 (|xr| + |xi|) max|a| + 2^-126 of the float64 value (three
// roundings of at most 2^-24 relative each, the float32 cast of the symbols included; 5x
// margin), so every (m, k) whose float64 value can reach the section maximum has
// v32 >= max v32 - 2 eps.  A single candidate IS the float64 argmax; several (ties such as the
// reference's duplicated 16-QAM point, or near-ties) are compared in float64 with np.argmax's
// rule; a section with a non-finite input is evaluated entirely in float64.  PF pays where
// the group is small (few lanes, many positions per lane: the persistent epilogue).
template <int KK, int G, bool PF, class LD>
__device__ __forceinline__ void decide_section(const DecConst& c, int M, int g, const LD& ld, int& bi_out, int& mm_out,
                                               double& se_out) {
    constexpr int K = KK;
    constexpr int KU = KUnroll<KK>::value;
    bool full = true;
    float thr = 0.f;
    int ncand = 0, first = 0x7fffffff;
    if (PF) {
        float vmax = -INFINITY, xs = 0.f;
        int bad = 0;
        for (int m = g; m < M; m += G) {
            float2 xv, xt, xe;
            ld(m, xv, xt, xe);
            bad |= !(fabsf(xv.x) <= FLT_MAX && fabsf(xv.y) <= FLT_MAX);
            xs = fmaxf(xs, fabsf(xv.x) + fabsf(xv.y));
#pragma unroll KU
            for (int k = 0; k < K; ++k) vmax = fmaxf(vmax, fmaf(xv.x, c.re32[k], xv.y * c.im32[k]));
        }
        vmax = dec_group_reduce<G>(vmax, [](float a, float b) { return fmaxf(a, b); });
        xs = dec_group_reduce<G>(xs, [](float a, float b) { return fmaxf(a, b); });
        bad = dec_group_reduce<G>(bad, [](int a, int b) { return a | b; });
        thr = vmax - 2.f * (xs * c.amax * 0x1p-20f + 0x1p-126f);
        if (!bad) {
            for (int m = g; m < M; m += G) {
                float2 xv, xt, xe;
                ld(m, xv, xt, xe);
#pragma unroll KU
                for (int k = 0; k < K; ++k) {
                    const bool cand = fmaf(xv.x, c.re32[k], xv.y * c.im32[k]) >= thr;
                    first = (cand && first == 0x7fffffff) ? m * K + k : first;
                    ncand += cand ? 1 : 0;
                }
            }
            ncand = dec_group_reduce<G>(ncand, [](int a, int b) { return a + b; });
            first = dec_group_reduce<G>(first, [](int a, int b) { return a < b ? a : b; });
        }
        full = bad != 0;
    }
    int bi = first;
    if (!PF || full || ncand > 1) {
        double bv = -INFINITY;
        bool bn = false;
        bi = 0x7fffffff;
        for (int m = g; m < M; m += G) {
            float2 xv, xt, xe;
            ld(m, xv, xt, xe);
            const double xr = (double)xv.x, xi = (double)xv.y;
#pragma unroll KU
            for (int k = 0; k < K; ++k) {
                if (!PF || full || fmaf(xv.x, c.re32[k], xv.y * c.im32[k]) >= thr) {
                    const double v = __fma_rn(xr, c.re[k], __dmul_rn(xi, c.im[k]));
                    const bool vn = v != v;
                    const int f = m * K + k;
                    if (dec_better(v, f, vn, bv, bi, bn)) { bv = v; bi = f; bn = vn; }
                }
            }
        }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            const double ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            const bool on = __shfl_xor((int)bn, o, 64) != 0;
            if (dec_better(ov, oi, on, bv, bi, bn)) { bv = ov; bi = oi; bn = on; }
        }
    }
    section_tail<KK, G>(c, M, g, ld, bi, bi_out, mm_out, se_out);
}

// Counter contributions of one decided section s (global section index b * L + l).
template <int KK>
__device__ __forceinline__ void count_section(const DecConst& c, long long s, int M, int L, int Na, int Lin, int bi,
                                              double se, long long sym, long long idx, long long ibmask,
                                              DecPart& q) {
    constexpr int K = KK;
    constexpr int KU = KUnroll<KK>::value;
    const int mh = bi / K, kh = bi - mh * K;
    const long long sbmask = (1LL << c.sbits) - 1;
    const long long ih = s * M + mh;           // flat index of the chosen entry
    long long sh = 0;
#pragma unroll KU
    for (int k = 0; k < K; ++k)
        if (k == kh) sh = c.gray[k];
    q.ier += (ih != idx);
    q.ser += (sh != sym);
    q.iber += __popcll((unsigned long long)((ih ^ idx) & ibmask));
    q.sber += __popcll((unsigned long long)((sh ^ sym) & sbmask));
    const int si = (int)s;                     // B * L < 2^31 (asserted by the callers' sizes)
    const int lin = (si % L) / Na;
    q.mse += se;
    if (lin == 0) q.msef += se;
    if (lin == Lin / 2) q.msem += se;
    if (lin == Lin - 1) q.mseL += se;
}

__host__ inline DecConst to_decconst(const amp_constellation* c) {
    DecConst d;
    d.K = c->K;
    d.real_alpha = 1;
    d.sbits = c->symbol_bits;
    for (int i = 0; i < AMP_MAX_K; ++i) {
        const bool v = i < c->K;
        d.re[i] = v ? c->re64[i] : 0.0;
        d.im[i] = v ? c->im64[i] : 0.0;
        if (v && c->im64[i] != 0.0) d.real_alpha = 0;
        d.re32[i] = v ? (float)c->re64[i] : 0.f;
        d.im32[i] = v ? (float)c->im64[i] : 0.f;
        d.gray[i] = v ? (unsigned char)c->gray[i] : 0;
    }
    double am = 0.0;
    for (int i = 0; i < c->K; ++i) am = fmax(am, fmax(fabs(c->re64[i]), fabs(c->im64[i])));
    d.amax = (float)(am * (1.0 + 1e-6));
    return d;
}

__device__ __forceinline__ long long dec_ibmask(int ibits) { return (ibits >= 63) ? -1LL : ((1LL << ibits) - 1); }

// amp_counts from n per-workgroup records, folded by one whole workgroup (blockDim a multiple
// of 64, <= 1024) in a fixed order: strided per-thread sums, then lane and wave trees.
// `lds` >= 16 * sizeof(DecWG) bytes.  Thread 0 writes *out.
__device__ inline void dec_fold_block(const DecWG* w, int n, amp_counts* out, void* lds) {
    DecWG a;
    a.p = decpart_zero();
    a.ver = a.verf = a.verm = a.verL = a.fer = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const DecWG q = w[i];
        decpart_add(a.p, q.p);
        a.ver += q.ver; a.verf += q.verf; a.verm += q.verm; a.verL += q.verL; a.fer += q.fer;
    }
    a.p.ier = group_sum(a.p.ier, 64); a.p.ser = group_sum(a.p.ser, 64);
    a.p.iber = group_sum(a.p.iber, 64); a.p.sber = group_sum(a.p.sber, 64);
    a.p.mse = group_sum(a.p.mse, 64); a.p.msef = group_sum(a.p.msef, 64);
    a.p.msem = group_sum(a.p.msem, 64); a.p.mseL = group_sum(a.p.mseL, 64);
    a.ver = group_sum(a.ver, 64); a.verf = group_sum(a.verf, 64); a.verm = group_sum(a.verm, 64);
    a.verL = group_sum(a.verL, 64); a.fer = group_sum(a.fer, 64);
    DecWG* sw = reinterpret_cast<DecWG*>(lds);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        amp_counts c;
        c.ier = c.ser = c.iber = c.sber = 0;
        c.ver = c.verf = c.verm = c.verL = c.fer = 0;
        c.mse = c.msef = c.msem = c.mseL = 0.0;
        for (int v = 0; v < (int)(blockDim.x >> 6); ++v) {
            const DecWG& q = sw[v];
            c.ier += q.p.ier; c.ser += q.p.ser; c.iber += q.p.iber; c.sber += q.p.sber;
            c.mse += q.p.mse; c.msef += q.p.msef; c.msem += q.p.msem; c.mseL += q.p.mseL;
            c.ver += q.ver; c.verf += q.verf; c.verm += q.verm; c.verL += q.verL; c.fer += q.fer;
        }
        *out = c;
    }
    __syncthreads();
}

}  // namespace amp
