// amp_denoise.h — block-sparse constellation denoiser (posterior mean/variance of a
// section holding exactly one nonzero drawn from the constellation).
//
// Restates VAMPLayer.segmented_denoiser (vamp.py:96-119), BAMPLayer.segmented_denoiser
// (bamp.py:66-77) and SCAMPLayer.denoiser (scamp.py:61-68):
//   xi[m,k]   = Re((r_m / tau_m) * conj(a_k))
//   eta[m,k]  = exp(xi[m,k] - shift)
//   xmmse_m   = sum_k a_k eta[m,k] / Z,      Z = sum_{m,k} eta
//   var_m     = |xmmse_m|^2 (1 - P_m) + sum_k |xmmse_m - a_k|^2 eta[m,k] / Z,  P_m = sum_k eta[m,k] / Z
//
// Fast path: each section is shifted by its OWN max (the softmax is shift-invariant): float32
// logits, exp((xi - max) * log2 e) as one v_mul + v_exp_f32 (scaling AFTER the subtraction keeps
// the dominant weights' exponents exact; folding log2 e into the symbols costs one more
// rounding of |xi| and measurably moves the allclose early exit), float32 sums per position,
// float64 section sum Z so that 1 - P_m = (Z - Z_m)/Z has no cancellation.
// The reference shifts by max|xi| over the WHOLE batch in float64 (vamp.py:112); the few
// sections for which that matters (normaliser out of the normal float64 range) are redone by
// exact_section_f64 after the batch reduction — the fast path reports per section its max
// logit and its max |logit| (natural units) for that decision.
//
// Mapping: one section per group of G = min(M, 64) lanes (M a power of two), each lane owns
// PPL = M / G positions; reductions are xor-shuffles inside the group.
#pragma once

#include <float.h>

#include "amp_common.h"

namespace amp {

#define AMP_LOG2E 1.44269504088896340736f

// Diagnostic precision switches (default 0: the product arithmetic).  AMP_DEN_EXACT_EXP: every
// softmax weight as float(exp(double(x) - double(m))) (correctly rounded); AMP_DEN_DIV: 1 / Z by
// an IEEE division instead of v_rcp_f32.  tools/den_isolate.py measures their effect on the
// early exit.
#ifndef AMP_DEN_EXACT_EXP
#define AMP_DEN_EXACT_EXP 0
#endif
#ifndef AMP_DEN_DIV
#define AMP_DEN_DIV 0
#endif
// exp(x - m) for a logit x and its shift m (natural units)
__device__ __forceinline__ float den_exp(float x, float m) {
#if AMP_DEN_EXACT_EXP
    return (float)exp((double)x - (double)m);
#else
    return __builtin_amdgcn_exp2f((x - m) * AMP_LOG2E);
#endif
}
__device__ __forceinline__ float den_rcp(float z) {
#if AMP_DEN_DIV
    return 1.0f / z;
#else
    return __builtin_amdgcn_rcpf(z);
#endif
}

// Which waves of the workgroup share a denoiser call: this wave's index among them and their
// count (default: every wave of the workgroup).  The wave-specialized engine
// (amp_vamp_persist_kernel.h, WS) hands half the sections to a subset of its waves.
struct DenWaves {
    int wave, nw;
    __device__ static DenWaves block() { return DenWaves{(int)(threadIdx.x >> 6), (int)(blockDim.x >> 6)}; }
};

// A uniform kernel-argument value taken through readfirstlane: the loads stay scalar loads of
// the kernarg segment (left alone, memcpyopt merged consecutive constellation loads into a copy
// of c.re into a private array, i.e. scratch memory, once Const held 64 points).
__device__ __forceinline__ float kval(const float& x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

// Policy interface (per lane; `sec` is the caller's local section id):
//   void load(int sec, int m, float& rr, float& ri, float& inv_tau) const;
//   void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const;
//   void section(int sec, float secmax, float secabs) const;     // group lane 0
// KK: the constellation size as a compile-time constant (1, 2, 4, 8, 16 or 64).
//
// M <= 64 form (G = M lanes per section, compile-time): one position per lane, U sections
// per lane group in flight (independent dependency chains for the scheduler).  Everything is
// float32: Z and the exclusive sums Z - Z_m by group_sum_excl_c, 1 / Z by v_rcp_f32 (Z >= 1:
// the section max term is exp(0)).  The constellation is held in VGPRs (uniform values, but
// as SGPR operands they spill in the big fused kernels).  Section statistics (max logit,
// max |logit|, non-finite input) are kept per lane in float32 and folded into the float64
// PartAcc once at the end.
template <bool kVar, int KK, int U, int G, class P>
__device__ __forceinline__ void denoise_sections_g(const P& pol, int nsec, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    const int lane = threadIdx.x & 63, wave = dw.wave;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    const int nw = dw.nw;
    float cre[KK], cim[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) {
        cre[k] = kval(c.re[k]); cim[k] = kval(c.im[k]);
        asm volatile("" : "+v"(cre[k]), "+v"(cim[k]));
    }
    float st_abs = 0.f, st_min = INFINITY;
    bool st_bad = false;
    for (int base = wave * gpw * U; base < nsec; base += nw * gpw * U) {   // wave-uniform trip count
        int sec[U];
        bool act[U];
        float xk[U][KK], smax[U], sabs[U];
        float ur[U], ui[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            sec[u] = base + u * gpw + gid;
            act[u] = sec[u] < nsec;
            float rr, ri, it;
            pol.load(act[u] ? sec[u] : nsec - 1, g, rr, ri, it);
            ur[u] = rr * it; ui[u] = ri * it;   // c64 / f32 == multiply by the reciprocal
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (act[u]) st_bad |= !(fabsf(ur[u]) <= FLT_MAX && fabsf(ui[u]) <= FLT_MAX);
            float lmax = -FLT_MAX, lmin = FLT_MAX;
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                xk[u][k] = fmaf(ur[u], cre[k], ui[u] * cim[k]);
                lmax = fmaxf(lmax, xk[u][k]);
                lmin = fminf(lmin, xk[u][k]);
            }
            smax[u] = lmax;
            sabs[u] = fmaxf(lmax, -lmin);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { smax[u] = group_fmax_c<G>(smax[u]); sabs[u] = group_fmax_c<G>(sabs[u]); }
        float zt[U], ze[U], sr[U], si[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float zm = 0.f, a = 0.f, b = 0.f;
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                const float e = den_exp(xk[u][k], smax[u]);
                xk[u][k] = e;
                zm += e;
                a = fmaf(cre[k], e, a);
                b = fmaf(cim[k], e, b);
            }
            zt[u] = zm; ze[u] = 0.f; sr[u] = a; si[u] = b;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) group_sum_excl_c<G>(zt[u], ze[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float iz = den_rcp(zt[u]);
            const float xr = sr[u] * iz, xi = si[u] * iz;
            float var = 0.f;
            if (kVar) {
                float vs = 0.f;
#pragma unroll
                for (int k = 0; k < KK; ++k) {
                    const float dr = xr - cre[k], di = xi - cim[k];
                    vs = fmaf(fmaf(dr, dr, di * di), xk[u][k], vs);
                }
                var = (xr * xr + xi * xi) * (ze[u] * iz) + vs * iz;
            }
            if (act[u]) {
                pol.store(sec[u], g, xr, xi, var, pa);
                st_abs = nan_max(st_abs, sabs[u]);
                st_min = nan_min(st_min, smax[u]);
                if (g == 0) pol.section(sec[u], smax[u], sabs[u]);
            }
        }
    }
    pa.maxabs = st_bad ? __longlong_as_double(0x7ff8000000000000LL) : nan_max(pa.maxabs, (double)st_abs);
    pa.minsecmax = nan_min(pa.minsecmax, (double)st_min);
}

// Packed-math form of denoise_sections_g (KK even): the per-symbol work runs on
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 over pairs — two symbols per instruction for
// the logits and their shift, the (re, im) pair for the sums and the variance — so one
// position costs ~140 VALU instructions instead of ~300.  Same rounding per element as the
// scalar form (each packed lane is the same IEEE operation).
typedef float f32x2 __attribute__((ext_vector_type(2)));

// The constellation as packed operands, kept in VGPRs: (re_k, re_k+1), (im_k, im_k+1) and
// (re_k, im_k).
template <int KK>
struct DenRegs {
    f32x2 pre[KK / 2], pim[KK / 2], sym[KK];
    __device__ __forceinline__ void load(const Const& c) {
#pragma unroll
        for (int h = 0; h < KK / 2; ++h) {
            pre[h] = f32x2{kval(c.re[2 * h]), kval(c.re[2 * h + 1])};
            pim[h] = f32x2{kval(c.im[2 * h]), kval(c.im[2 * h + 1])};
            asm volatile("" : "+v"(pre[h]), "+v"(pim[h]));
        }
#pragma unroll
        for (int k = 0; k < KK; ++k) {
            sym[k] = f32x2{kval(c.re[k]), kval(c.im[k])};
            asm volatile("" : "+v"(sym[k]));
        }
    }
};

// Diagnostic hook (amp_vamp_debug_dump): a policy may record the intermediate ze / vs of the
// variance; the generic form records nothing.
template <class P>
__device__ __forceinline__ void den_debug(const P&, int, int, float, float) {}

// Per-lane section statistics, folded into the float64 PartAcc once at the end.
struct DenStat {
    float st_abs = 0.f, st_min = INFINITY;
    bool st_bad = false;
    __device__ __forceinline__ void fold(PartAcc& pa) const {
        pa.maxabs = st_bad ? __longlong_as_double(0x7ff8000000000000LL) : nan_max(pa.maxabs, (double)st_abs);
        pa.minsecmax = nan_min(pa.minsecmax, (double)st_min);
    }
};

// One step of the packed denoiser: sections base + u * gpw + gid (u < U) of this wave.
// FULL: every one of them exists (< nsec): no branches at all, so the step can be scheduled
// into a surrounding MFMA stream (the section statistics are then stored by every lane of the
// group — the same value).
template <bool kVar, int KK, int U, int G, bool FULL, class P>
__device__ __forceinline__ void denoise_step_gp(const P& pol, int base, int nsec, const DenRegs<KK>& R, PartAcc& pa,
                                                DenStat& S) {
    static_assert(KK % 2 == 0, "packed form needs an even constellation size");
    constexpr int KH = KK / 2;
    const int lane = threadIdx.x & 63;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    int sec[U];
    bool act[U];
    f32x2 xk[U][KH];
    float smax[U], sabs[U], ur[U], ui[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        sec[u] = base + u * gpw + gid;
        act[u] = FULL || sec[u] < nsec;
        float rr, ri, it;
        pol.load(act[u] ? sec[u] : nsec - 1, g, rr, ri, it);
        ur[u] = rr * it; ui[u] = ri * it;   // c64 / f32 == multiply by the reciprocal
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool bad = !(fabsf(ur[u]) <= FLT_MAX && fabsf(ui[u]) <= FLT_MAX);
        S.st_bad |= act[u] && bad;
        const f32x2 u2 = f32x2{ur[u], ur[u]}, v2 = f32x2{ui[u], ui[u]};
        float lmax = -FLT_MAX, lmin = FLT_MAX;
#pragma unroll
        for (int h = 0; h < KH; ++h) {
            xk[u][h] = __builtin_elementwise_fma(u2, R.pre[h], v2 * R.pim[h]);
            lmax = fmaxf(lmax, fmaxf(xk[u][h].x, xk[u][h].y));
            lmin = fminf(lmin, fminf(xk[u][h].x, xk[u][h].y));
        }
        smax[u] = lmax;
        sabs[u] = fmaxf(lmax, -lmin);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { smax[u] = group_fmax_c<G>(smax[u]); sabs[u] = group_fmax_c<G>(sabs[u]); }
    float zt[U], ze[U];
    f32x2 s2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const f32x2 m2 = f32x2{smax[u], smax[u]};
        const f32x2 l2 = f32x2{AMP_LOG2E, AMP_LOG2E};
        f32x2 z2 = f32x2{0.f, 0.f}, a2 = f32x2{0.f, 0.f};
#pragma unroll
        for (int h = 0; h < KH; ++h) {
#if AMP_DEN_EXACT_EXP
            const f32x2 e = f32x2{den_exp(xk[u][h].x, smax[u]), den_exp(xk[u][h].y, smax[u])};
            (void)m2; (void)l2;
#else
            const f32x2 d = (xk[u][h] - m2) * l2;
            const f32x2 e = f32x2{__builtin_amdgcn_exp2f(d.x), __builtin_amdgcn_exp2f(d.y)};
#endif
            xk[u][h] = e;
            z2 += e;
            a2 = __builtin_elementwise_fma(R.sym[2 * h], f32x2{e.x, e.x}, a2);
            a2 = __builtin_elementwise_fma(R.sym[2 * h + 1], f32x2{e.y, e.y}, a2);
        }
        zt[u] = z2.x + z2.y; ze[u] = 0.f; s2[u] = a2;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) group_sum_excl_c<G>(zt[u], ze[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const float iz = den_rcp(zt[u]);
        const f32x2 x2 = s2[u] * f32x2{iz, iz};
        float var = 0.f;
        if (kVar) {
            f32x2 v2 = f32x2{0.f, 0.f};
#pragma unroll
            for (int h = 0; h < KH; ++h) {
                const f32x2 d0 = x2 - R.sym[2 * h], d1 = x2 - R.sym[2 * h + 1];
                v2 = __builtin_elementwise_fma(d0 * d0, f32x2{xk[u][h].x, xk[u][h].x}, v2);
                v2 = __builtin_elementwise_fma(d1 * d1, f32x2{xk[u][h].y, xk[u][h].y}, v2);
            }
            var = (x2.x * x2.x + x2.y * x2.y) * (ze[u] * iz) + (v2.x + v2.y) * iz;
            den_debug(pol, sec[u], g, ze[u], v2.x + v2.y);
        }
        if (FULL) {
            pol.store(sec[u], g, x2.x, x2.y, var, pa);
            S.st_abs = nan_max(S.st_abs, sabs[u]);
            S.st_min = nan_min(S.st_min, smax[u]);
            pol.section(sec[u], smax[u], sabs[u]);
        } else if (act[u]) {
            pol.store(sec[u], g, x2.x, x2.y, var, pa);
            S.st_abs = nan_max(S.st_abs, sabs[u]);
            S.st_min = nan_min(S.st_min, smax[u]);
            if (g == 0) pol.section(sec[u], smax[u], sabs[u]);
        }
    }
}

// ---- Product-grid form (square QAM-like alphabets: Const::grid == R) ----
// Every point is (gre[i], gim[j]) of an R x R grid, so the logits and their exponentials factor
// over rows and columns:
//   xi_ij = X_i + Y_j,   X_i = Re(r / tau) gre_i,   Y_j = Im(r / tau) gim_j
//   exp(xi_ij - smax) = er_i ei_j f,  er_i = exp(X_i - max X), ei_j = exp(Y_j - max Y),
//                                     f = exp(max X + max Y - smax)
// and every per-position sum of vamp.py:113-118 is a sum over rows of a row factor times a
// column sum weighted by the table's multiplicities c_ij (0, 1, 2; all 1 for a full grid):
//   z_m = f sum_i er_i S_i,           S_i = sum_j c_ij ei_j
//   sum_k a_k eta_k = f (sum_i gre_i er_i S_i, sum_i er_i T_i),   T_i = sum_j c_ij gim_j ei_j
//   sum_k |x - a_k|^2 eta_k = f sum_i er_i ((Re x - gre_i)^2 S_i + V_i),
//                                     V_i = sum_j c_ij (Im x - gim_j)^2 ei_j
// A position costs 2R + 1 exponentials and O(R^2) FMAs (O(R) for a full grid) instead of K
// exponentials and ~12 K operations.  Every sum adds non-negative terms (a missing grid point
// has weight 0: nothing is subtracted), so nothing cancels; the float32 rounding differs from
// the direct form by a few ulp (the reference works in float64 throughout).  The max / min
// logit of a position are max X + max Y / min X + min Y: a linear form over the grid takes its
// extremes at the corners, which are in the table (checked on the host, amp_host.h).
// Multiplicity patterns of the grid points (compile-time, so the unrolled sums below fold:
// weight 0 drops a term, 1 is an add, 2 an FMA by 2):
//   GRID_FULL  every grid point once (QPSK, square 64-QAM);
//   GRID_REF16 the reference's 16-QAM table (config.py:112) on the sorted grid
//              {-3,-1,1,3}/sqrt(10): -1+3j twice, 1-3j missing.
enum { GRID_FULL = 1, GRID_REF16 = 2 };
template <int PAT>
__device__ __forceinline__ constexpr float grid_cnt(int i, int j) {
    if constexpr (PAT == GRID_REF16) return (i == 1 && j == 3) ? 2.f : (i == 2 && j == 0) ? 0.f : 1.f;
    else return 1.f;
}

template <int R>
struct GridRegs {
    float re[R], im[R];
    __device__ __forceinline__ void load(const Const& c) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            re[i] = kval(c.gre[i]); im[i] = kval(c.gim[i]);
            asm volatile("" : "+v"(re[i]), "+v"(im[i]));
        }
    }
};

template <bool kVar, int R, int PAT, int U, int G, class P>
__device__ __forceinline__ void denoise_step_grid(const P& pol, int base, int nsec, const GridRegs<R>& Q,
                                                  PartAcc& pa, DenStat& S) {
    constexpr bool FULLG = PAT == GRID_FULL;
    const int lane = threadIdx.x & 63;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    int sec[U];
    bool act[U];
    float X[U][R], Y[U][R], mx[U], my[U], lmx[U], smax[U], sabs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        sec[u] = base + u * gpw + gid;
        act[u] = sec[u] < nsec;
        float rr, ri, it;
        pol.load(act[u] ? sec[u] : nsec - 1, g, rr, ri, it);
        const float ur = rr * it, ui = ri * it;   // c64 / f32 == multiply by the reciprocal
        S.st_bad |= act[u] && !(fabsf(ur) <= FLT_MAX && fabsf(ui) <= FLT_MAX);
        float ax = -FLT_MAX, nx = FLT_MAX, ay = -FLT_MAX, ny = FLT_MAX;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            X[u][i] = ur * Q.re[i];
            Y[u][i] = ui * Q.im[i];
            ax = fmaxf(ax, X[u][i]); nx = fminf(nx, X[u][i]);
            ay = fmaxf(ay, Y[u][i]); ny = fminf(ny, Y[u][i]);
        }
        mx[u] = ax; my[u] = ay;
        lmx[u] = ax + ay;                          // max logit of the position (a corner)
        smax[u] = lmx[u];
        sabs[u] = fmaxf(lmx[u], -(nx + ny));       // max |logit|
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { smax[u] = group_fmax_c<G>(smax[u]); sabs[u] = group_fmax_c<G>(sabs[u]); }
    float zt[U], ze[U], ar[U], ai[U], f[U];
    float er[U][R], ei[U][R], Sr[U][FULLG ? 1 : R];
    float SI[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        f[u] = den_exp(lmx[u], smax[u]);
#pragma unroll
        for (int i = 0; i < R; ++i) {
            er[u][i] = den_exp(X[u][i], mx[u]);
            ei[u][i] = den_exp(Y[u][i], my[u]);
        }
        if constexpr (FULLG) {
            float sr = 0.f, si = 0.f, a = 0.f, b = 0.f;
#pragma unroll
            for (int i = 0; i < R; ++i) {
                sr += er[u][i]; si += ei[u][i];
                a = fmaf(Q.re[i], er[u][i], a);
                b = fmaf(Q.im[i], ei[u][i], b);
            }
            SI[u] = si; Sr[u][0] = sr;
            zt[u] = (sr * si) * f[u];
            ar[u] = (a * si) * f[u];
            ai[u] = (sr * b) * f[u];
        } else {
            float z = 0.f, a = 0.f, b = 0.f, w[R];
#pragma unroll
            for (int j = 0; j < R; ++j) w[j] = Q.im[j] * ei[u][j];
#pragma unroll
            for (int i = 0; i < R; ++i) {
                float si = 0.f, ti = 0.f;
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const float cw = grid_cnt<PAT>(i, j);
                    if (cw == 1.f) { si += ei[u][j]; ti += w[j]; }
                    else if (cw == 2.f) { si = fmaf(2.f, ei[u][j], si); ti = fmaf(2.f, w[j], ti); }
                }
                Sr[u][i] = si;
                const float es = er[u][i] * si;
                z += es;
                a = fmaf(Q.re[i], es, a);
                b = fmaf(er[u][i], ti, b);
            }
            zt[u] = z * f[u];
            ar[u] = a * f[u];
            ai[u] = b * f[u];
        }
        ze[u] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) group_sum_excl_c<G>(zt[u], ze[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const float iz = den_rcp(zt[u]);
        const float xr = ar[u] * iz, xi = ai[u] * iz;
        float var = 0.f;
        if (kVar) {
            float vs;
            if constexpr (FULLG) {
                float vr = 0.f, vi = 0.f;
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const float dr = xr - Q.re[i], di = xi - Q.im[i];
                    vr = fmaf(dr * dr, er[u][i], vr);
                    vi = fmaf(di * di, ei[u][i], vi);
                }
                vs = fmaf(vr, SI[u], Sr[u][0] * vi) * f[u];
            } else {
                float d[R];
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const float di = xi - Q.im[j];
                    d[j] = (di * di) * ei[u][j];
                }
                float acc = 0.f;
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    float vi = 0.f;
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        const float cw = grid_cnt<PAT>(i, j);
                        if (cw == 1.f) vi += d[j];
                        else if (cw == 2.f) vi = fmaf(2.f, d[j], vi);
                    }
                    const float dr = xr - Q.re[i];
                    acc = fmaf(er[u][i], fmaf(dr * dr, Sr[u][i], vi), acc);
                }
                vs = acc * f[u];
            }
            var = (xr * xr + xi * xi) * (ze[u] * iz) + vs * iz;
        }
        if (act[u]) {
            pol.store(sec[u], g, xr, xi, var, pa);
            S.st_abs = nan_max(S.st_abs, sabs[u]);
            S.st_min = nan_min(S.st_min, smax[u]);
            if (g == 0) pol.section(sec[u], smax[u], sabs[u]);
        }
    }
}

// denoise_step_grid with U = 2 written on float pairs (one element per section in flight): the
// same operations in the same order per element — bit-identical results — issued as packed
// v_pk_mul / v_pk_add / v_pk_fma (two positions per instruction); max / min, exp, rcp and the
// DPP reductions stay per element.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v f2fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v f2splat(float v) { return f2v{v, v}; }

template <bool kVar, int R, int PAT, int G, class P>
__device__ __forceinline__ void denoise_step_grid2(const P& pol, int base, int nsec, const GridRegs<R>& Q,
                                                   PartAcc& pa, DenStat& S) {
    constexpr bool FULLG = PAT == GRID_FULL;
    const int lane = threadIdx.x & 63;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    int sec[2];
    bool act[2];
    f2v ur, ui;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        sec[u] = base + u * gpw + gid;
        act[u] = sec[u] < nsec;
        float rr, ri, it;
        pol.load(act[u] ? sec[u] : nsec - 1, g, rr, ri, it);
        ur[u] = rr * it;   // c64 / f32 == multiply by the reciprocal
        ui[u] = ri * it;
        S.st_bad |= act[u] && !(fabsf(ur[u]) <= FLT_MAX && fabsf(ui[u]) <= FLT_MAX);
    }
    f2v X[R], Y[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        X[i] = ur * f2splat(Q.re[i]);
        Y[i] = ui * f2splat(Q.im[i]);
    }
    f2v mx, my, lmx, smax, sabs;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float ax = -FLT_MAX, nx = FLT_MAX, ay = -FLT_MAX, ny = FLT_MAX;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            ax = fmaxf(ax, X[i][u]); nx = fminf(nx, X[i][u]);
            ay = fmaxf(ay, Y[i][u]); ny = fminf(ny, Y[i][u]);
        }
        mx[u] = ax; my[u] = ay;
        lmx[u] = ax + ay;                          // max logit of the position (a corner)
        smax[u] = group_fmax_c<G>(lmx[u]);
        sabs[u] = group_fmax_c<G>(fmaxf(lmx[u], -(nx + ny)));   // max |logit|
    }
    const f2v l2e = f2splat(AMP_LOG2E);
#if AMP_DEN_EXACT_EXP
    f2v f = {den_exp(lmx.x, smax.x), den_exp(lmx.y, smax.y)};
#else
    f2v targ = (lmx - smax) * l2e;
    f2v f = {__builtin_amdgcn_exp2f(targ.x), __builtin_amdgcn_exp2f(targ.y)};
#endif
    f2v er[R], ei[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
#if AMP_DEN_EXACT_EXP
        er[i] = f2v{den_exp(X[i].x, mx.x), den_exp(X[i].y, mx.y)};
        ei[i] = f2v{den_exp(Y[i].x, my.x), den_exp(Y[i].y, my.y)};
#else
        const f2v xa = (X[i] - mx) * l2e, ya = (Y[i] - my) * l2e;
        er[i] = f2v{__builtin_amdgcn_exp2f(xa.x), __builtin_amdgcn_exp2f(xa.y)};
        ei[i] = f2v{__builtin_amdgcn_exp2f(ya.x), __builtin_amdgcn_exp2f(ya.y)};
#endif
    }
    f2v zt, ar, ai, SI = f2splat(0.f);
    f2v Sr[FULLG ? 1 : R];
    if constexpr (FULLG) {
        f2v sr = f2splat(0.f), si = f2splat(0.f), a = f2splat(0.f), b = f2splat(0.f);
#pragma unroll
        for (int i = 0; i < R; ++i) {
            sr += er[i]; si += ei[i];
            a = f2fma(f2splat(Q.re[i]), er[i], a);
            b = f2fma(f2splat(Q.im[i]), ei[i], b);
        }
        SI = si; Sr[0] = sr;
        zt = (sr * si) * f;
        ar = (a * si) * f;
        ai = (sr * b) * f;
    } else {
        f2v z = f2splat(0.f), a = f2splat(0.f), b = f2splat(0.f), w[R];
#pragma unroll
        for (int j = 0; j < R; ++j) w[j] = f2splat(Q.im[j]) * ei[j];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            f2v si = f2splat(0.f), ti = f2splat(0.f);
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const float cw = grid_cnt<PAT>(i, j);
                if (cw == 1.f) { si += ei[j]; ti += w[j]; }
                else if (cw == 2.f) { si = f2fma(f2splat(2.f), ei[j], si); ti = f2fma(f2splat(2.f), w[j], ti); }
            }
            Sr[i] = si;
            const f2v es = er[i] * si;
            z += es;
            a = f2fma(f2splat(Q.re[i]), es, a);
            b = f2fma(er[i], ti, b);
        }
        zt = z * f;
        ar = a * f;
        ai = b * f;
    }
    float ze[2] = {0.f, 0.f}, zt1[2] = {zt.x, zt.y};
#pragma unroll
    for (int u = 0; u < 2; ++u) group_sum_excl_c<G>(zt1[u], ze[u]);
    const f2v iz = {den_rcp(zt1[0]), den_rcp(zt1[1])};
    const f2v xr = ar * iz, xi = ai * iz;
    f2v var = f2splat(0.f);
    if (kVar) {
        f2v vs;
        if constexpr (FULLG) {
            f2v vr = f2splat(0.f), vi = f2splat(0.f);
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const f2v dr = xr - f2splat(Q.re[i]), di = xi - f2splat(Q.im[i]);
                vr = f2fma(dr * dr, er[i], vr);
                vi = f2fma(di * di, ei[i], vi);
            }
            vs = f2fma(vr, SI, Sr[0] * vi) * f;
        } else {
            f2v d[R];
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const f2v di = xi - f2splat(Q.im[j]);
                d[j] = (di * di) * ei[j];
            }
            f2v acc = f2splat(0.f);
#pragma unroll
            for (int i = 0; i < R; ++i) {
                f2v vi = f2splat(0.f);
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const float cw = grid_cnt<PAT>(i, j);
                    if (cw == 1.f) vi += d[j];
                    else if (cw == 2.f) vi = f2fma(f2splat(2.f), d[j], vi);
                }
                const f2v dr = xr - f2splat(Q.re[i]);
                acc = f2fma(er[i], f2fma(dr * dr, Sr[i], vi), acc);
            }
            vs = acc * f;
        }
        const f2v zev = {ze[0], ze[1]};
        var = (xr * xr + xi * xi) * (zev * iz) + vs * iz;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (act[u]) {
            pol.store(sec[u], g, xr[u], xi[u], var[u], pa);
            S.st_abs = nan_max(S.st_abs, sabs[u]);
            S.st_min = nan_min(S.st_min, smax[u]);
            if (g == 0) pol.section(sec[u], smax[u], sabs[u]);
        }
    }
}

#ifndef AMP_DEN_PACKED_GRID
#define AMP_DEN_PACKED_GRID 1
#endif

// Grid dimension of a compile-time constellation size (0: no product-grid form).
template <int KK>
constexpr int grid_r() { return KK == 4 ? 2 : KK == 16 ? 4 : KK == 64 ? 8 : 0; }

// The grid loop over this wave's sections; returns false (nothing done) when c is not a grid of
// the size KK admits.  c.grid / c.gfull are kernel arguments: the branch is uniform.
template <bool kVar, int KK, int U, int G, bool PKG = true, class P>
__device__ __forceinline__ bool denoise_sections_grid(const P& pol, int nsec, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    constexpr int R = grid_r<KK>();
    if constexpr (R == 0) {
        return false;
    } else {
        const int grid = __builtin_amdgcn_readfirstlane(c.grid), gfull = __builtin_amdgcn_readfirstlane(c.gfull);
        if (grid != R) return false;
        const int wave = dw.wave;
        constexpr int gpw = 64 / G;
        const int nw = dw.nw;
        DenStat S;
        GridRegs<R> Q;
        Q.load(c);
        if (gfull == GRID_FULL) {
            for (int base = wave * gpw * U; base < nsec; base += nw * gpw * U) {   // wave-uniform trip count
                if constexpr (PKG && U == 2 && AMP_DEN_PACKED_GRID)
                    denoise_step_grid2<kVar, R, GRID_FULL, G>(pol, base, nsec, Q, pa, S);
                else
                    denoise_step_grid<kVar, R, GRID_FULL, U, G>(pol, base, nsec, Q, pa, S);
            }
        } else if constexpr (R == 4) {
            for (int base = wave * gpw * U; base < nsec; base += nw * gpw * U) {
                if constexpr (PKG && U == 2 && AMP_DEN_PACKED_GRID)
                    denoise_step_grid2<kVar, R, GRID_REF16, G>(pol, base, nsec, Q, pa, S);
                else
                    denoise_step_grid<kVar, R, GRID_REF16, U, G>(pol, base, nsec, Q, pa, S);
            }
        }
        S.fold(pa);
        return true;
    }
}

template <bool kVar, int KK, int U, int G, class P>
__device__ __forceinline__ void denoise_sections_gp(const P& pol, int nsec, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    if (denoise_sections_grid<kVar, KK, U, G>(pol, nsec, c, pa, dw)) return;
    const int wave = dw.wave;
    constexpr int gpw = 64 / G;
    const int nw = dw.nw;
    DenRegs<KK> R;
    R.load(c);
    DenStat S;
    for (int base = wave * gpw * U; base < nsec; base += nw * gpw * U)   // wave-uniform trip count
        denoise_step_gp<kVar, KK, U, G, false>(pol, base, nsec, R, pa, S);
    S.fold(pa);
}

// Which float32 forms run on the packed VALU (v_pk_*_f32):
//   PK_NONE  every float32 operation scalar (the product grid still applies);
//   PK_ALL   the packed per-point form (denoise_step_gp) and the packed product grid (grid2);
//   PK_GRID  the packed product grid only; alphabets that are not a grid of the compile-time
//            size (16PSK at KK = 16, QPSK {1, j, -1, -j}) run the scalar per-point form.
// The engines that place two waves on one SIMD use PK_NONE or PK_GRID, because there the packed
// per-point variance accumulation of denoise_step_gp was measured to lose one half of a
// v_pk_fma_f32 result in lanes 48-63 now and then (results not reproducible run to
// run; the scalar form was bit-identical in every run).  PK_ALL == true keeps the old bool callers.
enum { PK_NONE = 0, PK_ALL = 1, PK_GRID = 2 };

// Runtime M (a power of two <= 64) -> the compile-time group size.
template <bool kVar, int KK, int U, int G, int PK, class P>
__device__ __forceinline__ void denoise_sections_sel(const P& pol, int nsec, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    if constexpr (PK == PK_ALL && KK % 2 == 0) {
        denoise_sections_gp<kVar, KK, U, G>(pol, nsec, c, pa, dw);
    } else {
        if (denoise_sections_grid<kVar, KK, U, G, PK == PK_GRID>(pol, nsec, c, pa, dw)) return;
        denoise_sections_g<kVar, KK, U, G>(pol, nsec, c, pa, dw);
    }
}
template <bool kVar, int KK, int U, int PK = PK_ALL, class P>
__device__ __forceinline__ void denoise_sections_u(const P& pol, int nsec, int M, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    switch (M) {
    case 64: denoise_sections_sel<kVar, KK, U, 64, PK>(pol, nsec, c, pa, dw); break;
    case 32: denoise_sections_sel<kVar, KK, U, 32, PK>(pol, nsec, c, pa, dw); break;
    case 16: denoise_sections_sel<kVar, KK, U, 16, PK>(pol, nsec, c, pa, dw); break;
    case 8: denoise_sections_sel<kVar, KK, U, 8, PK>(pol, nsec, c, pa, dw); break;
    case 4: denoise_sections_sel<kVar, KK, U, 4, PK>(pol, nsec, c, pa, dw); break;
    case 2: denoise_sections_sel<kVar, KK, U, 2, PK>(pol, nsec, c, pa, dw); break;
    default: denoise_sections_sel<kVar, KK, U, 1, PK>(pol, nsec, c, pa, dw); break;
    }
}

// 64-QAM form (KK > 16): the same arithmetic per element as denoise_sections_g, but the 64
// points are streamed from the scalar cache in chunks of 8 (rolled loop: 128 uniform operands
// do not fit the scalar register file) and nothing per point is kept in registers — the
// logits are re-formed in each of the three passes (max, exp sums, variance) and the
// variance pass recomputes exp(xi - max): the same bits as the first exp (2 x 64 v_exp_f32
// per position instead of 64, against 5 GEMM launches per iteration at cfg5).
// One position per lane (G = M <= 64 lanes per section).
template <bool kVar, int KK, int G, class P>
__device__ __forceinline__ void denoise_sections_wide(const P& pol, int nsec, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    static_assert(KK % 8 == 0, "chunks of 8 points");
    if (denoise_sections_grid<kVar, KK, 1, G>(pol, nsec, c, pa, dw)) return;   // square 64-QAM
    const int lane = threadIdx.x & 63, wave = dw.wave;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    const int nw = dw.nw;
    // the table in LDS: the rolled loops below index it at runtime, which on the by-value kernel
    // argument made the compiler copy the whole Const into scratch memory at every kernel entry
    __shared__ float s_cre[KK], s_cim[KK];
    __syncthreads();
    if (threadIdx.x == 0) {   // constant offsets into the kernel argument (scalar loads)
#pragma unroll
        for (int k = 0; k < KK; ++k) { s_cre[k] = kval(c.re[k]); s_cim[k] = kval(c.im[k]); }
    }
    __syncthreads();
    DenStat S;
    for (int base = wave * gpw; base < nsec; base += nw * gpw) {   // wave-uniform trip count
        const int sec = base + gid;
        const bool act = sec < nsec;
        float rr, ri, it;
        pol.load(act ? sec : nsec - 1, g, rr, ri, it);
        const float ur = rr * it, ui = ri * it;   // c64 / f32 == multiply by the reciprocal
        if (act) S.st_bad |= !(fabsf(ur) <= FLT_MAX && fabsf(ui) <= FLT_MAX);
        float lmax = -FLT_MAX, lmin = FLT_MAX;
#pragma unroll 1
        for (int k0 = 0; k0 < KK; k0 += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float x = fmaf(ur, s_cre[k0 + j], ui * s_cim[k0 + j]);
                lmax = fmaxf(lmax, x);
                lmin = fminf(lmin, x);
            }
        }
        const float smax = group_fmax_c<G>(lmax), sabs = group_fmax_c<G>(fmaxf(lmax, -lmin));
        float zm = 0.f, a = 0.f, b = 0.f;
#pragma unroll 1
        for (int k0 = 0; k0 < KK; k0 += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float cr = s_cre[k0 + j], ci = s_cim[k0 + j];
                const float e = den_exp(fmaf(ur, cr, ui * ci), smax);
                zm += e;
                a = fmaf(cr, e, a);
                b = fmaf(ci, e, b);
            }
        }
        float zt = zm, ze = 0.f;
        group_sum_excl_c<G>(zt, ze);
        const float iz = den_rcp(zt);
        const float xr = a * iz, xi = b * iz;
        float var = 0.f;
        if (kVar) {
            float vs = 0.f;
#pragma unroll 1
            for (int k0 = 0; k0 < KK; k0 += 8) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float cr = s_cre[k0 + j], ci = s_cim[k0 + j];
                    const float e = den_exp(fmaf(ur, cr, ui * ci), smax);
                    const float dr = xr - cr, di = xi - ci;
                    vs = fmaf(fmaf(dr, dr, di * di), e, vs);
                }
            }
            var = (xr * xr + xi * xi) * (ze * iz) + vs * iz;
        }
        if (act) {
            pol.store(sec, g, xr, xi, var, pa);
            S.st_abs = nan_max(S.st_abs, sabs);
            S.st_min = nan_min(S.st_min, smax);
            if (g == 0) pol.section(sec, smax, sabs);
        }
    }
    S.fold(pa);
}

template <bool kVar, int KK, class P>
__device__ __forceinline__ void denoise_sections_wide_m(const P& pol, int nsec, int M, const Const& c, PartAcc& pa, DenWaves dw = DenWaves::block()) {
    switch (M) {
    case 64: denoise_sections_wide<kVar, KK, 64>(pol, nsec, c, pa, dw); break;
    case 32: denoise_sections_wide<kVar, KK, 32>(pol, nsec, c, pa, dw); break;
    case 16: denoise_sections_wide<kVar, KK, 16>(pol, nsec, c, pa, dw); break;
    case 8: denoise_sections_wide<kVar, KK, 8>(pol, nsec, c, pa, dw); break;
    case 4: denoise_sections_wide<kVar, KK, 4>(pol, nsec, c, pa, dw); break;
    case 2: denoise_sections_wide<kVar, KK, 2>(pol, nsec, c, pa, dw); break;
    default: denoise_sections_wide<kVar, KK, 1>(pol, nsec, c, pa, dw); break;
    }
}

template <bool kVar, int KK, class P>
__device__ __forceinline__ void denoise_sections(const P& pol, int nsec, int M, const Const& c, PartAcc& pa) {
    if constexpr (KK > 16) {
        // 64-QAM: M <= 64 (check_dims); the generic M > 64 form below is not instantiated (its
        // registers would set the whole kernel's occupancy)
        denoise_sections_wide_m<kVar, KK>(pol, nsec, M, c, pa);
        return;
    } else {
    if (M <= 64) {
        denoise_sections_u<kVar, KK, 1>(pol, nsec, M, c, pa);
        return;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int G = M < 64 ? M : 64;
    const int PPL = M / G;
    const int gpw = 64 / G;
    const int gid = lane / G, g = lane - gid * G;
    const int nw = blockDim.x >> 6;
    for (int base = wave * gpw; base < nsec; base += nw * gpw) {   // wave-uniform trip count
        const int sec = base + gid;
        const bool act = sec < nsec;
        const int ss = act ? sec : nsec - 1;
        float lmax = -FLT_MAX, lmin = FLT_MAX;
        bool bad = false;
        {
            // M > 64: PPL positions per lane, logits recomputed per pass.
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
                bad |= !(fabsf(ur) <= FLT_MAX && fabsf(ui) <= FLT_MAX);
#pragma unroll
                for (int k = 0; k < KK; ++k) {
                    {
                        const float x = fmaf(ur, c.re[k], ui * c.im[k]);
                        lmax = fmaxf(lmax, x);
                        lmin = fminf(lmin, x);
                    }
                }
            }
            const float smax = group_fmax(lmax, 64);
            double zl = 0.0;
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
                float zm = 0.f;
#pragma unroll
                for (int k = 0; k < KK; ++k)
                    zm += __builtin_amdgcn_exp2f((fmaf(ur, c.re[k], ui * c.im[k]) - smax) * AMP_LOG2E);
                zl += (double)zm;
            }
            const double z = group_sum(zl, 64);
            const double iz = 1.0 / z;
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
                float zm = 0.f, sr = 0.f, si = 0.f;
                float ek[KK];
#pragma unroll
                for (int k = 0; k < KK; ++k) {
                    {
                        const float e = __builtin_amdgcn_exp2f((fmaf(ur, c.re[k], ui * c.im[k]) - smax) * AMP_LOG2E);
                        ek[k] = e;
                        zm += e;
                        sr = fmaf(c.re[k], e, sr);
                        si = fmaf(c.im[k], e, si);
                    }
                }
                const float xr = (float)((double)sr * iz), xi = (float)((double)si * iz);
                float var = 0.f;
                if (kVar) {
                    const float omp = (float)((z - (double)zm) * iz);
                    float vs = 0.f;
#pragma unroll
                    for (int k = 0; k < KK; ++k) {
                        {
                            const float dr = xr - c.re[k], di = xi - c.im[k];
                            vs = fmaf(fmaf(dr, dr, di * di), ek[k], vs);
                        }
                    }
                    var = (xr * xr + xi * xi) * omp + (float)((double)vs * iz);
                }
                if (act) pol.store(sec, g + p * 64, xr, xi, var, pa);
            }
            const float sabs = group_fmax(fmaxf(lmax, -lmin), 64);
            if (act) {
                const double sm = (double)smax, sa = (double)sabs;
                pa.maxabs = bad ? __longlong_as_double(0x7ff8000000000000LL) : nan_max(pa.maxabs, sa);
                pa.minsecmax = nan_min(pa.minsecmax, sm);
                if (g == 0) pol.section(sec, (float)sm, (float)sa);
            }
        }
    }
    }
}

// max |xi| of one section in float64, exactly as the reference forms the logits.
// ld(m, rr, ri, inv_tau).
template <class LD>
__device__ double section_absmax_f64(const LD& ld, int M, const Const64& c) {
    double mx = 0.0;
    for (int m = 0; m < M; ++m) {
        float rr, ri, it;
        ld(m, rr, ri, it);
        const double ur = (double)(rr * it), ui = (double)(ri * it);
        for (int k = 0; k < c.K; ++k) mx = fmax(mx, fabs(ur * c.re[k] + ui * c.im[k]));
    }
    return mx;
}

// Reference-exact float64 evaluation of ONE section with the batch-global shift G, for the
// sections whose reference softmax leaves the normal float64 range (AMP_DANGER): the exact
// op sequence of vamp.py:111-119 / bamp.py:69-77 / scamp.py:64-67 —
//   xi = Re((r*(1/tau)) conj a) (float64), eta = exp(xi - G), Z = sum_m sum_k eta,
//   xmmse = sum_k a eta / Z  (complex alphabets: * (1/Z), which is inf for a denormal Z;
//                             real alphabets: a true float64 division),
//   var = |xmmse|^2 (1 - Z_m / Z) + sum_k |xmmse - a_k|^2 eta / Z,
// so inf / NaN / denormal-quantised results come out exactly as the reference's do.
// One thread per section (rare path).  ld(m, rr, ri, inv_tau); st(m, xr, xi, var).
template <bool kVar, class LD, class ST>
__device__ void exact_section_f64(const LD& ld, const ST& st, int M, const Const64& c, double G) {
    const int K = c.K;
    double Z = 0.0;
    for (int m = 0; m < M; ++m) {
        float rr, ri, it;
        ld(m, rr, ri, it);
        const double ur = (double)(rr * it), ui = (double)(ri * it);
        double zm = 0.0;
        for (int k = 0; k < K; ++k) zm += exp((ur * c.re[k] + ui * c.im[k]) - G);
        Z += zm;
    }
    const double rz = 1.0 / Z;
    for (int m = 0; m < M; ++m) {
        float rr, ri, it;
        ld(m, rr, ri, it);
        const double ur = (double)(rr * it), ui = (double)(ri * it);
        double zm = 0.0, sr = 0.0, si = 0.0;
        for (int k = 0; k < K; ++k) {
            const double e = exp((ur * c.re[k] + ui * c.im[k]) - G);
            zm += e;
            sr += c.re[k] * e;
            si += c.im[k] * e;
        }
        double xr, xi;
        if (c.real_alpha) { xr = sr / Z; xi = 0.0; }
        else { xr = sr * rz; xi = si * rz; }
        float var = 0.f;
        if (kVar) {
            const double ax = c.real_alpha ? fabs(xr) : hypot(xr, xi);
            const double var0 = ax * ax * (1.0 - zm / Z);
            double vs = 0.0;
            for (int k = 0; k < K; ++k) {
                // eta recomputed (the same bits as above; no per-point array: 64-QAM)
                const double e = exp((ur * c.re[k] + ui * c.im[k]) - G);
                const double dr = xr - c.re[k], di = xi - c.im[k];
                const double h = c.real_alpha ? fabs(dr) : hypot(dr, di);
                vs += h * h * e;
            }
            var = (float)(var0 + vs / Z);
        }
        st(m, (float)xr, (float)xi, var);
    }
}

// The rare-path driver shared by the reduction kernels (one workgroup):
//  1. exact float64 batch max |xi| (G) from the sections whose float32 estimate is within the
//     fast path's slack of the float32 batch max;
//  2. exact recompute of every section whose max logit lies below G + AMP_DANGER (+ slack).
// secmax / secabs: per-section float32 estimates (natural units) written by the fast path.
// LDF(s) returns the section's loader; STF(s) its store functor.  Returns #recomputed
// sections (workgroup-uniform) and the exact G in *G_out.
template <bool kVar, class LDF, class STF>
__device__ int fixup_sections(int S, int M, const float* secmax, const float* secabs, double G32, const Const64& c,
                              const LDF& ldf, const STF& stf, double* G_out, double* lds_d) {
    const double slack = logit_slack(G32);
    double gm = 0.0;
    for (int s = threadIdx.x; s < S; s += blockDim.x)
        if ((double)secabs[s] >= G32 - slack) gm = fmax(gm, section_absmax_f64(ldf(s), M, c));
    gm = group_max(gm, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds_d[threadIdx.x >> 6] = gm;
    __syncthreads();
    double G = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) G = fmax(G, lds_d[w]);
    __syncthreads();
    int cnt = 0;
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
        if ((double)secmax[s] - G < AMP_DANGER + slack) {
            exact_section_f64<kVar>(ldf(s), stf(s), M, c, G);
            ++cnt;
        }
    }
    cnt = group_sum(cnt, 64);
    if ((threadIdx.x & 63) == 0) lds_d[threadIdx.x >> 6] = (double)cnt;
    __syncthreads();
    int total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) total += (int)lds_d[w];
    __syncthreads();
    *G_out = G;
    return total;
}

}  // namespace amp
