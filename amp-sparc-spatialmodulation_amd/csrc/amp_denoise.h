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

// Policy interface (per lane; `sec` is the caller's local section id):
//   void load(int sec, int m, float& rr, float& ri, float& inv_tau) const;
//   void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const;
//   void section(int sec, float secmax, float secabs) const;     // group lane 0
// KK: the constellation size as a compile-time constant (1, 2, 4, 8 or 16).
template <bool kVar, int KK, class P>
__device__ __forceinline__ void denoise_sections(const P& pol, int nsec, int M, const Const& c, PartAcc& pa) {
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
        if (PPL == 1) {
            float rr, ri, it;
            pol.load(ss, g, rr, ri, it);
            const float ur = rr * it, ui = ri * it;   // c64 / f32 == multiply by the reciprocal
            bad = !(fabsf(ur) <= FLT_MAX && fabsf(ui) <= FLT_MAX);
            float xk[KK];
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                {
                    xk[k] = fmaf(ur, c.re[k], ui * c.im[k]);
                    lmax = fmaxf(lmax, xk[k]);
                    lmin = fminf(lmin, xk[k]);
                }
            }
            const float smax = group_fmax(lmax, G);
            float zm = 0.f, sr = 0.f, si = 0.f;
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                {
                    const float e = __builtin_amdgcn_exp2f((xk[k] - smax) * AMP_LOG2E);
                    xk[k] = e;
                    zm += e;
                    sr = fmaf(c.re[k], e, sr);
                    si = fmaf(c.im[k], e, si);
                }
            }
            const double z = group_sum((double)zm, G);
            const double iz = 1.0 / z;
            const float xr = (float)((double)sr * iz), xi = (float)((double)si * iz);
            float var = 0.f;
            if (kVar) {
                const float omp = (float)((z - (double)zm) * iz);
                float vs = 0.f;
#pragma unroll
                for (int k = 0; k < KK; ++k) {
                    {
                        const float dr = xr - c.re[k], di = xi - c.im[k];
                        vs = fmaf(fmaf(dr, dr, di * di), xk[k], vs);
                    }
                }
                var = (xr * xr + xi * xi) * omp + (float)((double)vs * iz);
            }
            if (act) pol.store(sec, g, xr, xi, var, pa);
            const float sabs = group_fmax(fmaxf(lmax, -lmin), G);
            if (act) {
                const double sm = (double)smax, sa = (double)sabs;
                pa.maxabs = bad ? __longlong_as_double(0x7ff8000000000000LL) : nan_max(pa.maxabs, sa);
                pa.minsecmax = nan_min(pa.minsecmax, sm);
                if (g == 0) pol.section(sec, (float)sm, (float)sa);
            }
        } else {
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
        double eta[AMP_MAX_K];
        double zm = 0.0, sr = 0.0, si = 0.0;
#pragma unroll
        for (int k = 0; k < AMP_MAX_K; ++k) {
            if (k < K) {
                const double e = exp((ur * c.re[k] + ui * c.im[k]) - G);
                eta[k] = e;
                zm += e;
                sr += c.re[k] * e;
                si += c.im[k] * e;
            }
        }
        double xr, xi;
        if (c.real_alpha) { xr = sr / Z; xi = 0.0; }
        else { xr = sr * rz; xi = si * rz; }
        float var = 0.f;
        if (kVar) {
            const double ax = c.real_alpha ? fabs(xr) : hypot(xr, xi);
            const double var0 = ax * ax * (1.0 - zm / Z);
            double vs = 0.0;
#pragma unroll
            for (int k = 0; k < AMP_MAX_K; ++k) {
                if (k < K) {
                    const double dr = xr - c.re[k], di = xi - c.im[k];
                    const double h = c.real_alpha ? fabs(dr) : hypot(dr, di);
                    vs += h * h * eta[k];
                }
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
