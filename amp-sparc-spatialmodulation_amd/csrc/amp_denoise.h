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
// The reference takes shift = max |xi| over the WHOLE batch and evaluates in float64,
// which makes a section 0/0 = NaN when all of its logits lie more than 745.13 below that
// global max.  Here each section is shifted by its own max (exact softmax, float32 exp,
// float64 section sum Z so 1 - P_m has no cancellation) and the kernel reports the
// section max and the block max|xi|; the NaN outcome is then applied by the caller
// from the batch-global reduction (SURVEY.md §8(a) A4 "NaN rule").
//
// Mapping: one section per group of G = min(M, 64) lanes (M a power of two), each lane
// owns PPL = M / G positions; reductions are xor-shuffles inside the group.
#pragma once

#include "amp_common.h"

namespace amp {

// Policy interface (all calls are per lane; `sec` is the caller's local section id):
//   void load(int sec, int m, float& rr, float& ri, float& inv_tau) const;
//   void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const;
//   void section(int sec, float secmax) const;     // called by the group's lane 0
template <bool kVar, class P>
__device__ __forceinline__ void denoise_sections(const P& pol, int nsec, int M, const Const& c, PartAcc& pa) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int G = M < 64 ? M : 64;
    const int PPL = M / G;
    const int gpw = 64 / G;
    const int gid = lane / G, g = lane - gid * G;
    const int K = c.K;
    for (int base = wave * gpw; base < nsec; base += (AMP_WG / 64) * gpw) {  // wave-uniform trip count
        const int sec = base + gid;
        const bool act = sec < nsec;
        const int ss = act ? sec : nsec - 1;
        if (PPL == 1) {
            float rr, ri, it;
            pol.load(ss, g, rr, ri, it);
            const float ur = rr * it, ui = ri * it;   // c64 / f32 == multiply by the reciprocal
            float xk[AMP_MAX_K];
            float lmax = -INFINITY, lmin = INFINITY;
            int kmax = 0, kmin = 0;
#pragma unroll
            for (int k = 0; k < AMP_MAX_K; ++k) {
                if (k < K) {
                    xk[k] = fmaf(ur, c.re[k], ui * c.im[k]);
                    if (xk[k] > lmax) { lmax = xk[k]; kmax = k; }
                    if (xk[k] < lmin) { lmin = xk[k]; kmin = k; }
                    if (xk[k] != xk[k]) lmax = lmin = xk[k];
                }
            }
            // the batch max |xi| and the section max in float64, as the reference forms them
            const double x64max = (double)ur * c.re64[kmax] + (double)ui * c.im64[kmax];
            const double x64min = (double)ur * c.re64[kmin] + (double)ui * c.im64[kmin];
            const double labs = (lmax != lmax) ? (double)lmax : nan_max(fabs(x64max), fabs(x64min));
            const double smax64 = group_max_nan((lmax != lmax) ? (double)lmax : x64max, G);
            const float smax = group_max_nan(lmax, G);
            float zm = 0.f, sr = 0.f, si = 0.f;
#pragma unroll
            for (int k = 0; k < AMP_MAX_K; ++k) {
                if (k < K) {
                    const float e = __expf(xk[k] - smax);
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
                for (int k = 0; k < AMP_MAX_K; ++k) {
                    if (k < K) {
                        const float dr = xr - c.re[k], di = xi - c.im[k];
                        vs = fmaf(fmaf(dr, dr, di * di), xk[k], vs);
                    }
                }
                var = (xr * xr + xi * xi) * omp + (float)((double)vs * iz);
            }
            if (act) {
                pol.store(sec, g, xr, xi, var, pa);
                pa.maxabs = nan_max(pa.maxabs, labs);
                pa.minsecmax = nan_min(pa.minsecmax, smax64);
                if (g == 0) pol.section(sec, smax64);
            }
        } else {
            // M > 64: PPL positions per lane, logits recomputed per pass.
            float lmax = -INFINITY;
            double lmax64 = -INFINITY, labs = 0.0;
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
#pragma unroll
                for (int k = 0; k < AMP_MAX_K; ++k) {
                    if (k < K) {
                        const float x = fmaf(ur, c.re[k], ui * c.im[k]);
                        const double x64 = (double)ur * c.re64[k] + (double)ui * c.im64[k];
                        lmax = nan_max(lmax, x);
                        lmax64 = nan_max(lmax64, x64);
                        labs = nan_max(labs, fabs(x64));
                    }
                }
            }
            const double smax64 = group_max_nan(lmax64, 64);
            const float smax = group_max_nan(lmax, 64);
            double zl = 0.0;
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
                float zm = 0.f;
#pragma unroll
                for (int k = 0; k < AMP_MAX_K; ++k)
                    if (k < K) zm += __expf(fmaf(ur, c.re[k], ui * c.im[k]) - smax);
                zl += (double)zm;
            }
            const double z = group_sum(zl, 64);
            const double iz = 1.0 / z;
            for (int p = 0; p < PPL; ++p) {
                float rr, ri, it;
                pol.load(ss, g + p * 64, rr, ri, it);
                const float ur = rr * it, ui = ri * it;
                float zm = 0.f, sr = 0.f, si = 0.f;
                float ek[AMP_MAX_K];
#pragma unroll
                for (int k = 0; k < AMP_MAX_K; ++k) {
                    if (k < K) {
                        const float e = __expf(fmaf(ur, c.re[k], ui * c.im[k]) - smax);
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
                    for (int k = 0; k < AMP_MAX_K; ++k) {
                        if (k < K) {
                            const float dr = xr - c.re[k], di = xi - c.im[k];
                            vs = fmaf(fmaf(dr, dr, di * di), ek[k], vs);
                        }
                    }
                    var = (xr * xr + xi * xi) * omp + (float)((double)vs * iz);
                }
                if (act) pol.store(sec, g + p * 64, xr, xi, var, pa);
            }
            if (act) {
                pa.maxabs = nan_max(pa.maxabs, labs);
                pa.minsecmax = nan_min(pa.minsecmax, smax64);
                if (g == 0) pol.section(sec, smax64);
            }
        }
    }
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
__device__ void exact_section_f64(const LD& ld, const ST& st, int M, const Const& c, double G) {
    const int K = c.K;
    double Z = 0.0;
    for (int m = 0; m < M; ++m) {
        float rr, ri, it;
        ld(m, rr, ri, it);
        const double ur = (double)(rr * it), ui = (double)(ri * it);
        double zm = 0.0;
        for (int k = 0; k < K; ++k) zm += exp((ur * c.re64[k] + ui * c.im64[k]) - G);
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
                const double e = exp((ur * c.re64[k] + ui * c.im64[k]) - G);
                eta[k] = e;
                zm += e;
                sr += c.re64[k] * e;
                si += c.im64[k] * e;
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
                    const double dr = xr - c.re64[k], di = xi - c.im64[k];
                    const double h = c.real_alpha ? fabs(dr) : hypot(dr, di);
                    vs += h * h * eta[k];
                }
            }
            var = (float)(var0 + vs / Z);
        }
        st(m, (float)xr, (float)xi, var);
    }
}

}  // namespace amp
