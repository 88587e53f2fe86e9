// amp_shrink.hip — the element-wise shrinkage denoisers of Shrink (shrink.py:8-166).
//
// These are the reference's prior-based alternatives to the block-sparse section denoiser
// (amp_denoise.h): `bayes` (shrink.py:78-96, the denoiser of vamp2.py:46), `shrinkOOK`
// (shrink.py:139-157) and the section-wise leave-one-out `sw_shrinkOOK` (shrink.py:58-76).
// `shrink` and `lasso` (shrink.py:98-137) raise in the reference for every input (torch.sign
// of a complex tensor, an unbound local, a missing attribute), so they have no kernel; the
// host class raises the same exceptions.
//
// All three are streaming kernels over [count] elements (HBM-bound: 8-16 B in, 4-8 B out
// per element; the K exps of `bayes` are VALU work far below the memory time).  Every
// element is one lane; sw_shrinkOOK's section sums are xor-butterfly reductions inside a
// wavefront when M is a power of two <= 64, otherwise one wavefront walks a section.
//
// Arithmetic mirrors the reference's torch ops one rounding at a time (-ffp-contract=off):
// true float32 division for real / real, multiply-by-reciprocal for complex64 / float32
// (torch's c64 / f32), regularize_exp (shrink.py:163-166) as `v >= f32(log(FLT_MAX)) ->
// f32(log(FLT_MAX) - 1)`, regularize_zero (shrink.py:159-161) as `0 -> 1e-9f`.
#include <algorithm>

#include "amp_host.h"

namespace amp {

constexpr float SHR_REG_MAX = (float)88.72283905206835;   // np.log(torch.finfo(float32).max)
constexpr float SHR_REG_SET = (float)87.72283905206835;   // max - 1 (shrink.py:165)
constexpr float SHR_TOL = 1.0e-9f;                         // torch.tensor(1.0e-9) (shrink.py:28)

__device__ __forceinline__ float reg_exp(float v) { return v >= SHR_REG_MAX ? SHR_REG_SET : v; }

// expf whose denormal results are correctly rounded: ocml's expf returns 0 a little above the
// bottom of the denormal range where the reference's (CPU) exp still returns 2^-149, and that
// one denormal decides whether bayes' norm is 0 (-> 1e-9 -> 0) or a denormal whose reciprocal
// is inf (-> NaN).  Below log(FLT_MIN) the float64 exp rounded to float32 is used instead.
__device__ __forceinline__ float texpf(float v) {
    return v < -87.33654475f ? (float)exp((double)v) : expf(v);
}

struct ShrinkK {
    long long count;
    int cplx;             // r (and the bayes output) complex64, else float32
    int cov_vec;          // cov per element, else cov_scalar
    float cov_scalar;
    const float* r;       // float2 when cplx
    const float* cov;
    float p0, ps, theta;
    float sre[AMP_MAX_K], sim[AMP_MAX_K];
    int K;
    int M;                // sw_shrinkOOK section length
};

__device__ __forceinline__ void load_r(const ShrinkK& P, long long e, float& rr, float& ri) {
    if (P.cplx) {
        const float2 v = reinterpret_cast<const float2*>(P.r)[e];
        rr = v.x; ri = v.y;
    } else {
        rr = P.r[e]; ri = 0.0f;
    }
}
__device__ __forceinline__ float load_cov(const ShrinkK& P, long long e) { return P.cov_vec ? P.cov[e] : P.cov_scalar; }

// |z| as torch.abs: correctly rounded hypot for complex64, fabs for float32.
__device__ __forceinline__ float tabs(bool cplx, float re, float im) { return cplx ? hypotf(re, im) : fabsf(re); }

// bayes (shrink.py:91-96):  G(s) = exp(-|r-s|^2/cov); norm = regularize_zero(P0 G(0) + Ps sum_k G(a_k));
// exp = Ps * sum_k a_k G(a_k) / norm.
template <int KK>
__global__ __launch_bounds__(AMP_WG) void shrink_bayes_kernel(ShrinkK P, float* out) {
    const bool cplx = P.cplx != 0;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < P.count;
         e += (long long)gridDim.x * blockDim.x) {
        float rr, ri;
        load_r(P, e, rr, ri);
        const float cov = load_cov(P, e);
        float a0 = tabs(cplx, rr, ri);
        const float g0 = texpf(-(a0 * a0) / cov);
        float gs = 0.0f, xr = 0.0f, xi = 0.0f;
        constexpr int KU = KK > 16 ? 8 : KK;   // 64-QAM: chunks of 8 uniform operands
#pragma unroll KU
        for (int k = 0; k < KK; ++k) {
            const float dr = rr - P.sre[k], di = ri - P.sim[k];
            const float a = tabs(cplx, dr, di);
            const float g = texpf(-(a * a) / cov);
            gs = gs + g;
            xr = xr + P.sre[k] * g;
            xi = xi + P.sim[k] * g;
        }
        float norm = P.p0 * g0 + P.ps * gs;
        if (norm == 0.0f) norm = SHR_TOL;
        xr = P.ps * xr;
        xi = P.ps * xi;
        if (cplx) {
            const float inv = 1.0f / norm;
            reinterpret_cast<float2*>(out)[e] = make_float2(xr * inv, xi * inv);
        } else {
            out[e] = xr / norm;
        }
    }
}

// shrinkOOK (shrink.py:152-156): eta = exp(reg(theta + (1 - 2 Re r)/cov)); exp = 1/(1 + eta + tol);
// der = nan_to_num(2 eta exp^2 / cov); block partial sums of der (float64) for dxdr = der.mean().
__global__ __launch_bounds__(AMP_WG) void shrink_ook_kernel(ShrinkK P, float* out, double* parts) {
    __shared__ double s_part[AMP_WG / AMP_WAVE];
    double acc = 0.0;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < P.count;
         e += (long long)gridDim.x * blockDim.x) {
        float rr, ri;
        load_r(P, e, rr, ri);
        const float cov = load_cov(P, e);
        const float eta = texpf(reg_exp(P.theta + (1.0f - 2.0f * rr) / cov));
        const float x = 1.0f / ((1.0f + eta) + SHR_TOL);
        float der = ((2.0f * eta) * (x * x)) / cov;
        if (der != der) der = 0.0f;
        else if (der == INFINITY) der = 3.402823466e38f;
        else if (der == -INFINITY) der = -3.402823466e38f;
        out[e] = x;
        acc += (double)der;
    }
    acc = group_sum(acc, AMP_WAVE);
    if ((threadIdx.x & (AMP_WAVE - 1)) == 0) s_part[threadIdx.x / AMP_WAVE] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < AMP_WG / AMP_WAVE; ++w) t += s_part[w];
        parts[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(AMP_WG) void shrink_mean_kernel(const double* parts, int nparts, long long count,
                                                             float* mean) {
    __shared__ double s_part[AMP_WG / AMP_WAVE];
    double acc = 0.0;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += parts[i];
    acc = group_sum(acc, AMP_WAVE);
    if ((threadIdx.x & (AMP_WAVE - 1)) == 0) s_part[threadIdx.x / AMP_WAVE] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < AMP_WG / AMP_WAVE; ++w) t += s_part[w];
        mean[0] = (float)(t / (double)count);
    }
}

// sw_shrinkOOK (shrink.py:68-76), one element: Lr (already regularised in place, as the
// reference's regularize_exp mutates Lr), e = exp(Lr), S = the section's sum of e.
__device__ __forceinline__ void sw_finish(float lr, float el, float S, float& x, float& var) {
    const float le = -logf(S - el);
    const float eta = texpf(reg_exp(lr + le));
    x = eta / (1.0f + eta);
    var = x * (1.0f - x);
}
__device__ __forceinline__ float sw_logit(const ShrinkK& P, long long e) {
    float rr, ri;
    load_r(P, e, rr, ri);
    return reg_exp((2.0f * rr - 1.0f) / load_cov(P, e));
}

// M a power of two <= 64: one lane per element, the section is an aligned group of M lanes.
__global__ __launch_bounds__(AMP_WG) void shrink_sw_group_kernel(ShrinkK P, float2* xo, float* vo) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long total = (P.count + AMP_WG - 1) / AMP_WG * AMP_WG;   // whole waves stay in the loop
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += stride) {
        const bool in = e < P.count;
        const float lr = in ? sw_logit(P, e) : 0.0f;
        const float el = in ? texpf(lr) : 0.0f;
        const float S = group_sum(el, P.M);
        if (in) {
            float x, var;
            sw_finish(lr, el, S, x, var);
            xo[e] = make_float2(x, 0.0f);
            vo[e] = var;
        }
    }
}

// any M: one wavefront per section, two passes over it (sum, then outputs).
__global__ __launch_bounds__(AMP_WG) void shrink_sw_wave_kernel(ShrinkK P, float2* xo, float* vo) {
    const long long S = P.count / P.M;
    const int lane = threadIdx.x & (AMP_WAVE - 1);
    const long long waves = (long long)gridDim.x * (AMP_WG / AMP_WAVE);
    for (long long s = blockIdx.x * (long long)(AMP_WG / AMP_WAVE) + threadIdx.x / AMP_WAVE; s < S; s += waves) {
        const long long o = s * P.M;
        float acc = 0.0f;
        for (int m = lane; m < P.M; m += AMP_WAVE) acc += texpf(sw_logit(P, o + m));
        acc = group_sum(acc, AMP_WAVE);
        for (int m = lane; m < P.M; m += AMP_WAVE) {
            const float lr = sw_logit(P, o + m);
            float x, var;
            sw_finish(lr, texpf(lr), acc, x, var);
            xo[o + m] = make_float2(x, 0.0f);
            vo[o + m] = var;
        }
    }
}

static int shrink_grid(long long count) {
    return (int)std::max(1LL, std::min((count + AMP_WG - 1) / AMP_WG, 8192LL));
}

static int fill_args(ShrinkK& P, long long count, int cplx, const void* r, float cov_scalar, const void* cov_vec) {
    AMP_REQUIRE(count >= 0, "shrink: count %lld < 0", count);
    AMP_REQUIRE(r || count == 0, "shrink: null r");
    P = ShrinkK{};
    P.count = count;
    P.cplx = cplx ? 1 : 0;
    P.cov_vec = cov_vec ? 1 : 0;
    P.cov_scalar = cov_scalar;
    P.r = (const float*)r;
    P.cov = (const float*)cov_vec;
    return AMP_OK;
}

}  // namespace amp

using namespace amp;

extern "C" {

int amp_shrink_bayes(const amp_constellation* c, int64_t count, int32_t is_complex, const void* r, float cov_scalar,
                     const void* cov_vec, float P0, float Ps, void* out, void* stream) {
    ShrinkK P;
    int rc = fill_args(P, count, is_complex, r, cov_scalar, cov_vec);
    if (rc) return rc;
    AMP_REQUIRE(c && c->K >= 1 && c->K <= AMP_MAX_K && is_pow2(c->K) && c->K != 32,
                "amp_shrink_bayes: constellation size K = %d must be 1, 2, 4, 8, 16 or 64", c ? c->K : 0);
    AMP_REQUIRE(out || count == 0, "amp_shrink_bayes: null out");
    if (!is_complex)
        for (int k = 0; k < c->K; ++k)
            AMP_REQUIRE(c->im[k] == 0.0f, "amp_shrink_bayes: real r needs a real constellation");
    P.p0 = P0;
    P.ps = Ps;
    P.K = c->K;
    for (int k = 0; k < AMP_MAX_K; ++k) {
        P.sre[k] = k < c->K ? c->re[k] : 0.f;
        P.sim[k] = k < c->K ? c->im[k] : 0.f;
    }
    if (count == 0) return AMP_OK;
    hipStream_t st = (hipStream_t)stream;
    const dim3 g(shrink_grid(count)), b(AMP_WG);
    float* o = (float*)out;
    switch (c->K) {
    case 1: hipLaunchKernelGGL(shrink_bayes_kernel<1>, g, b, 0, st, P, o); break;
    case 2: hipLaunchKernelGGL(shrink_bayes_kernel<2>, g, b, 0, st, P, o); break;
    case 4: hipLaunchKernelGGL(shrink_bayes_kernel<4>, g, b, 0, st, P, o); break;
    case 8: hipLaunchKernelGGL(shrink_bayes_kernel<8>, g, b, 0, st, P, o); break;
    case 16: hipLaunchKernelGGL(shrink_bayes_kernel<16>, g, b, 0, st, P, o); break;
    default: hipLaunchKernelGGL(shrink_bayes_kernel<64>, g, b, 0, st, P, o); break;
    }
    AMP_LAUNCH_CHECK("shrink_bayes");
    return AMP_OK;
}

size_t amp_shrink_ook_workspace_bytes(int64_t count) {
    return sizeof(double) * (size_t)shrink_grid(std::max<int64_t>(count, 1));
}

int amp_shrink_ook(int64_t count, int32_t is_complex, const void* r, float cov_scalar, const void* cov_vec,
                   float theta, void* exp_out, void* dxdr_out, void* ws, size_t ws_bytes, void* stream) {
    ShrinkK P;
    int rc = fill_args(P, count, is_complex, r, cov_scalar, cov_vec);
    if (rc) return rc;
    AMP_REQUIRE(count > 0, "amp_shrink_ook: empty input (the reference's mean of nothing is NaN)");
    AMP_REQUIRE(exp_out && dxdr_out && ws, "amp_shrink_ook: null pointer argument");
    AMP_REQUIRE(ws_bytes >= amp_shrink_ook_workspace_bytes(count), "amp_shrink_ook: workspace too small");
    P.theta = theta;
    hipStream_t st = (hipStream_t)stream;
    const int g = shrink_grid(count);
    hipLaunchKernelGGL(shrink_ook_kernel, dim3(g), dim3(AMP_WG), 0, st, P, (float*)exp_out, (double*)ws);
    AMP_LAUNCH_CHECK("shrink_ook");
    hipLaunchKernelGGL(shrink_mean_kernel, dim3(1), dim3(AMP_WG), 0, st, (const double*)ws, g, (long long)count,
                       (float*)dxdr_out);
    AMP_LAUNCH_CHECK("shrink_mean");
    return AMP_OK;
}

int amp_shrink_sw_ook(int64_t sections, int32_t M, int32_t is_complex, const void* r, float cov_scalar,
                      const void* cov_vec, void* exp_out, void* var_out, void* stream) {
    AMP_REQUIRE(M >= 1 && sections >= 0, "amp_shrink_sw_ook: sections %lld, M %d", (long long)sections, M);
    ShrinkK P;
    int rc = fill_args(P, sections * (int64_t)M, is_complex, r, cov_scalar, cov_vec);
    if (rc) return rc;
    AMP_REQUIRE((exp_out && var_out) || sections == 0, "amp_shrink_sw_ook: null output");
    P.M = M;
    if (sections == 0) return AMP_OK;
    hipStream_t st = (hipStream_t)stream;
    if (M <= AMP_WAVE && is_pow2(M)) {
        hipLaunchKernelGGL(shrink_sw_group_kernel, dim3(shrink_grid(P.count)), dim3(AMP_WG), 0, st, P,
                           (float2*)exp_out, (float*)var_out);
    } else {
        const long long wgs = (sections + AMP_WG / AMP_WAVE - 1) / (AMP_WG / AMP_WAVE);
        hipLaunchKernelGGL(shrink_sw_wave_kernel, dim3((int)std::min(wgs, 8192LL)), dim3(AMP_WG), 0, st, P,
                           (float2*)exp_out, (float*)var_out);
    }
    AMP_LAUNCH_CHECK("shrink_sw_ook");
    return AMP_OK;
}

}  // extern "C"
