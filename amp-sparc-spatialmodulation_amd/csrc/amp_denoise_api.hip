// amp_denoise_api.hip — the block-sparse denoiser as a standalone op
// (VAMPLayer.segmented_denoiser vamp.py:96-119, BAMPLayer.segmented_denoiser bamp.py:66-77,
//  SCAMPLayer.denoiser scamp.py:61-68).
// Three launches: sections -> (xmmse, var, section max, block partials); one workgroup
// reduces the partials to the batch max|xi|; sections whose reference float64 softmax
// leaves the normal range are recomputed with the reference's exact arithmetic.
#include <algorithm>

#include "amp_denoise.h"
#include "amp_host.h"

namespace amp {

struct DnK {
    int N, L, M, S, mode;
    float tau_scalar_inv;
    const float2* r;
    const float* tau;
    float2* xm;
    float* var;
    double* secmax;
    Partial* parts;
    int nblk;
    double* G;
    Const c;
};

struct DnPolicy {
    const DnK* P;
    int sec0;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const size_t o = (size_t)(sec0 + sec) * P->M + m;
        const float2 v = P->r[o];
        rr = v.x; ri = v.y;
        it = (P->mode == 0) ? P->tau_scalar_inv : 1.0f / (P->tau[o] * 0.5f);
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const {
        const size_t o = (size_t)(sec0 + sec) * P->M + m;
        P->xm[o] = make_float2(xr, xi);
        if (P->var) P->var[o] = var;
        pa.sumvar += (double)var;
    }
    __device__ __forceinline__ void section(int sec, double smax) const { P->secmax[sec0 + sec] = smax; }
};

__global__ __launch_bounds__(AMP_WG) void denoise_kernel(DnK P) {
    __shared__ __attribute__((aligned(16))) float lds[64];
    const int G = P.M < 64 ? P.M : 64;
    const int per = (AMP_WG / 64) * (64 / G);       // sections per workgroup pass
    PartAcc pa;
    for (int sec0 = blockIdx.x * per; sec0 < P.S; sec0 += gridDim.x * per) {
        DnPolicy pol{&P, sec0};
        const int n = min(per, P.S - sec0);
        if (P.mode == 2)
            denoise_sections<false>(pol, n, P.M, P.c, pa);
        else
            denoise_sections<true>(pol, n, P.M, P.c, pa);
    }
    part_block_store(pa, P.parts + blockIdx.x, lds);
}

__global__ __launch_bounds__(AMP_WG) void denoise_reduce_kernel(DnK P) {
    __shared__ __attribute__((aligned(16))) float lds[64];
    const PartAcc pa = part_reduce_all(P.parts, P.nblk, lds);
    if (threadIdx.x == 0) *P.G = pa.maxabs;
}

__global__ void denoise_fix_kernel(DnK P) {
    const double G = *P.G;
    for (int sec = blockIdx.x * blockDim.x + threadIdx.x; sec < P.S; sec += gridDim.x * blockDim.x) {
        if (!(P.secmax[sec] - G < AMP_DANGER)) continue;
        const size_t o0 = (size_t)sec * P.M;
        auto ld = [&](int m, float& rr, float& ri, float& it) {
            const float2 v = P.r[o0 + m];
            rr = v.x; ri = v.y;
            it = (P.mode == 0) ? P.tau_scalar_inv : 1.0f / (P.tau[o0 + m] * 0.5f);
        };
        auto st = [&](int m, float xr, float xi, float var) {
            P.xm[o0 + m] = make_float2(xr, xi);
            if (P.var) P.var[o0 + m] = var;
        };
        if (P.mode == 2)
            exact_section_f64<false>(ld, st, P.M, P.c, G);
        else
            exact_section_f64<true>(ld, st, P.M, P.c, G);
    }
}

static int dn_nblk(const amp_dims* d) {
    const int G = d->M < 64 ? d->M : 64;
    const int per = (AMP_WG / 64) * (64 / G);
    return std::max(1, std::min(cdiv(d->B * d->L, per), 2048));
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_block_denoise_workspace_bytes(const amp_dims* d) {
    if (!d) return 0;
    Carve cv(nullptr);
    cv.take<double>((size_t)d->B * d->L);
    cv.take<Partial>((size_t)dn_nblk(d));
    cv.take<double>(2);
    return cv.off;
}

int amp_block_denoise(const amp_dims* d, const amp_constellation* c, const void* r, int32_t tau_mode,
                      float tau_scalar, const void* tau_vec, void* xmmse, void* var, void* ws, size_t ws_bytes,
                      void* stream) {
    int rc = check_dims(d, c, false);
    if (rc) return rc;
    AMP_REQUIRE(r && xmmse && ws, "amp_block_denoise: null pointer argument");
    AMP_REQUIRE(tau_mode >= 0 && tau_mode <= 2, "amp_block_denoise: tau_mode %d", tau_mode);
    AMP_REQUIRE(tau_mode == 0 || tau_vec, "amp_block_denoise: tau_vec required for tau_mode %d", tau_mode);
    AMP_REQUIRE(tau_mode == 2 || var, "amp_block_denoise: var output required");
    AMP_REQUIRE(ws_bytes >= amp_block_denoise_workspace_bytes(d), "amp_block_denoise: workspace too small");
    DnK P;
    P.N = d->N; P.L = d->L; P.M = d->M; P.S = d->B * d->L; P.mode = tau_mode;
    P.tau_scalar_inv = 1.0f / tau_scalar;
    P.r = (const float2*)r; P.tau = (const float*)tau_vec; P.xm = (float2*)xmmse;
    P.var = (tau_mode == 2) ? nullptr : (float*)var;
    Carve cv(ws);
    P.secmax = cv.take<double>((size_t)P.S);
    P.nblk = dn_nblk(d);
    P.parts = cv.take<Partial>((size_t)P.nblk);
    P.G = cv.take<double>(2);
    P.c = to_const(c);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(denoise_kernel, dim3(P.nblk), dim3(AMP_WG), 0, st, P);
    AMP_LAUNCH_CHECK("denoise");
    hipLaunchKernelGGL(denoise_reduce_kernel, dim3(1), dim3(AMP_WG), 0, st, P);
    AMP_LAUNCH_CHECK("denoise_reduce");
    const int g = std::max(1, std::min(cdiv(P.S, 256), 1024));
    hipLaunchKernelGGL(denoise_fix_kernel, dim3(g), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("denoise_fix");
    return AMP_OK;
}

}  // extern "C"
