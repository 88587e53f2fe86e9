// amp_denoise_api.hip — the block-sparse denoiser as a standalone op
// (VAMPLayer.segmented_denoiser vamp.py:96-119, BAMPLayer.segmented_denoiser bamp.py:66-77,
//  SCAMPLayer.denoiser scamp.py:61-68).
// Three launches: sections -> (xmmse, var, section max / max|xi|, block partials); one
// workgroup reduces the partials and, when some section is near the edge of the float64
// range, settles the exact float64 batch max|xi|; sections whose reference float64 softmax
// leaves the normal range are then recomputed with the reference's exact arithmetic (and a
// NaN / inf anywhere makes every section NaN, as torch's max|xi| propagates it).
#include <algorithm>

#include "amp_denoise.h"
#include "amp_host.h"

namespace amp {

struct DnK {
    int N, L, M, S, mode;   // mode 3 (internal): tau = tau[0], a device scalar (vamp2's gamma)
    float tau_scalar_inv;
    const int* skip;        // non-null and set: every launch is a no-op (a stopped loop)
    const float2* r;
    const float* tau;
    float2* xm;
    float* var;
    float* secmax;
    float* secabs;
    Partial* parts;
    int nblk;
    double* G;          // [0] exact batch max|xi|, [1] action: 0 none, 1 fix-up, 2 all NaN, [2] slack
    Const c;
};

constexpr int DRWG = 1024;

struct DnPolicy {
    const DnK* P;
    int sec0;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const size_t o = (size_t)(sec0 + sec) * P->M + m;
        const float2 v = P->r[o];
        rr = v.x; ri = v.y;
        it = (P->mode == 0) ? P->tau_scalar_inv : (P->mode == 3) ? 1.0f / P->tau[0] : 1.0f / (P->tau[o] * 0.5f);
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const {
        const size_t o = (size_t)(sec0 + sec) * P->M + m;
        P->xm[o] = make_float2(xr, xi);
        if (P->var) P->var[o] = var;
        pa.sumvar += (double)var;
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        P->secmax[sec0 + sec] = smax;
        P->secabs[sec0 + sec] = sabs;
    }
};

template <int KK>
__global__ __launch_bounds__(AMP_WG) void denoise_kernel(DnK P) {
    if (P.skip && *P.skip) return;
    __shared__ __attribute__((aligned(16))) float lds[64];
    const int G = P.M < 64 ? P.M : 64;
    const int per = (AMP_WG / 64) * (64 / G);       // sections per workgroup pass
    PartAcc pa;
    for (int sec0 = blockIdx.x * per; sec0 < P.S; sec0 += gridDim.x * per) {
        DnPolicy pol{&P, sec0};
        const int n = min(per, P.S - sec0);
        if (P.mode == 2)
            denoise_sections<false, KK>(pol, n, P.M, P.c, pa);
        else
            denoise_sections<true, KK>(pol, n, P.M, P.c, pa);
    }
    part_block_store(pa, P.parts + blockIdx.x, lds);
}

struct DnLoad {
    const DnK* P;
    size_t o0;
    __device__ __forceinline__ void operator()(int m, float& rr, float& ri, float& it) const {
        const float2 v = P->r[o0 + m];
        rr = v.x; ri = v.y;
        it = (P->mode == 0) ? P->tau_scalar_inv : (P->mode == 3) ? 1.0f / P->tau[0] : 1.0f / (P->tau[o0 + m] * 0.5f);
    }
};

__global__ __launch_bounds__(DRWG) void denoise_reduce_kernel(DnK P, Const64 c64) {
    if (P.skip && *P.skip) return;
    __shared__ __attribute__((aligned(16))) float lds[512];
    __shared__ double s_d[DRWG / 64];
    const PartAcc pa = part_reduce_all(P.parts, P.nblk, lds);
    double act = 0.0, G = pa.maxabs;
    if (part_allnan(pa)) {
        act = 2.0;
    } else if (part_danger(pa)) {
        // exact float64 max|xi| over the candidate sections
        const double slack = logit_slack(pa.maxabs);
        double gm = 0.0;
        for (int s = threadIdx.x; s < P.S; s += blockDim.x)
            if ((double)P.secabs[s] >= pa.maxabs - slack)
                gm = fmax(gm, section_absmax_f64(DnLoad{&P, (size_t)s * P.M}, P.M, c64));
        gm = group_max(gm, 64);
        if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = gm;
        __syncthreads();
        G = 0.0;
        for (int w = 0; w < DRWG / 64; ++w) G = fmax(G, s_d[w]);
        act = 1.0;
    }
    if (threadIdx.x == 0) {
        P.G[0] = G;
        P.G[1] = act;
        P.G[2] = logit_slack(pa.maxabs);
    }
}

__global__ void denoise_fix_kernel(DnK P, Const64 c64) {
    if (P.skip && *P.skip) return;
    const double G = P.G[0], act = P.G[1], slack = P.G[2];
    if (act == 0.0) return;
    if (act == 2.0) {
        const float q = __int_as_float(0x7fc00000);
        for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < (size_t)P.S * P.M;
             e += (size_t)gridDim.x * blockDim.x) {
            P.xm[e] = make_float2(q, q);
            if (P.var) P.var[e] = q;
        }
        return;
    }
    for (int sec = blockIdx.x * blockDim.x + threadIdx.x; sec < P.S; sec += gridDim.x * blockDim.x) {
        if (!((double)P.secmax[sec] - G < AMP_DANGER + slack)) continue;
        const size_t o0 = (size_t)sec * P.M;
        auto st = [&](int m, float xr, float xi, float var) {
            P.xm[o0 + m] = make_float2(xr, xi);
            if (P.var) P.var[o0 + m] = var;
        };
        if (P.mode == 2)
            exact_section_f64<false>(DnLoad{&P, o0}, st, P.M, c64, G);
        else
            exact_section_f64<true>(DnLoad{&P, o0}, st, P.M, c64, G);
    }
}

static int dn_nblk(const amp_dims* d) {
    const int G = d->M < 64 ? d->M : 64;
    const int per = (AMP_WG / 64) * (64 / G);
    return std::max(1, std::min(cdiv(d->B * d->L, per), 2048));
}

static int denoise_launch(const amp_dims* d, const amp_constellation* c, const float2* r, int mode, float tau_inv,
                          const float* tau, float2* xmmse, float* var, void* ws, const int* skip, hipStream_t st) {
    DnK P;
    P.N = d->N; P.L = d->L; P.M = d->M; P.S = d->B * d->L; P.mode = mode;
    P.tau_scalar_inv = tau_inv;
    P.skip = skip;
    P.r = r; P.tau = tau; P.xm = xmmse;
    P.var = var;
    Carve cv(ws);
    P.secmax = cv.take<float>((size_t)P.S);
    P.secabs = cv.take<float>((size_t)P.S);
    P.nblk = dn_nblk(d);
    P.parts = cv.take<Partial>((size_t)P.nblk);
    P.G = cv.take<double>(4);
    P.c = to_const(c);
    const Const64 c64 = to_const64(c);
    switch (P.c.K) {
    case 1: hipLaunchKernelGGL(denoise_kernel<1>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    case 2: hipLaunchKernelGGL(denoise_kernel<2>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    case 4: hipLaunchKernelGGL(denoise_kernel<4>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    case 8: hipLaunchKernelGGL(denoise_kernel<8>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    case 16: hipLaunchKernelGGL(denoise_kernel<16>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    default: hipLaunchKernelGGL(denoise_kernel<64>, dim3(P.nblk), dim3(AMP_WG), 0, st, P); break;
    }
    AMP_LAUNCH_CHECK("denoise");
    hipLaunchKernelGGL(denoise_reduce_kernel, dim3(1), dim3(DRWG), 0, st, P, c64);
    AMP_LAUNCH_CHECK("denoise_reduce");
    const int g = std::max(1, std::min(cdiv(P.S, 256), 1024));
    hipLaunchKernelGGL(denoise_fix_kernel, dim3(g), dim3(256), 0, st, P, c64);
    AMP_LAUNCH_CHECK("denoise_fix");
    return AMP_OK;
}

size_t block_denoise_ws_bytes(const amp_dims* d) {
    Carve cv(nullptr);
    cv.take<float>((size_t)d->B * d->L);
    cv.take<float>((size_t)d->B * d->L);
    cv.take<Partial>((size_t)dn_nblk(d));
    cv.take<double>(4);
    return cv.off;
}

// The denoiser at tau = *tau_dev (a device scalar; vamp2's gamma), skipped while *skip != 0.
int block_denoise_dev(const amp_dims* d, const amp_constellation* c, const float2* r, const float* tau_dev,
                      float2* xm, float* var, void* ws, const int* skip, hipStream_t st) {
    return denoise_launch(d, c, r, 3, 0.0f, tau_dev, xm, var, ws, skip, st);
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_block_denoise_workspace_bytes(const amp_dims* d) { return d ? block_denoise_ws_bytes(d) : 0; }

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
    return denoise_launch(d, c, (const float2*)r, tau_mode, 1.0f / tau_scalar, (const float*)tau_vec, (float2*)xmmse,
                          (tau_mode == 2) ? nullptr : (float*)var, ws, nullptr, (hipStream_t)stream);
}

}  // extern "C"
