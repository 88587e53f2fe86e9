// amp_vamp2.hip — the damped "Rangan" VAMP of vamp2.py (vamp2.py:12-131) on the GPU.
//
// Per iteration (a stopped loop turns every later launch into a no-op; no host sync):
//   1. (xmmse, var) = block denoiser of r at tau = gamma (vamp2.py:62, 79-88; the device-scalar
//      tau mode of amp_denoise_api.hip, with the reference's float64 batch-max rules);
//   2. v2_stats:   per-block float64 sum of var and the allclose count against the previous var;
//   3. v2_scalars: one workgroup folds them (fixed order) into alpha, gamma~, d = s^2 / (s^2 +
//      sigma2 gamma~), d.mean(), the damped gamma and d / d.mean() (vamp2.py:64-75);
//   4. v2_rt:      xmmse <- rho xmmse + (1 - rho) xmmse_prev; r~ = (xmmse - alpha r) / (1 - alpha)
//      (vamp2.py:63, 66);
//   5. GEMM q = Vh r~ (the launch engine's f32 MFMA GEMM, amp_weights.hip);
//   6. v2_z:       z = (d / d.mean()) (y~ - q) (vamp2.py:77);
//   7. GEMM (eta V) z;  v2_r: r = r~ + (eta V) z, the early exit of vamp2.py:129 takes effect.
// Tracker (vamp2.py:12-26): y~ = (Uh y) / s (GEMM + one element-wise pass), r = 0, var = 1,
// xmmse = 0, gamma = 1.  Scalars are float32 0-dim values in the reference's op order; the
// Python floats (sigma2, eta, rho) enter as float32 where torch casts them.
#include <algorithm>

#include "amp_gemm.h"
#include "amp_host.h"

namespace amp {

int block_denoise_dev(const amp_dims* d, const amp_constellation* c, const float2* r, const float* tau_dev,
                      float2* xm, float* var, void* ws, const int* skip, hipStream_t st);
size_t block_denoise_ws_bytes(const amp_dims* d);

struct V2Scal {
    float gamma;        // T.gamma (vamp2.py:21, 73)
    float alpha;        // vamp2.py:64
    float inv1ma;       // 1 / (1 - alpha) (c64 / f32 = multiply by the reciprocal)
    float gamma_tilde;  // vamp2.py:67-69
    float dm;           // d.mean()
    int stopped;        // the loop has stopped: later launches are no-ops
    int stop_pending;   // allclose held this iteration (vamp2.py:129): stop after the r update
    int T;              // executed iterations
    int last;           // index of the var buffer holding the last iteration's var
    int nan;            // the last denoiser call produced non-finite values
    int pad[2];
};

struct V2Part {
    double sumvar;
    unsigned notclose;
    unsigned nonfinite;
};

constexpr int V2_BLK = 256;
constexpr int V2_NBLK = 1024;

struct V2K {
    int B, N, k, max_iter;
    float sigma2f, etaf, rho, omr;
    const float* s;
    float *ytil, *r, *xm, *xmd, *var0, *var1, *rt, *z, *q, *radd, *dd, *etarow;
    V2Scal* sc;
    V2Part* parts;
    amp_status* status;
};

__global__ void v2_init(V2K P) {
    const size_t BN = (size_t)P.B * P.N;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN; e += (size_t)gridDim.x * blockDim.x) {
        P.r[2 * e] = 0.f; P.r[2 * e + 1] = 0.f;            // vamp2.py:23
        P.xm[2 * e] = 0.f; P.xm[2 * e + 1] = 0.f;          // vamp2.py:25
        P.var0[e] = 1.f;                                   // vamp2.py:24
    }
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < (size_t)P.N; e += (size_t)gridDim.x * blockDim.x)
        P.etarow[e] = P.etaf;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        V2Scal s{};
        s.gamma = 1.0f;
        s.last = 0;
        *P.sc = s;
    }
}

// y~ = (Uh y) / s (vamp2.py:22), in place on the GEMM output [B][2k]
__global__ void v2_ytil(V2K P) {
    const size_t Bk = (size_t)P.B * P.k;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < Bk; e += (size_t)gridDim.x * blockDim.x) {
        const int j = (int)(e % P.k);
        const float inv = 1.0f / P.s[j];
        P.ytil[2 * e] *= inv;
        P.ytil[2 * e + 1] *= inv;
    }
}

__device__ __forceinline__ bool torch_close_f(float a, float b) {   // torch.allclose element rule
    if (a == b) return true;
    const float d = fabsf(a - b);
    return __builtin_isfinite(d) && d <= 1.0e-8f + fabsf(1.0e-5f * b);
}

__global__ __launch_bounds__(V2_BLK) void v2_stats(V2K P, int t) {
    if (P.sc->stopped) return;
    const float* vn = (t & 1) ? P.var0 : P.var1;   // this iteration's var (t even -> var1)
    const float* vp = (t & 1) ? P.var1 : P.var0;
    const size_t BN = (size_t)P.B * P.N;
    double s = 0.0;
    unsigned nc = 0, nf = 0;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN; e += (size_t)gridDim.x * blockDim.x) {
        const float v = vn[e];
        s += (double)v;
        nc += torch_close_f(v, vp[e]) ? 0u : 1u;
        nf += __builtin_isfinite(v) ? 0u : 1u;
    }
    s = group_sum(s, 64);
    nc = group_sum(nc, 64);
    nf = group_sum(nf, 64);
    __shared__ V2Part sw[V2_BLK / 64];
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = V2Part{s, nc, nf};
    __syncthreads();
    if (threadIdx.x == 0) {
        V2Part o = sw[0];
        for (int w = 1; w < V2_BLK / 64; ++w) { o.sumvar += sw[w].sumvar; o.notclose += sw[w].notclose; o.nonfinite += sw[w].nonfinite; }
        P.parts[blockIdx.x] = o;
    }
}

__device__ __forceinline__ float clampf_v2(float v, float lo, float hi) {   // torch.max then torch.min (NaN kept)
    v = (v != v) ? v : (v < lo ? lo : v);
    return (v != v) ? v : (v > hi ? hi : v);
}

__global__ __launch_bounds__(256) void v2_scalars(V2K P, int nblk, int t) {
    if (P.sc->stopped) return;
    __shared__ double s_d[4];
    __shared__ unsigned s_u[4][2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // fixed-order fold of the block partials
    double sv = 0.0;
    unsigned nc = 0, nf = 0;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) { sv += P.parts[b].sumvar; nc += P.parts[b].notclose; nf += P.parts[b].nonfinite; }
    sv = group_sum(sv, 64); nc = group_sum(nc, 64); nf = group_sum(nf, 64);
    if (lane == 0) { s_d[wave] = sv; s_u[wave][0] = nc; s_u[wave][1] = nf; }
    __syncthreads();
    sv = s_d[0] + s_d[1] + s_d[2] + s_d[3];
    nc = s_u[0][0] + s_u[1][0] + s_u[2][0] + s_u[3][0];
    nf = s_u[0][1] + s_u[1][1] + s_u[2][1] + s_u[3][1];
    V2Scal S = *P.sc;
    const float gamma = S.gamma;
    const float mean = (float)(sv / ((double)P.B * (double)P.N));                  // T.var.mean()
    const float alpha = mean * gamma;                                                // vamp2.py:64
    float gt = (gamma * (1.0f - alpha)) / alpha;                                     // vamp2.py:67
    gt = clampf_v2(gt, 1.0e-11f, 1.0e11f);                                           // vamp2.py:68-69
    const float sg = P.sigma2f * gt;
    // d = s^2 / (s^2 + sigma2 gamma~) (vamp2.py:71) and its mean, float64 sum of the f32 values
    double ds = 0.0;
    for (int i = lane; i < P.k; i += 64) {
        const float s2 = P.s[i] * P.s[i];
        ds += (double)(s2 / (s2 + sg));
    }
    ds = group_sum(ds, 64);                        // every wave: the same order, the same value
    const float dm = (float)(ds / (double)P.k);
    const float g = (gt * dm) / (P.etaf - dm);                                       // vamp2.py:72
    const float gnew = P.rho * g + P.omr * gamma;                                    // vamp2.py:73
    for (int i = threadIdx.x; i < P.k; i += blockDim.x) {
        const float s2 = P.s[i] * P.s[i];
        P.dd[i] = (s2 / (s2 + sg)) / dm;                                             // d / d.mean()
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        S.alpha = alpha;
        S.inv1ma = 1.0f / (1.0f - alpha);
        S.gamma_tilde = gt;
        S.dm = dm;
        S.gamma = gnew;
        S.stop_pending = (nc == 0) ? 1 : 0;                                          // vamp2.py:129
        S.nan = nf ? 1 : 0;
        S.last = (t & 1) ? 0 : 1;
        S.T = t + 1;
        *P.sc = S;
    }
}

// xmmse <- rho xmmse + (1 - rho) xmmse_prev (vamp2.py:63); r~ = (xmmse - alpha r) / (1 - alpha) (:66)
__global__ void v2_rt(V2K P) {
    if (P.sc->stopped) return;
    const float alpha = P.sc->alpha, inv = P.sc->inv1ma;
    const size_t n2 = (size_t)P.B * P.N * 2;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n2; e += (size_t)gridDim.x * blockDim.x) {
        const float x = P.rho * P.xmd[e] + P.omr * P.xm[e];
        P.xm[e] = x;
        P.rt[e] = (x - alpha * P.r[e]) * inv;
    }
}

// z = (d / d.mean()) (y~ - q)   (vamp2.py:77)
__global__ void v2_z(V2K P) {
    if (P.sc->stopped) return;
    const size_t Bk = (size_t)P.B * P.k;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < Bk; e += (size_t)gridDim.x * blockDim.x) {
        const float w = P.dd[e % P.k];
        P.z[2 * e] = w * (P.ytil[2 * e] - P.q[2 * e]);
        P.z[2 * e + 1] = w * (P.ytil[2 * e + 1] - P.q[2 * e + 1]);
    }
}

// r = r~ + (eta V) z (vamp2.py:77); the allclose break (vamp2.py:129) takes effect after it
__global__ void v2_r(V2K P) {
    if (P.sc->stopped) return;
    const size_t n2 = (size_t)P.B * P.N * 2;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n2; e += (size_t)gridDim.x * blockDim.x)
        P.r[e] = P.rt[e] + P.radd[e];
}

__global__ void v2_step_end(V2K P) {
    if (P.sc->stopped) return;
    if (P.sc->stop_pending) P.sc->stopped = 1;
}

__global__ void v2_finish(V2K P) {
    const int last = P.sc->last;
    if (last == 1) {
        const size_t BN = (size_t)P.B * P.N;
        for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN; e += (size_t)gridDim.x * blockDim.x)
            P.var0[e] = P.var1[e];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const V2Scal S = *P.sc;
        amp_status st;
        st.T = S.T;
        st.nan_state = S.nan;
        st.stopped = S.stopped;
        st.gemm = AMP_ARITH_F32;
        st.last_scalar[0] = S.gamma; st.last_scalar[1] = S.alpha; st.last_scalar[2] = S.gamma_tilde;
        st.last_scalar[3] = S.dm;
        *P.status = st;
    }
}

struct V2Ws {
    float *Wuh, *Wvh, *Wv, *ytil, *xmd, *var1, *rt, *z, *q, *radd, *dd, *etarow;
    V2Scal* sc;
    V2Part* parts;
    void* dn;
    size_t bytes;
    int kap0, ncp0, kap1, ncp1, kap2, ncp2;
};

static V2Ws v2_carve(const amp_dims* d, int k, void* base) {
    V2Ws w;
    w.kap0 = round_up(2 * d->n, GBK); w.ncp0 = round_up(2 * k, 128);      // Uh:  o < k, j < n
    w.kap1 = round_up(2 * d->N, GBK); w.ncp1 = round_up(2 * k, 128);      // Vh:  o < k, j < N
    w.kap2 = round_up(2 * k, GBK); w.ncp2 = round_up(2 * d->N, 128);      // eta V: o < N, j < k
    Carve cv(base);
    w.Wuh = cv.take<float>((size_t)w.ncp0 * w.kap0);
    w.Wvh = cv.take<float>((size_t)w.ncp1 * w.kap1);
    w.Wv = cv.take<float>((size_t)w.ncp2 * w.kap2);
    const size_t BN2 = (size_t)d->B * d->N * 2, Bk2 = (size_t)d->B * k * 2;
    w.ytil = cv.take<float>(Bk2);
    w.xmd = cv.take<float>(BN2);
    w.var1 = cv.take<float>((size_t)d->B * d->N);
    w.rt = cv.take<float>(BN2);
    w.z = cv.take<float>(Bk2);
    w.q = cv.take<float>(Bk2);
    w.radd = cv.take<float>(BN2);
    w.dd = cv.take<float>((size_t)k);
    w.etarow = cv.take<float>((size_t)d->N);
    w.sc = cv.take<V2Scal>(1);
    w.parts = cv.take<V2Part>(V2_NBLK);
    const size_t dnb = block_denoise_ws_bytes(d);
    w.dn = cv.take<unsigned char>(dnb);
    w.bytes = cv.off;
    return w;
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_vamp2_workspace_bytes(const amp_dims* d, int32_t k) {
    if (!d || k <= 0) return 0;
    return v2_carve(d, k, nullptr).bytes;
}

int amp_vamp2_run(const amp_dims* d, const amp_constellation* c, const amp_vamp2_args* a, void* stream) {
    int rc = check_dims(d, c);
    if (rc) return rc;
    AMP_REQUIRE(a && a->U && a->s && a->Vh && a->y && a->r && a->xmmse && a->var && a->status && a->ws,
                "amp_vamp2_run: null pointer argument");
    AMP_REQUIRE(a->k > 0 && a->k <= d->N && a->k <= d->n, "amp_vamp2_run: k = %d must be min(n, N)", a->k);
    AMP_REQUIRE(a->max_iter > 0, "amp_vamp2_run: max_iter must be positive");
    const int k = a->k;
    const V2Ws w = v2_carve(d, k, a->ws);
    AMP_REQUIRE(a->ws_bytes >= w.bytes, "amp_vamp2_run: workspace %zu < %zu bytes", a->ws_bytes, w.bytes);
    hipStream_t st = (hipStream_t)stream;
    V2K P;
    P.B = d->B; P.N = d->N; P.k = k; P.max_iter = a->max_iter;
    P.sigma2f = (float)a->sigma2;                       // Python float * f32 tensor (vamp2.py:71)
    const double eta = (double)d->N / (double)k;        // vamp2.py:26
    P.etaf = (float)eta;
    P.rho = (float)a->damping;                          // vamp2.py:63, 73
    P.omr = (float)(1.0 - a->damping);
    P.s = (const float*)a->s;
    P.ytil = w.ytil; P.r = (float*)a->r; P.xm = (float*)a->xmmse; P.xmd = w.xmd;
    P.var0 = (float*)a->var; P.var1 = w.var1; P.rt = w.rt; P.z = w.z; P.q = w.q; P.radd = w.radd; P.dd = w.dd;
    P.etarow = w.etarow; P.sc = w.sc; P.parts = w.parts; P.status = (amp_status*)a->status;
    const size_t BN = (size_t)d->B * d->N;
    const int gEl = (int)std::min<size_t>((BN + 255) / 256, 2048);
    const int gk = (int)std::min<size_t>(((size_t)d->B * k + 255) / 256, 2048);
    hipLaunchKernelGGL(v2_init, dim3(gEl), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("v2_init");
    // Uh:    X[o][j] = conj(U[j][o]),          o < k, j < n   (vamp2.py:15, 22)
    rc = build_cweight((const float2*)a->U, 1, k, 1, nullptr, k, d->n, w.Wuh, w.kap0, w.ncp0, st);
    // Vh:    X[o][j] = Vh[o][j],               o < k, j < N   (vamp2.py:77)
    if (!rc) rc = build_cweight((const float2*)a->Vh, d->N, 1, 0, nullptr, k, d->N, w.Wvh, w.kap1, w.ncp1, st);
    // eta V: X[o][j] = eta conj(Vh[j][o]),     o < N, j < k   ((T.eta * T.V) @ ..., vamp2.py:77)
    if (!rc) rc = build_cweight((const float2*)a->Vh, 1, d->N, 1, w.etarow, d->N, k, w.Wv, w.kap2, w.ncp2, st);
    if (!rc) rc = gemm_store((const float*)a->y, 2 * d->n, d->B, 2 * d->n, w.Wuh, w.kap0, w.ncp0, w.ytil, 2 * k, 2 * k, st);
    if (rc) return rc;
    hipLaunchKernelGGL(v2_ytil, dim3(gk), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("v2_ytil");
    const int nblk = (int)std::min<size_t>((BN + V2_BLK - 1) / V2_BLK, V2_NBLK);
    for (int t = 0; t < a->max_iter; ++t) {
        float* vnew = (t & 1) ? P.var0 : P.var1;
        rc = block_denoise_dev(d, c, (const float2*)P.r, &w.sc->gamma, (float2*)P.xmd, vnew, w.dn, &w.sc->stopped, st);
        if (rc) return rc;
        hipLaunchKernelGGL(v2_stats, dim3(nblk), dim3(V2_BLK), 0, st, P, t);
        AMP_LAUNCH_CHECK("v2_stats");
        hipLaunchKernelGGL(v2_scalars, dim3(1), dim3(256), 0, st, P, nblk, t);
        AMP_LAUNCH_CHECK("v2_scalars");
        hipLaunchKernelGGL(v2_rt, dim3(gEl), dim3(256), 0, st, P);
        AMP_LAUNCH_CHECK("v2_rt");
        rc = gemm_store(P.rt, 2 * d->N, d->B, 2 * d->N, w.Wvh, w.kap1, w.ncp1, P.q, 2 * k, 2 * k, st);   // runs after a stop too: its output is then unused
        if (rc) return rc;
        hipLaunchKernelGGL(v2_z, dim3(gk), dim3(256), 0, st, P);
        AMP_LAUNCH_CHECK("v2_z");
        rc = gemm_store(P.z, 2 * k, d->B, 2 * k, w.Wv, w.kap2, w.ncp2, P.radd, 2 * d->N, 2 * d->N, st);
        if (rc) return rc;
        hipLaunchKernelGGL(v2_r, dim3(gEl), dim3(256), 0, st, P);
        AMP_LAUNCH_CHECK("v2_r");
        hipLaunchKernelGGL(v2_step_end, dim3(1), dim3(64), 0, st, P);
        AMP_LAUNCH_CHECK("v2_step_end");
    }
    hipLaunchKernelGGL(v2_finish, dim3(gEl), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("v2_finish");
    return AMP_OK;
}

}  // extern "C"
