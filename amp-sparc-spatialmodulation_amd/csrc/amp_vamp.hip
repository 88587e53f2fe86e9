// amp_vamp.hip — VAMP (SVD form) detector, device-resident iteration loop.
//
// Restates VAMP.forward (vamp.py:159-187): Tracker (vamp.py:12-28), T x
// VAMPLayer.forward (vamp.py:56-94), the allclose early exit (vamp.py:185).
//
// Per iteration t, three launches on one stream, no host synchronisation:
//   vamp_k1<t>  GEMM1  q = Vh r~ with r~ = (xmmse - dxdr r) ns formed in the A-operand
//               prologue (vamp.py:89-91, 67), LMMSE epilogue w = scale (y~ + vr q) - q
//               (vamp.py:68-72).
//   vamp_k2<t>  GEMM2  V w, epilogue x~ = Vw + r~, r = (x~ - alpha r~)/(1 - alpha)
//               (vamp.py:72-79), then the section denoiser on the LDS tile (vamp.py:84,
//               96-119) -> xmmse, var, per-section max logit, workgroup partials.
//   vamp_r<t>   one workgroup: reduce the partials (sum var, max|xi|, allclose count);
//               recompute in exact float64 the rare sections whose reference softmax
//               leaves the normal range (amp_denoise.h, exact_section_f64); then the batch
//               scalars of iteration t+1 (vamp.py:85-94, 66-82) or the stop record
//               (vamp.py:185-186).  Later iterations of a stopped loop are no-ops.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "amp_persist.h"
#include "amp_vamp.h"

namespace amp {

static float* g_dump = nullptr;
float* debug_dump_ptr() { return g_dump; }

__global__ __launch_bounds__(RWG) void vamp_init_scalars(VampK P) {
    __shared__ __attribute__((aligned(16))) float lds[64];
    const VampIter it = vamp_first_iter(P, lds);
    if (threadIdx.x == 0) P.iters[0] = it;
}

// r~ = (xmmse - dxdr * r) * normScalar (vamp.py:91), formed while loading GEMM1's A tile.
// Staged in two steps like ALoadPlain (amp_gemm.h): both loads at a clamped address, the formula
// and the zeroing of out-of-range elements at the LDS store.
struct ALoadRt {
    const float* __restrict__ xm;
    const float* __restrict__ r;
    int lda, rows, ka;
    float dxdr, ns;
    struct Raw {
        float4 x, q;
    };
    __device__ __forceinline__ Raw raw(int row, int k) const {
        const size_t o = (size_t)min(row, rows - 1) * lda + min(k, ka - 4);
        return Raw{*reinterpret_cast<const float4*>(xm + o), *reinterpret_cast<const float4*>(r + o)};
    }
    __device__ __forceinline__ float4 fin(const Raw& v, int row, int k) const {
        const bool ok = row < rows && k < ka;
        const float4 x = v.x, q = v.q;
        const float4 f = make_float4((x.x - dxdr * q.x) * ns, (x.y - dxdr * q.y) * ns, (x.z - dxdr * q.z) * ns,
                                     (x.w - dxdr * q.w) * ns);
        return ok ? f : make_float4(0.f, 0.f, 0.f, 0.f);
    }
};

__global__ __launch_bounds__(AMP_WG) void vamp_k1(VampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const VampIter it = P.iters[t];
    if (it.stopped) return;
    const GemmTile tile = xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * 128;
    const int twoN = 2 * P.N, twok = 2 * P.k;
    gemm_tile<128>(ALoadRt{P.xm, P.r, twoN, P.B, twoN, it.dxdr_prev, it.ns_prev}, P.Wt1, P.kap1, row0, col0, lds);
    using C = GemmCfg<128>;
    // w = scale * (y~ + vr * q) - q   (vamp.py:68-72; `x_tilde - q` is what V @ consumes).  Every
    // load of this thread's elements first, unconditional at a clamped index (the w stores may
    // alias them as far as the compiler knows, and a branch around a load serialises the loads'
    // latencies: amp_gemm.h ALoadPlain); out-of-range elements are never stored
    constexpr int IT = GBM * 128 / AMP_WG;
    float yv[IT], s2v[IT];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
        const int e = threadIdx.x + u * AMP_WG;
        const int row = min(row0 + (e >> 7), P.B - 1), col = min(col0 + (e & 127), twok - 1);
        yv[u] = P.ytil[(size_t)row * twok + col];
        s2v[u] = P.s2[col >> 1];
    }
#pragma unroll
    for (int u = 0; u < IT; ++u) {
        const int e = threadIdx.x + u * AMP_WG;
        const int rho = e >> 7, cc = e & 127;
        const int row = row0 + rho, col = col0 + cc;
        if (row < P.B && col < twok) {
            const float q = lds[rho * C::LDC + cc];
            const float sc = 1.0f / (s2v[u] + it.vr);
            const size_t o = (size_t)row * twok + col;
            P.w[o] = sc * (yv[u] + it.vr * q) - q;
        }
    }
}

struct VampDenoisePolicy {
    const float* tile;
    int ldc, spr, M, N, L, row0, colc0;
    float inv_sigma2;
    float* xm;
    float* var_new;
    const float* var_prev;
    float* secmax;
    float* secabs;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const float2 v = *reinterpret_cast<const float2*>(tile + rho * ldc + 2 * (sj * M + m));
        rr = v.x; ri = v.y; it = inv_sigma2;
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * N + colc0 + sj * M + m;
        *reinterpret_cast<float2*>(xm + 2 * o) = make_float2(xr, xi);
        var_new[o] = var;
        pa.sumvar += (double)var;
        pa.notclose += torch_close(var, var_prev[o]) ? 0u : 1u;     // vamp.py:185
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * L + (colc0 / M) + sj;
        secmax[o] = smax;
        secabs[o] = sabs;
    }
};

template <int BN, int KK>
__global__ __launch_bounds__(AMP_WG) void vamp_k2(VampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const VampIter it = P.iters[t];
    if (it.stopped) return;
    using C = GemmCfg<BN>;
    const GemmTile tile = xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * BN;
    const int twoN = 2 * P.N, twok = 2 * P.k;
    gemm_tile<BN>(ALoadPlain{P.w, twok, P.B, twok}, P.Wt2, P.kap2, row0, col0, lds);
    // x~ = V w + r~ ; r = (x~ - alpha r~) / (1 - alpha)   (vamp.py:72, 79)
    const int nrows = min(GBM, P.B - row0), ncols = min(BN, twoN - col0);
    {
        // every load of this thread's elements first, unconditional at a clamped index (see vamp_k1)
        constexpr int IT = GBM * BN / AMP_WG;
        float xv[IT], rv[IT];
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int e = threadIdx.x + u * AMP_WG;
            const size_t o = (size_t)(row0 + min(e / BN, nrows - 1)) * twoN + col0 + min(e % BN, ncols - 1);
            xv[u] = P.xm[o];
            rv[u] = P.r[o];
        }
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int e = threadIdx.x + u * AMP_WG;
            const int rho = e / BN, cc = e % BN;
            if (rho < nrows && cc < ncols) {
                const size_t o = (size_t)(row0 + rho) * twoN + col0 + cc;
                const float rt = (xv[u] - it.dxdr_prev * rv[u]) * it.ns_prev;
                const float xt = lds[rho * C::LDC + cc] + rt;
                const float rn = (xt - it.alpha * rt) * it.inv1ma;
                P.r[o] = rn;
                lds[rho * C::LDC + cc] = rn;
            }
        }
    }
    __syncthreads();
    VampDenoisePolicy pol;
    pol.tile = lds; pol.ldc = C::LDC; pol.M = P.M; pol.N = P.N; pol.L = P.L;
    pol.spr = (ncols / 2) / P.M; pol.row0 = row0; pol.colc0 = col0 / 2;
    pol.inv_sigma2 = it.inv_sigma2;
    pol.xm = P.xm;
    pol.var_new = var_buf(P, t);
    pol.var_prev = var_buf(P, t + 1);
    pol.secmax = P.secmax;
    pol.secabs = P.secabs;
    PartAcc pa;
    denoise_sections<true, KK>(pol, nrows * pol.spr, P.M, P.c, pa);
    part_block_store(pa, P.parts + (size_t)t * P.nblk2 + blockIdx.y * gridDim.x + blockIdx.x, lds + C::CTILE_FLOATS);
}

// One workgroup after K2(t): partial reduction, exact float64 fix-up of out-of-range
// sections, allclose decision and the scalars of iteration t+1.
__global__ __launch_bounds__(RWG) void vamp_r(VampK P, Const64 c64, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    __shared__ double s_fix[RWG / 64];
    __shared__ unsigned s_nc[RWG / 64];
    const VampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) P.iters[t + 1] = cur;
        return;
    }
    PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk2, P.nblk2, lds);
    int fixed = 0;
    if (part_allnan(pa)) {
        // the reference's G is NaN / inf: every section of this iteration is NaN
        if (!cur.fixed_all) nan_fill(P.xm, var_buf(P, t), (size_t)P.B * P.N);
        pa.sumvar = __longlong_as_double(0x7ff8000000000000LL);
        pa.notclose = 1;
        fixed = -1;
    } else if (part_danger(pa)) {
        // exact float64 G, then exact float64 recompute of every section below the danger
        // line (rare); the recomputed values replace the fast-path ones in the reductions
        float* vn = var_buf(P, t);
        const float* vp = var_buf(P, t + 1);
        const float inv = cur.inv_sigma2;
        const float2* r2 = reinterpret_cast<const float2*>(P.r);
        float2* x2 = reinterpret_cast<float2*>(P.xm);
        const int M = P.M;
        double dsum = 0.0;
        int dnc = 0;
        auto ldf = [=](int s) {
            const size_t o0 = (size_t)s * M;
            return [=](int m, float& rr, float& ri, float& it) {
                const float2 v = r2[o0 + m];
                rr = v.x; ri = v.y; it = inv;
            };
        };
        auto stf = [&](int s) {
            const size_t o0 = (size_t)s * M;
            return [&, o0](int m, float xr, float xi, float var) {
                const size_t o = o0 + m;
                const float old = vn[o];
                dsum += (double)var - (double)old;
                dnc += (torch_close(var, vp[o]) ? 0 : 1) - (torch_close(old, vp[o]) ? 0 : 1);
                x2[o] = make_float2(xr, xi);
                vn[o] = var;
            };
        };
        double G;
        fixed = fixup_sections<true>(P.B * P.L, P.M, P.secmax, P.secabs, pa.maxabs, c64, ldf, stf, &G, s_fix);
        pa.maxabs = G;
        dsum = group_sum(dsum, 64);
        dnc = group_sum(dnc, 64);
        if ((threadIdx.x & 63) == 0) {
            s_fix[threadIdx.x >> 6] = dsum;
            s_nc[threadIdx.x >> 6] = (unsigned)dnc;
        }
        __syncthreads();
        double d = 0.0;
        unsigned nc = 0;
        for (int w = 0; w < RWG / 64; ++w) { d += s_fix[w]; nc += s_nc[w]; }
        // (sum - old) + new, in float64
        pa.sumvar += d;
        pa.notclose += nc;
        __syncthreads();
    }
    const VampIter nx = vamp_advance(P, cur, pa, fixed, t, lds);
    if (threadIdx.x == 0) {
        P.iters[t + 1] = nx;
        if (nx.stopped || t + 1 == P.max_iter) *P.status = vamp_make_status(P, cur, nx, fixed);
    }
}

// ---- trial-sharded iteration (amp_vamp_run_sharded; SURVEY §8(e) exact-compat mode) ----
// Each rank holds a contiguous slice of the batch; vamp_k1 / vamp_k2 run on it unchanged.  The
// batch-global values of vamp_r (sum var, allclose count, max|xi|, min section max, and on the
// rare path the exact float64 max|xi| and the recomputed sections' deltas) go through the
// registered all-reduce hook in three stages, so every rank derives the scalars a single
// whole-batch forward derives (up to the float64 summation order of var.mean()).
//   xr1: local partials -> xs.sum / xs.mx            [hook: SUM sum[2], MAX mx[2]]
//   xr2: all-NaN / no-danger iterations advance here; the rare path publishes its local
//        exact max|xi| candidate -> xs.gmax          [hook: MAX gmax[1]]
//   xr3: rare path: exact recompute of the local out-of-range sections -> xs.fix
//                                                     [hook: SUM fix[3]]
//   xr4: rare path: fold the deltas and advance.
// Every stage runs on every rank every iteration (stopped iterations carry zeros), so the
// hook calls match across ranks with no host synchronisation.
__device__ inline PartAcc xs_global(const XState& x) {
    PartAcc pa;
    pa.sumvar = x.sum[0];
    pa.notclose = (uint32_t)x.sum[1];
    pa.maxabs = x.mx[0];
    pa.minsecmax = -x.mx[1];
    return pa;
}

__global__ __launch_bounds__(RWG) void vamp_xr1(VampK P, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    XState* xs = P.xs;
    if (P.iters[t].stopped) {
        if (threadIdx.x == 0) { xs->sum[0] = xs->sum[1] = 0.0; xs->mx[0] = xs->mx[1] = 0.0; }
        return;
    }
    const PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk2, P.nblk2, lds);
    if (threadIdx.x == 0) {
        xs->sum[0] = pa.sumvar;
        xs->sum[1] = (double)pa.notclose;
        // a NaN / inf max|xi| (the reference's all-NaN iteration) must win the MAX: +inf
        xs->mx[0] = (pa.maxabs <= 1.7976931348623157e308) ? pa.maxabs : INFINITY;
        xs->mx[1] = (pa.minsecmax == pa.minsecmax) ? -pa.minsecmax : INFINITY;
    }
}

__global__ __launch_bounds__(RWG) void vamp_xr2(VampK P, Const64 c64, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    XState* xs = P.xs;
    const VampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) { P.iters[t + 1] = cur; xs->mode = 0; xs->gmax[0] = 0.0; }
        return;
    }
    PartAcc pa = xs_global(*xs);
    if (!part_allnan(pa) && part_danger(pa)) {
        // the rare path: this rank's exact float64 max|xi| over its candidate sections
        const float inv = cur.inv_sigma2;
        const float2* r2 = reinterpret_cast<const float2*>(P.r);
        const int M = P.M;
        const double G32 = pa.maxabs, slack = logit_slack(G32);
        double gm = 0.0;
        for (int s = threadIdx.x; s < P.B * P.L; s += blockDim.x) {
            if (!((double)P.secabs[s] >= G32 - slack)) continue;
            const size_t o0 = (size_t)s * M;
            gm = fmax(gm, section_absmax_f64([=](int m, float& rr, float& ri, float& it) {
                const float2 v = r2[o0 + m];
                rr = v.x; ri = v.y; it = inv;
            }, M, c64));
        }
        gm = group_max(gm, 64);
        double* sd = reinterpret_cast<double*>(lds);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sd[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            double G = 0.0;
            for (int w = 0; w < RWG / 64; ++w) G = fmax(G, sd[w]);
            xs->gmax[0] = G;
            xs->mode = 2;
        }
        return;
    }
    int fixed = 0;
    if (part_allnan(pa)) {
        if (!cur.fixed_all) nan_fill(P.xm, var_buf(P, t), (size_t)P.B * P.N);
        pa.sumvar = __longlong_as_double(0x7ff8000000000000LL);
        pa.notclose = 1;
        fixed = -1;
    }
    const VampIter nx = vamp_advance(P, cur, pa, fixed, t, lds);
    if (threadIdx.x == 0) {
        P.iters[t + 1] = nx;
        if (nx.stopped || t + 1 == P.max_iter) *P.status = vamp_make_status(P, cur, nx, fixed);
        xs->mode = 0;
        xs->gmax[0] = 0.0;
    }
}

__global__ __launch_bounds__(RWG) void vamp_xr3(VampK P, Const64 c64, int t) {
    __shared__ double s_d[3][RWG / 64];
    XState* xs = P.xs;
    if (xs->mode != 2) {
        if (threadIdx.x == 0) xs->fix[0] = xs->fix[1] = xs->fix[2] = 0.0;
        return;
    }
    const VampIter cur = P.iters[t];
    const PartAcc pa = xs_global(*xs);
    const double G = xs->gmax[0], slack = logit_slack(pa.maxabs);
    float* vn = var_buf(P, t);
    const float* vp = var_buf(P, t + 1);
    const float inv = cur.inv_sigma2;
    const float2* r2 = reinterpret_cast<const float2*>(P.r);
    float2* x2 = reinterpret_cast<float2*>(P.xm);
    const int M = P.M;
    double dsum = 0.0;
    int dnc = 0, cnt = 0;
    for (int s = threadIdx.x; s < P.B * P.L; s += blockDim.x) {
        if (!((double)P.secmax[s] - G < AMP_DANGER + slack)) continue;
        ++cnt;
        const size_t o0 = (size_t)s * M;
        exact_section_f64<true>(
            [=](int m, float& rr, float& ri, float& it) {
                const float2 v = r2[o0 + m];
                rr = v.x; ri = v.y; it = inv;
            },
            [&](int m, float xr, float xi, float var) {
                const size_t o = o0 + m;
                const float old = vn[o];
                dsum += (double)var - (double)old;
                dnc += (torch_close(var, vp[o]) ? 0 : 1) - (torch_close(old, vp[o]) ? 0 : 1);
                x2[o] = make_float2(xr, xi);
                vn[o] = var;
            },
            M, c64, G);
    }
    dsum = group_sum(dsum, 64);
    dnc = group_sum(dnc, 64);
    cnt = group_sum(cnt, 64);
    if ((threadIdx.x & 63) == 0) {
        s_d[0][threadIdx.x >> 6] = dsum; s_d[1][threadIdx.x >> 6] = (double)dnc; s_d[2][threadIdx.x >> 6] = (double)cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0, c = 0.0;
        for (int w = 0; w < RWG / 64; ++w) { a += s_d[0][w]; b += s_d[1][w]; c += s_d[2][w]; }
        xs->fix[0] = a; xs->fix[1] = b; xs->fix[2] = c;
    }
}

__global__ __launch_bounds__(RWG) void vamp_xr4(VampK P, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    const XState* xs = P.xs;
    if (xs->mode != 2) return;
    const VampIter cur = P.iters[t];
    PartAcc pa = xs_global(*xs);
    pa.sumvar += xs->fix[0];                                   // (sum - old) + new, in float64
    pa.notclose = (uint32_t)((long long)pa.notclose + (long long)xs->fix[1]);
    pa.maxabs = xs->gmax[0];
    const int fixed = (int)xs->fix[2];
    const VampIter nx = vamp_advance(P, cur, pa, fixed, t, lds);
    if (threadIdx.x == 0) {
        P.iters[t + 1] = nx;
        if (nx.stopped || t + 1 == P.max_iter) *P.status = vamp_make_status(P, cur, nx, fixed);
    }
}

__global__ void vamp_init_kernel(VampK P) {
    // Tracker (vamp.py:22-26) in the form the fused kernels consume:
    //   xmmse = p, r = 0 so that r~ = (xmmse - 0*r)*1 = p   (vamp.py:25)
    //   var buffer 1 = ones: the `prev` of iteration 0      (vamp.py:24, 182)
    const float p = (float)P.sparsity;
    const size_t BN_ = (size_t)P.B * P.N;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN_; e += (size_t)gridDim.x * blockDim.x) {
        reinterpret_cast<float2*>(P.xm)[e] = make_float2(p, 0.f);
        reinterpret_cast<float2*>(P.r)[e] = make_float2(0.f, 0.f);
        P.var1[e] = 1.0f;
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P.k; i += gridDim.x * blockDim.x) P.s2[i] = P.s[i] * P.s[i];
}

// The last executed iteration wrote var into buffer (T-1)&1; buffer 0 is the caller's.
__global__ void vamp_output_kernel(VampK P) {
    const int T = P.status->T;
    if (((T - 1) & 1) == 0) return;
    const size_t BN_ = (size_t)P.B * P.N;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN_; e += (size_t)gridDim.x * blockDim.x)
        P.var0[e] = P.var1[e];
}

// AMP_VAMP_GEMM=f32: AMP_GEMM_AUTO keeps the f32-MFMA persistent GEMMs (measurement / A-B runs)
bool gemm_f32_requested() {
    static const bool v = [] {
        const char* e = diag_env("AMP_VAMP_GEMM");
        return e && e[0] == 'f';
    }();
    return v;
}

// AMP_VAMP_GEMM=h2 makes AUTO pick the fp16x2 form (A/B runs only: 22-bit operands)
static bool gemm_h2_requested() {
    static const bool v = [] {
        const char* e = diag_env("AMP_VAMP_GEMM");
        return e && e[0] == 'h';
    }();
    return v;
}

// The persistent engine's GEMM arithmetic for a shape whose planes fit (amp_vamp_args.gemm):
// 0 f32 MFMA, 1 bf16x3, 2 fp16x2.  AUTO: bf16x3 — the fastest form whose operands keep all 24
// bits of an f32 (three 8-bit pieces) and whose dropped product terms are < 2^-24 relative, i.e.
// the reference's c64 operand precision (vamp.py:67, 72).  fp16x2 (two 11-bit pieces, 22 bits,
// the 2^-22 lo.lo term dropped) is narrower than the reference and runs only when asked for
// (AMP_GEMM_H2 or AMP_VAMP_GEMM=h2).
// AMP_GEMM_I8 (3): int8x4 block fixed point — 31-bit operands per row / column, more accurate than
// an f32 sum (amp_persist.h gemm_i8).
static bool gemm_i8_requested() {   // AMP_VAMP_GEMM=i8: AUTO picks int8x4 (A/B runs)
    static const bool v = [] {
        const char* e = diag_env("AMP_VAMP_GEMM");
        return e && e[0] == 'i';
    }();
    return v;
}
static int vamp_gemm_mode(int gemm, bool fits) {
    if (gemm == AMP_GEMM_I8) return 3;
    if (gemm == AMP_GEMM_H2) return 2;
    if (gemm == AMP_GEMM_X3) return 1;
    if (gemm == AMP_GEMM_F32 || !fits || gemm_f32_requested()) return 0;
    return gemm_h2_requested() ? 2 : gemm_i8_requested() ? 3 : 1;
}

int vamp_gemm_select(const amp_dims* d, int k, int gemm) {
    const bool fits = vamp_persist_x3_fits(d->N, k, d->L);
    if ((gemm == AMP_GEMM_X3 || gemm == AMP_GEMM_H2 || gemm == AMP_GEMM_I8) && !fits) return 0;
    return vamp_gemm_mode(gemm, fits);
}

static int vamp_setup(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, VampK& P, Const64& c64,
                      int chans = 1) {
    int rc = check_dims(d, c);
    if (rc) return rc;
    AMP_REQUIRE(a && a->U && a->s && a->Vh && a->y && a->r && a->xmmse && a->var && a->status && a->ws,
                "amp_vamp: null pointer argument");
    AMP_REQUIRE(a->k > 0 && a->k <= d->N && a->k <= d->n && a->k % 2 == 0, "amp_vamp: k = %d must be min(n, N), even",
                a->k);
    AMP_REQUIRE(a->max_iter > 0, "amp_vamp: max_iter must be positive");
    const VampWs w = vamp_carve(d, a->k, a->max_iter, a->ws, chans);
    AMP_REQUIRE(a->ws_bytes >= w.bytes, "amp_vamp: workspace %zu < %zu bytes", a->ws_bytes, w.bytes);
    vamp_geometry(d, a->k, P);
    P.max_iter = a->max_iter;
    P.noise_var = a->noise_var;
    P.sparsity = a->sparsity;
    P.Wt0 = w.Wt0; P.Wt1 = w.Wt1; P.Wt2 = w.Wt2;
    P.s = (const float*)a->s; P.s2 = w.s2; P.ytil = w.ytil; P.w = w.w;
    P.r = (float*)a->r; P.xm = (float*)a->xmmse;
    P.var0 = (float*)a->var;
    P.var1 = w.var1;
    P.secmax = w.secmax; P.secabs = w.secabs; P.parts = w.parts; P.iters = w.iters; P.status = (amp_status*)a->status;
    P.nwg = cdiv(d->B, PBM);
    P.Bmean = d->B;
    P.xs = w.xs;
    P.E = 1;
    P.wpe = P.nwg;
    P.Wq0 = w.Wq0; P.Wq1 = w.Wq1; P.Wq2 = w.Wq2; P.pparts = w.pparts; P.pxch = w.pxch; P.pbar = w.pbar;
    P.gen = 0;
    P.ytil_in_kernel = 0;
    P.dec_on = 0; P.ibits = 0; P.xtrue = nullptr; P.sym = nullptr; P.idx = nullptr; P.counts = nullptr;
    P.host_rec = nullptr;
    P.fold_in = fold_in_kernel() ? 1 : 0;
    P.dwg = w.dwg;
    P.y = (const float*)a->y;
    P.trace = nullptr;
    P.c = to_const(c);
    c64 = to_const64(c);
    AMP_REQUIRE(a->gemm >= AMP_GEMM_AUTO && a->gemm <= AMP_GEMM_I8, "amp_vamp: gemm %d", a->gemm);
    const bool x3_fits = vamp_persist_x3_fits(d->N, a->k, d->L);
    AMP_REQUIRE((a->gemm != AMP_GEMM_X3 && a->gemm != AMP_GEMM_H2 && a->gemm != AMP_GEMM_I8) || x3_fits,
                "amp_vamp: the split-precision engines need k == N, N %% 64 == 0 and "
                "their LDS carve within 160 KB (N = %d, L = %d)", d->N, d->L);
    P.x3 = vamp_gemm_mode(a->gemm, x3_fits);
    P.Wx1 = w.Wx1; P.Wx2 = w.Wx2;
    P.dump = debug_dump_ptr();
    P.wch = 0;
    P.sch = 0;
    P.wg_off = 0;
    P.nwg_x = P.nwg;
    P.row_off = 0;
    return AMP_OK;
}

static std::once_flag g_vamp_attr_once;
static int g_vamp_attr_rc = 0;

template <int KK>
static int vamp_k2_attrs() {
    int rc = set_lds_attr<128>((const void*)vamp_k2<128, KK>);
    return rc ? rc : set_lds_attr<256>((const void*)vamp_k2<256, KK>);
}

static int vamp_attrs() {
    std::call_once(g_vamp_attr_once, [] {
        int rc = set_lds_attr<128>((const void*)vamp_k1);
        if (!rc) rc = vamp_k2_attrs<1>();
        if (!rc) rc = vamp_k2_attrs<2>();
        if (!rc) rc = vamp_k2_attrs<4>();
        if (!rc) rc = vamp_k2_attrs<8>();
        if (!rc) rc = vamp_k2_attrs<16>();
        if (!rc) rc = vamp_k2_attrs<64>();
        g_vamp_attr_rc = rc;
    });
    return g_vamp_attr_rc;
}

template <int KK>
static void launch_k2_kk(const VampK& P, int t, hipStream_t st) {
    dim3 g2(cdiv(P.B, GBM), P.ncp2 / P.bn2);
    if (P.bn2 == 128)
        hipLaunchKernelGGL((vamp_k2<128, KK>), g2, dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, P, t);
    else
        hipLaunchKernelGGL((vamp_k2<256, KK>), g2, dim3(AMP_WG), GemmCfg<256>::LDS_BYTES, st, P, t);
}

// GEMM2 + denoiser, instantiated per constellation size (K is validated by check_dims)
static void launch_k2(const VampK& P, int t, hipStream_t st) {
    switch (P.c.K) {
    case 1: launch_k2_kk<1>(P, t, st); break;
    case 2: launch_k2_kk<2>(P, t, st); break;
    case 4: launch_k2_kk<4>(P, t, st); break;
    case 8: launch_k2_kk<8>(P, t, st); break;
    case 16: launch_k2_kk<16>(P, t, st); break;
    default: launch_k2_kk<64>(P, t, st); break;
    }
}


static int vamp_prepare_impl(const VampK& P, const amp_vamp_args* a, hipStream_t st) {
    int rc = vamp_attrs();
    if (rc) return rc;
    // Wt0: y~ = (s * U^H) y        (vamp.py:22)    X[o][j] = s_o conj(U[j][o]),  o < k, j < n
    rc = build_cweight((const float2*)a->U, 1, P.k, 1, P.s, P.k, P.n, (float*)P.Wt0, P.kap0, P.ncp0, st);
    if (rc) return rc;
    // Wt1: q = Vh r~               (vamp.py:67)    X[o][j] = Vh[o][j],           o < k, j < N
    rc = build_cweight((const float2*)a->Vh, P.N, 1, 0, nullptr, P.k, P.N, (float*)P.Wt1, P.kap1, P.ncp1, st);
    if (rc) return rc;
    // Wt2: V (x~ - q), V = Vh^H    (vamp.py:19,72) X[o][j] = conj(Vh[j][o]),     o < N, j < k
    rc = build_cweight((const float2*)a->Vh, 1, P.N, 1, nullptr, P.N, P.k, (float*)P.Wt2, P.kap2, P.ncp2, st);
    if (rc) return rc;
    const int g = (int)std::min<size_t>(((size_t)P.B * P.N + 255) / 256, 2048);
    hipLaunchKernelGGL(vamp_init_kernel, dim3(g), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("vamp_init");
    hipLaunchKernelGGL(vamp_init_scalars, dim3(1), dim3(RWG), 0, st, P);
    AMP_LAUNCH_CHECK("vamp_init_scalars");
    // y~ = (s * U^H) y as a GEMM over the batch
    return gemm_store((const float*)a->y, 2 * P.n, P.B, 2 * P.n, P.Wt0, P.kap0, P.ncp0, P.ytil, 2 * P.k, 2 * P.k, st);
}

// Persistent engine: ONE launch builds the 16x16x4-packed operators (Vh, V), the y~ operator
// s Uh and zeroes the barrier words; the Tracker's initial state and the iteration-0 scalars
// are formed inside vamp_persist.  y~ = (s Uh) y: on the fp16x2 engine inside vamp_persist's
// prologue (n == 2N; AMP_YTIL_IN_KERNEL=0 keeps the separate gemm_store launch), on the other
// arithmetics from gemm_store (the f32 engine can form it in-kernel with AMP_YTIL_IN_KERNEL=1: ~20
// us per forward, but its 16x16x4 summation order flipped the allclose early exit of a cfg2 QPSK
// 9 dB golden, T 4 vs the reference's 3).
static int ytil_in_kernel_env() {
    static const int v = [] {
        const char* e = diag_env("AMP_YTIL_IN_KERNEL");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    return v;
}

// y~ of the split-precision engines (bf16x3, int8x4) as its own bf16x3 launch (ytil_x3_launch,
// amp_vamp_persist_x3.hip); AMP_YTIL_X3=0 keeps the f32 gemm_store launch (A/B runs)
static bool ytil_x3_env() {
    static const bool v = [] {
        const char* e = diag_env("AMP_YTIL_X3");
        return !(e && e[0] == '0');
    }();
    return v;
}
bool ytil_x3_fits(int n, int k);
int ytil_x3_launch(const float* y, int n, int rows, const void* wq, float* ytil, int k, hipStream_t st,
                   int rows_per_op = 0, long long wq_stride = 0);

// Side-by-side epochs with a channel each (P.wch != 0): every epoch's split-precision operators
// (Vh, V, s Uh) from its own U / s / Vh (a->U + e * ch.U, ...), then y~ per epoch.
struct EpochChannels {
    long long U = 0, s = 0, Vh = 0;   // elements between epochs' U (c64), s (f32), Vh (c64)
};
static int vamp_persist_prepare_ch(VampK& P, const amp_vamp_args* a, const EpochChannels& ch, hipStream_t st) {
    const int pk = P.x3 == 3 ? WPACKI8 : WPACKX3;
    const long long q0 = (long long)16 * P.k * P.n;   // bytes between epochs' s Uh (the carve's f32 stride)
    // every epoch's three operators, CW_MAX_JOBS / 3 epochs per launch (the first zeroes the barrier words)
    constexpr int EPL = CW_MAX_JOBS / 3;
    for (int e0 = 0; e0 < P.E; e0 += EPL) {
        CWeightJob j[CW_MAX_JOBS];
        const int ne = std::min(EPL, P.E - e0);
        for (int i = 0; i < ne; ++i) {
            const int e = e0 + i;
            const float2* U = (const float2*)a->U + e * ch.U;
            const float2* Vh = (const float2*)a->Vh + e * ch.Vh;
            const float* sv = (const float*)a->s + e * ch.s;
            j[3 * i + 0] = CWeightJob{Vh, P.N, 1, 0, nullptr, P.k, P.N, (float*)((char*)P.Wx1 + e * P.wch), P.N, P.k, pk};
            j[3 * i + 1] = CWeightJob{Vh, 1, P.N, 1, nullptr, P.N, P.k, (float*)((char*)P.Wx2 + e * P.wch), P.k, P.N, pk};
            j[3 * i + 2] = CWeightJob{U, 1, P.k, 1, sv, P.k, P.n, (float*)((char*)P.Wq0 + e * q0), P.n, P.k, WPACKX3};
        }
        const int rc = build_cweights(j, 3 * ne, e0 == 0 ? P.pbar : nullptr, PBAR_WORDS, st);
        if (rc) return rc;
    }
    // y~ of every epoch in one launch, each row block with its epoch's s Uh
    return ytil_x3_launch((const float*)a->y, P.n, P.B * P.E, P.Wq0, P.ytil, P.k, st, P.B, q0);
}

static int vamp_persist_prepare(VampK& P, const amp_vamp_args* a, hipStream_t st, const EpochChannels* ch = nullptr) {
    static std::atomic<unsigned> gen{0};
    P.gen = ++gen;
    if (ch && P.wch) {
        P.ytil_in_kernel = 0;
        return vamp_persist_prepare_ch(P, a, *ch, st);
    }
    const int env = ytil_in_kernel_env();
    if (P.x3 == 2)
        P.ytil_in_kernel = (env != 0 && vamp_persist_ytil_h2(P)) ? 1 : 0;
    else
        P.ytil_in_kernel = (!P.x3 && env == 1 && vamp_persist_ytil_in_kernel(P)) ? 1 : 0;
    const bool yk = P.ytil_in_kernel != 0;
    const bool yx3 = !yk && (P.x3 == 1 || P.x3 == 3) && ytil_x3_env() && ytil_x3_fits(P.n, P.k);
    CWeightJob j[3];
    if (P.x3) {
        const int pk = P.x3 == 3 ? WPACKI8 : P.x3 == 2 ? WPACKH2 : WPACKX3;
        //   q = Vh r~    (vamp.py:67)    X[o][j] = Vh[o][j],           o < k, j < N   (bf16x3 / fp16x2 planes)
        j[0] = CWeightJob{(const float2*)a->Vh, P.N, 1, 0, nullptr, P.k, P.N, (float*)P.Wx1, P.N, P.k, pk};
        //   V (x~ - q)   (vamp.py:19,72) X[o][j] = conj(Vh[j][o]),     o < N, j < k
        j[1] = CWeightJob{(const float2*)a->Vh, 1, P.N, 1, nullptr, P.N, P.k, (float*)P.Wx2, P.k, P.N, pk};
    } else {
    //   q = Vh r~        (vamp.py:67)    X[o][j] = Vh[o][j],           o < k, j < N
    j[0] = CWeightJob{(const float2*)a->Vh, P.N, 1, 0, nullptr, P.k, P.N, (float*)P.Wq1, 2 * P.N, 2 * P.k, WPACK16};
    //   V (x~ - q)       (vamp.py:19,72) X[o][j] = conj(Vh[j][o]),     o < N, j < k
    j[1] = CWeightJob{(const float2*)a->Vh, 1, P.N, 1, nullptr, P.N, P.k, (float*)P.Wq2, 2 * P.k, 2 * P.N, WPACK16};
    }
    //   y~ = (s U^H) y   (vamp.py:22)    X[o][j] = s_o conj(U[j][o]),  o < k, j < n
    j[2] = (yk && P.x3 == 2)
               ? CWeightJob{(const float2*)a->U, 1, P.k, 1, P.s, P.k, P.n, (float*)P.Wq0, P.n, P.k, WPACKH2, YH2_EX}
           : yx3 ? CWeightJob{(const float2*)a->U, 1, P.k, 1, P.s, P.k, P.n, (float*)P.Wq0, P.n, P.k, WPACKX3}
           : yk ? CWeightJob{(const float2*)a->U, 1, P.k, 1, P.s, P.k, P.n, (float*)P.Wq0, 2 * P.n, 2 * P.k, WPACK16}
                : CWeightJob{(const float2*)a->U, 1, P.k, 1, P.s, P.k, P.n, (float*)P.Wt0, P.kap0, P.ncp0, WPACK32};
    int rc = build_cweights(j, 3, P.pbar, PBAR_WORDS, st);
    if (rc || yk) return rc;
    if (yx3) return ytil_x3_launch((const float*)a->y, P.n, P.B * P.E, P.Wq0, P.ytil, P.k, st);
    rc = vamp_attrs();
    if (rc) return rc;
    return gemm_store((const float*)a->y, 2 * P.n, P.B * P.E, 2 * P.n, P.Wt0, P.kap0, P.ncp0, P.ytil, 2 * P.k,
                      2 * P.k, st);
}

static int vamp_iterate_impl(const VampK& P, const Const64& c64, int t, hipStream_t st) {
    dim3 g1(cdiv(P.B, GBM), P.ncp1 / 128);
    hipLaunchKernelGGL(vamp_k1, g1, dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, P, t);
    AMP_LAUNCH_CHECK("vamp_k1");
    launch_k2(P, t, st);
    AMP_LAUNCH_CHECK("vamp_k2");
    hipLaunchKernelGGL(vamp_r, dim3(1), dim3(RWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("vamp_r");
    return AMP_OK;
}

static int vamp_finalize_impl(const VampK& P, hipStream_t st) {
    const int g = (int)std::min<size_t>(((size_t)P.B * P.N + 255) / 256, 2048);
    hipLaunchKernelGGL(vamp_output_kernel, dim3(g), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("vamp_output");
    return AMP_OK;
}

static int vamp_iterate_sharded(const VampK& P, const Const64& c64, int t, hipStream_t st, bool& hook_failed) {
    dim3 g1(cdiv(P.B, GBM), P.ncp1 / 128);
    hipLaunchKernelGGL(vamp_k1, g1, dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, P, t);
    AMP_LAUNCH_CHECK("vamp_k1");
    launch_k2(P, t, st);
    AMP_LAUNCH_CHECK("vamp_k2");
    hipLaunchKernelGGL(vamp_xr1, dim3(1), dim3(RWG), 0, st, P, t);
    AMP_LAUNCH_CHECK("vamp_xr1");
    // every hook call is made on every rank even after one failed: the ranks' collectives stay
    // matched and a failed rank's poisoned words reach the others (amp_sparc.h)
    hook_failed |= call_allreduce_hook(P.xs->sum, 2, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hook_failed |= call_allreduce_hook(P.xs->mx, 2, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(vamp_xr2, dim3(1), dim3(RWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("vamp_xr2");
    hook_failed |= call_allreduce_hook(P.xs->gmax, 1, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(vamp_xr3, dim3(1), dim3(RWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("vamp_xr3");
    hook_failed |= call_allreduce_hook(P.xs->fix, 3, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hipLaunchKernelGGL(vamp_xr4, dim3(1), dim3(RWG), 0, st, P, t);
    AMP_LAUNCH_CHECK("vamp_xr4");
    return AMP_OK;
}

}  // namespace amp

using namespace amp;

extern "C" {

int amp_vamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, int32_t B_global,
                         void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(allreduce_hook_set(), "amp_vamp_run_sharded: no all-reduce hook registered (amp_set_allreduce_hook)");
    AMP_REQUIRE(B_global >= d->B, "amp_vamp_run_sharded: B_global = %d < this rank's B = %d", B_global, d->B);
    P.Bmean = B_global;
    hipStream_t st = (hipStream_t)stream;
    rc = vamp_prepare_impl(P, a, st);
    bool hook_failed = false;
    for (int t = 0; t < P.max_iter && !rc; ++t) rc = vamp_iterate_sharded(P, c64, t, st, hook_failed);
    if (!rc && hook_failed) rc = hook_failure("vamp");
    return rc ? rc : vamp_finalize_impl(P, st);
}

// Diagnostic: one persistent-engine forward whose workgroups stamp s_memtime at every phase
// boundary: trace[(wg * max_iter + t) * 10 + phase], phases = start, r~ built, GEMM1, w stored,
// GEMM2 + r, partial published, barrier passed, scalars ready, denoiser done, vamp_advance started; then per
// workgroup [nwg * max_iter * 10 + 2 * wg] = s_memtime / s_memrealtime at kernel start and
// [nwg * max_iter * 10 + 2 * nwg + 2 * wg] the same pair at its end (trace: 4 nwg more words).
int amp_vamp_persist_trace(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* trace,
                           void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    const int ncu = device_cu_count();
    AMP_REQUIRE(trace && vamp_persist_eligible(d, a->k, ncu), "amp_vamp_persist_trace: not eligible / null trace");
    hipStream_t st = (hipStream_t)stream;
    rc = vamp_persist_prepare(P, a, st);
    if (rc) return rc;
    P.trace = (unsigned long long*)trace;
    return vamp_persist_launch(P, c64, DecConst{}, st, ncu);
}

int amp_vamp_select_gemm(const amp_dims* d, int32_t k, int32_t gemm) {
    if (!d || k <= 0 || gemm < AMP_GEMM_AUTO || gemm > AMP_GEMM_I8) return AMP_E_ARG;
    const bool fits = vamp_persist_x3_fits(d->N, k, d->L);
    if ((gemm == AMP_GEMM_X3 || gemm == AMP_GEMM_H2 || gemm == AMP_GEMM_I8) && !fits) return AMP_E_ARG;
    static const int code[4] = {AMP_GEMM_F32, AMP_GEMM_X3, AMP_GEMM_H2, AMP_GEMM_I8};
    return code[vamp_gemm_mode(gemm, fits)];
}

int amp_vamp_select_engine(const amp_dims* d, int32_t k, int32_t engine) {
    if (!d || k <= 0) return AMP_E_ARG;
    const bool elig = vamp_persist_eligible(d, k, device_cu_count());
    if (engine == AMP_ENGINE_PERSISTENT) return elig ? AMP_ENGINE_PERSISTENT : AMP_E_ARG;
    if (engine == AMP_ENGINE_AUTO && elig) return AMP_ENGINE_PERSISTENT;
    return engine == AMP_ENGINE_AUTO || engine == AMP_ENGINE_LAUNCHES ? AMP_ENGINE_LAUNCHES : AMP_E_ARG;
}

size_t amp_vamp_workspace_bytes(const amp_dims* d, int32_t k, int32_t max_iter) {
    if (!d || k <= 0 || max_iter <= 0) return 0;
    return vamp_carve(d, k, max_iter, nullptr).bytes;
}

int amp_vamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    return vamp_prepare_impl(P, a, (hipStream_t)stream);
}

int amp_vamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, int32_t t, void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(t >= 0 && t < a->max_iter, "amp_vamp_iterate: t = %d outside [0, %d)", t, a->max_iter);
    rc = vamp_attrs();
    if (rc) return rc;
    return vamp_iterate_impl(P, c64, t, (hipStream_t)stream);
}

int amp_vamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    return vamp_finalize_impl(P, (hipStream_t)stream);
}

int amp_vamp_run(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    AMP_REQUIRE(a->engine >= AMP_ENGINE_AUTO && a->engine <= AMP_ENGINE_PERSISTENT, "amp_vamp_run: engine %d",
                a->engine);
    const int ncu = device_cu_count();
    const bool elig = vamp_persist_eligible(d, a->k, ncu);
    AMP_REQUIRE(a->engine != AMP_ENGINE_PERSISTENT || elig,
                "amp_vamp_run: persistent engine needs k == N in {64, 128, 256}, M <= 64 and ceil(B/16) = %d <= "
                "%d CUs", cdiv(d->B, PBM), ncu);
    if (a->engine == AMP_ENGINE_PERSISTENT || (a->engine == AMP_ENGINE_AUTO && elig)) {
        rc = vamp_persist_prepare(P, a, st);
        if (rc) return rc;
        return vamp_persist_launch(P, c64, DecConst{}, st, ncu);
    }
    rc = vamp_prepare_impl(P, a, st);
    if (rc) return rc;
    for (int t = 0; t < P.max_iter; ++t) {
        rc = vamp_iterate_impl(P, c64, t, st);
        if (rc) return rc;
    }
    return vamp_finalize_impl(P, st);
}

int amp_vamp_detect_count(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                          const amp_vamp_decide_args* dec, void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(dec && dec->x && dec->sym && dec->idx && dec->counts, "amp_vamp_detect_count: null pointer argument");
    AMP_REQUIRE(dec->ibits_trunc >= 0 && dec->ibits_trunc < 64, "amp_vamp_detect_count: ibits_trunc out of range");
    AMP_REQUIRE(d->Lin * d->Na * d->M == d->N, "amp_vamp_detect_count: inconsistent dims");
    const int ncu = device_cu_count();
    AMP_REQUIRE(a->engine != AMP_ENGINE_LAUNCHES && vamp_persist_eligible(d, a->k, ncu),
                "amp_vamp_detect_count: needs the persistent engine (k == N in {64, 128, 256}, M <= 64, "
                "ceil(B/16) = %d <= %d CUs)", cdiv(d->B, PBM), ncu);
    hipStream_t st = (hipStream_t)stream;
    rc = vamp_persist_prepare(P, a, st);
    if (rc) return rc;
    P.dec_on = 1;
    P.ibits = dec->ibits_trunc;
    P.xtrue = (const float2*)dec->x;
    P.sym = (const long long*)dec->sym;
    P.idx = (const long long*)dec->idx;
    P.counts = (amp_counts*)dec->counts;
    P.host_rec = P.fold_in ? (unsigned char*)dec->host_record : nullptr;
    return vamp_persist_launch(P, c64, to_decconst(c), st, ncu);
}

int amp_vamp_max_epochs(const amp_dims* d, int32_t k) {
    if (!d || k <= 0 || d->B <= 0) return 0;
    return vamp_persist_max_epochs(d, k, device_cu_count());
}

int amp_vamp_max_epochs_gemm(const amp_dims* d, int32_t k, int32_t gemm) {
    if (!d || k <= 0 || d->B <= 0 || gemm < AMP_GEMM_AUTO || gemm > AMP_GEMM_I8) return 0;
    return vamp_persist_max_epochs(d, k, device_cu_count(), gemm);
}

int amp_vamp_epochs_ch_eligible(const amp_dims* d, int32_t k, int32_t gemm) {
    if (!d || k <= 0 || d->B <= 0 || gemm < AMP_GEMM_AUTO || gemm > AMP_GEMM_I8) return 0;
    if (vamp_persist_max_epochs(d, k, device_cu_count(), gemm) < 1) return 0;
    const int x3 = vamp_gemm_select(d, k, gemm);   // the check of amp_vamp_detect_count_epochs_ch
    return ((x3 == 1 || x3 == 3) && ytil_x3_fits(d->n, k)) ? 1 : 0;
}

size_t amp_vamp_epochs_workspace_bytes(const amp_dims* d, int32_t k, int32_t max_iter, int32_t epochs) {
    if (!d || k <= 0 || max_iter <= 0 || epochs < 1 || (long)d->B * epochs > (1L << 30)) return 0;
    amp_dims de = *d;
    de.B = d->B * epochs;   // the carve holds every epoch's rows, one granule pair per workgroup and
                            // one operator set per epoch (amp_vamp_detect_count_epochs_ch)
    return vamp_carve(&de, k, max_iter, nullptr, epochs).bytes;
}

int amp_vamp_debug_dump(void* buf) {
    g_dump = (float*)buf;
    return AMP_OK;
}

int amp_vamp_debug_offsets(const amp_dims* d, int32_t k, int32_t max_iter, int32_t epochs, uint64_t* out) {
    if (!d || !out || k <= 0 || max_iter <= 0 || epochs < 1) return AMP_E_ARG;
    amp_dims de = *d;
    de.B = d->B * epochs;
    char* const base = reinterpret_cast<char*>(uintptr_t{4096});   // a dummy base: offsets only
    const VampWs w = vamp_carve(&de, k, max_iter, base);
    out[0] = (uint64_t)((char*)w.pparts - base);
    out[1] = (uint64_t)((char*)w.pxch - base);
    out[2] = (uint64_t)((char*)w.pbar - base);
    out[3] = (uint64_t)((char*)w.dwg - base);
    out[4] = (uint64_t)((char*)w.ytil - base);
    return AMP_OK;
}

static int detect_count_epochs_impl(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                    const amp_vamp_decide_args* dec, int32_t epochs, const EpochChannels& ch,
                                    void* stream) {
    AMP_REQUIRE(d && epochs >= 1 && (long)d->B * epochs <= (1L << 30), "amp_vamp_detect_count_epochs: epochs = %d",
                epochs);
    const int ncu = device_cu_count();
    AMP_REQUIRE(a && a->engine != AMP_ENGINE_LAUNCHES && vamp_persist_eligible(d, a->k, ncu, epochs, a->gemm),
                "amp_vamp_detect_count_epochs: needs the persistent engine (k == N in {64, 128, 256}, M <= 64, "
                "B %% 16 == 0 when epochs > 1, epochs <= amp_vamp_max_epochs_gemm = %d)",
                a ? vamp_persist_max_epochs(d, a->k, ncu, a->gemm) : 0);
    amp_dims de = *d;
    de.B = d->B * epochs;
    VampK P;
    Const64 c64;
    int rc = vamp_setup(&de, c, a, P, c64, epochs);   // carve and buffers over all epochs' rows and channels
    if (rc) return rc;
    const bool per = ch.U || ch.s || ch.Vh;
    AMP_REQUIRE(!per || (ch.U > 0 && ch.s > 0 && ch.Vh > 0),
                "amp_vamp_detect_count_epochs_ch: strides must be all zero (one channel) or all positive");
    AMP_REQUIRE(!per || ((P.x3 == 1 || P.x3 == 3) && ytil_x3_fits(P.n, P.k)),
                "amp_vamp_detect_count_epochs_ch: a channel per epoch needs the bf16x3 or int8x4 engine and n == 2 k "
                "(gemm %d, n %d, k %d)", a->gemm, P.n, P.k);
    if (per) {
        P.wch = (long long)12 * P.k * P.N;    // the carve's stride of the X3 / I8 operators (3 k N floats)
        P.sch = (int)ch.s;
    }
    P.B = d->B;                               // the batch of one epoch (mean var, vamp.py:85)
    P.Bmean = d->B;
    P.E = epochs;
    P.wpe = cdiv(d->B, PBM);
    P.nwg = P.E * P.wpe;
    P.nwg_x = P.nwg;
    AMP_REQUIRE(P.x3 || P.nwg <= ncu, "amp_vamp_detect_count_epochs: %d workgroups need two per CU, which only the "
                "bf16x3 engine runs (gemm = AMP_GEMM_F32 holds at most %d epochs)", P.nwg, ncu / P.wpe);
    AMP_REQUIRE(dec && dec->x && dec->sym && dec->idx && dec->counts,
                "amp_vamp_detect_count_epochs: null pointer argument");
    AMP_REQUIRE(dec->ibits_trunc >= 0 && dec->ibits_trunc < 64, "amp_vamp_detect_count_epochs: ibits_trunc");
    AMP_REQUIRE(d->Lin * d->Na * d->M == d->N, "amp_vamp_detect_count_epochs: inconsistent dims");
    hipStream_t st = (hipStream_t)stream;
    rc = vamp_persist_prepare(P, a, st, &ch);
    if (rc) return rc;
    P.dec_on = 1;
    P.ibits = dec->ibits_trunc;
    P.xtrue = (const float2*)dec->x;
    P.sym = (const long long*)dec->sym;
    P.idx = (const long long*)dec->idx;
    P.counts = (amp_counts*)dec->counts;
    P.host_rec = P.fold_in ? (unsigned char*)dec->host_record : nullptr;
    return vamp_persist_launch(P, c64, to_decconst(c), st, ncu);
}

int amp_vamp_detect_count_epochs(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                 const amp_vamp_decide_args* dec, int32_t epochs, void* stream) {
    return detect_count_epochs_impl(d, c, a, dec, epochs, EpochChannels{}, stream);
}

int amp_vamp_detect_count_epochs_ch(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                    const amp_vamp_decide_args* dec, int32_t epochs, int64_t U_stride,
                                    int64_t s_stride, int64_t Vh_stride, void* stream) {
    AMP_REQUIRE(U_stride >= 0 && s_stride >= 0 && Vh_stride >= 0, "amp_vamp_detect_count_epochs_ch: negative stride");
    EpochChannels ch;
    ch.U = U_stride; ch.s = s_stride; ch.Vh = Vh_stride;
    return detect_count_epochs_impl(d, c, a, dec, epochs, ch, stream);
}

// ---- one batch's trials over several persistent grids (SURVEY §8(e) exact-compat mode) ----
// The shared exchange buffer: barrier words, the rare path's float64 words and the per-iteration
// granule pairs of every workgroup of the batch (the same carve on every rank).
struct ShardX {
    unsigned* pbar;
    double* pxch;
    Partial* pparts;
    size_t bytes;
};
static ShardX shard_carve(void* base, int nwx, int max_iter) {
    Carve cv(base);
    ShardX x;
    x.pbar = cv.take<unsigned>(PBAR_WORDS);
    x.pxch = cv.take<double>((size_t)max_iter * nwx * 4);
    x.pparts = cv.take<Partial>((size_t)max_iter * nwx);
    x.bytes = cv.off;
    return x;
}

size_t amp_vamp_shard_xbuf_bytes(int32_t B_global, int32_t max_iter) {
    if (B_global <= 0 || max_iter <= 0) return 0;
    return shard_carve(nullptr, cdiv(B_global, PBM), max_iter).bytes;
}

int amp_vamp_shard_reset(void* xbuf, void* stream) {
    AMP_REQUIRE(xbuf, "amp_vamp_shard_reset: null buffer");
    shard_forget(xbuf);   // the next forward's shards claim their CU ranges afresh
    const hipError_t e = hipMemsetAsync(xbuf, 0, PBAR_WORDS * sizeof(unsigned), (hipStream_t)stream);
    AMP_REQUIRE(e == hipSuccess, "amp_vamp_shard_reset: %s", hipGetErrorString(e));
    return AMP_OK;
}

int amp_vamp_detect_count_shard(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                const amp_vamp_decide_args* dec, const amp_vamp_shard* sh, void* stream) {
    AMP_REQUIRE(d && sh && sh->xbuf && a, "amp_vamp_detect_count_shard: null argument");
    // Co-residency by construction: every shard's grid spins on its partners' partials,
    // so all of them must be resident at once.  Two plain streams may share one hardware queue (there
    // are GPU_MAX_HW_QUEUES = 4 per process), and then the second grid's dispatch waits behind the
    // first grid's spin until its bounded wait aborts (gpurun r5c7; tools/shard_queue_probe.py).  So
    // a shard runs only on a stream of amp_stream_create_cu_range (its own queue and CUs), its
    // workgroups must fit that CU range, and the ranges of one generation's shards must not overlap.
    hipStream_t st = (hipStream_t)stream;
    const bool any_stream = diag_env("AMP_SHARD_ANY_STREAM") != nullptr;   // (the probe's diagnostic build only)
    int cu0 = 0, cu1 = 0;
    if (!any_stream) {
        AMP_REQUIRE(cu_range_of(st, &cu0, &cu1),
                    "amp_vamp_detect_count_shard: the stream must come from amp_stream_create_cu_range (plain streams "
                    "may share a hardware queue, and a shard's grid would then wait behind its partner's spin)");
        AMP_REQUIRE(d->B > 0 && (long)cdiv(d->B, PBM) <= (long)vamp_persist_wg_per_cu(d, a->k, a->gemm) * (cu1 - cu0),
                    "amp_vamp_detect_count_shard: %d workgroups do not fit the stream's CUs [%d, %d)", cdiv(d->B, PBM),
                    cu0, cu1);
    }
    AMP_REQUIRE(sh->row_offset >= 0 && sh->row_offset % PBM == 0 && sh->row_offset + d->B <= sh->B_global &&
                    (d->B % PBM == 0 || sh->row_offset + d->B == sh->B_global),
                "amp_vamp_detect_count_shard: rows [%d, %d) of %d (a shard starts at a multiple of %d trials and "
                "only the last may end off it)", sh->row_offset, sh->row_offset + d->B, sh->B_global, PBM);
    const int ncu = device_cu_count();
    AMP_REQUIRE(a && a->engine != AMP_ENGINE_LAUNCHES && vamp_persist_eligible(d, a->k, ncu, 1, a->gemm),
                "amp_vamp_detect_count_shard: needs the persistent engine for this shard's shape");
    AMP_REQUIRE(dec && dec->x && dec->sym && dec->idx && dec->counts, "amp_vamp_detect_count_shard: null pointer argument");
    AMP_REQUIRE(dec->ibits_trunc >= 0 && dec->ibits_trunc < 64, "amp_vamp_detect_count_shard: ibits_trunc");
    AMP_REQUIRE(d->Lin * d->Na * d->M == d->N, "amp_vamp_detect_count_shard: inconsistent dims");
    const int nwx = cdiv(sh->B_global, PBM);
    const ShardX x = shard_carve(sh->xbuf, nwx, a->max_iter);
    AMP_REQUIRE(sh->xbuf_bytes >= x.bytes, "amp_vamp_detect_count_shard: exchange buffer %zu < %zu bytes",
                sh->xbuf_bytes, x.bytes);
    AMP_REQUIRE(any_stream || shard_claim_range(sh->xbuf, sh->gen, cu0, cu1),
                "amp_vamp_detect_count_shard: CUs [%d, %d) overlap another shard of generation %u on this exchange "
                "buffer (the shards' grids must be co-resident: disjoint CU ranges)", cu0, cu1, sh->gen);
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);     // this shard's rows: workspace, operators, y~
    if (rc) return rc;
    rc = vamp_persist_prepare(P, a, st);
    if (rc) return rc;
    // the batch's exchange: this grid's workgroups at their global index, the batch's size for
    // var.mean() (vamp.py:85), the shared generation for the granule tags
    P.wg_off = sh->row_offset / PBM;
    P.nwg_x = nwx;
    P.wpe = nwx;
    P.E = 1;
    P.row_off = sh->row_offset;
    P.B = sh->B_global;
    P.Bmean = sh->B_global;
    P.pbar = x.pbar;
    P.pxch = x.pxch;
    P.pparts = x.pparts;
    P.gen = sh->gen;
    P.dec_on = 1;
    P.ibits = dec->ibits_trunc;
    P.xtrue = (const float2*)dec->x;
    P.sym = (const long long*)dec->sym;
    P.idx = (const long long*)dec->idx;
    P.counts = (amp_counts*)dec->counts;
    P.host_rec = P.fold_in ? (unsigned char*)dec->host_record : nullptr;
    return vamp_persist_launch(P, c64, to_decconst(c), st, ncu);
}

// Measurement helper (bench.py): one full forward with hipEvents between the launches on
// `stream`; ms_out[0..3] = average vamp_k1, vamp_k2, vamp_r duration per executed iteration,
// and the whole forward.  Synchronises the stream (not for use inside a timed region).
int amp_vamp_profile(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, float* ms_out,
                     void* stream) {
    VampK P;
    Const64 c64;
    int rc = vamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(ms_out, "amp_vamp_profile: null output");
    hipStream_t st = (hipStream_t)stream;
    const int ncu = device_cu_count();
    if (a->engine == AMP_ENGINE_PERSISTENT || (a->engine == AMP_ENGINE_AUTO && vamp_persist_eligible(d, a->k, ncu))) {
        // persistent engine: [0] prepare (weights + y~ GEMM), [1] the vamp_persist launch,
        // [2] 0, [3] the whole forward
        hipEvent_t e0, e1, e2;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&e2);
        (void)hipEventRecord(e0, st);
        rc = vamp_persist_prepare(P, a, st);
        (void)hipEventRecord(e1, st);
        if (!rc) rc = vamp_persist_launch(P, c64, DecConst{}, st, ncu);
        (void)hipEventRecord(e2, st);
        (void)hipStreamSynchronize(st);
        float m01 = 0.f, m12 = 0.f;
        (void)hipEventElapsedTime(&m01, e0, e1);
        (void)hipEventElapsedTime(&m12, e1, e2);
        ms_out[0] = m01; ms_out[1] = m12; ms_out[2] = 0.f; ms_out[3] = m01 + m12;
        (void)hipEventDestroy(e0); (void)hipEventDestroy(e1); (void)hipEventDestroy(e2);
        return rc;
    }
    const int n = P.max_iter;
    std::vector<hipEvent_t> ev(3 * n + 2);
    for (auto& e : ev) (void)hipEventCreate(&e);
    (void)hipEventRecord(ev[0], st);
    rc = vamp_prepare_impl(P, a, st);
    dim3 g1(cdiv(P.B, GBM), P.ncp1 / 128);
    for (int t = 0; t < n && !rc; ++t) {
        (void)hipEventRecord(ev[1 + 3 * t], st);
        hipLaunchKernelGGL(vamp_k1, g1, dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, P, t);
        (void)hipEventRecord(ev[2 + 3 * t], st);
        launch_k2(P, t, st);
        (void)hipEventRecord(ev[3 + 3 * t], st);
        hipLaunchKernelGGL(vamp_r, dim3(1), dim3(RWG), 0, st, P, c64, t);
    }
    if (!rc) rc = vamp_finalize_impl(P, st);
    (void)hipEventRecord(ev[3 * n + 1], st);
    (void)hipStreamSynchronize(st);
    amp_status s;
    (void)hipMemcpy(&s, P.status, sizeof(s), hipMemcpyDeviceToHost);
    const int T = s.T > 0 ? s.T : n;
    float k1 = 0.f, k2 = 0.f, rr = 0.f, ms = 0.f;
    for (int t = 0; t < T; ++t) {
        (void)(void)hipEventElapsedTime(&ms, ev[1 + 3 * t], ev[2 + 3 * t]); k1 += ms;
        (void)hipEventElapsedTime(&ms, ev[2 + 3 * t], ev[3 + 3 * t]); k2 += ms;
        (void)hipEventElapsedTime(&ms, ev[3 + 3 * t], t + 1 < n ? ev[1 + 3 * (t + 1)] : ev[3 * n + 1]); rr += ms;
    }
    (void)hipEventElapsedTime(&ms, ev[0], ev[3 * n + 1]);
    ms_out[0] = k1 / T; ms_out[1] = k2 / T; ms_out[2] = rr / T; ms_out[3] = ms;
    for (auto& e : ev) (void)hipEventDestroy(e);
    AMP_LAUNCH_CHECK("amp_vamp_profile");
    return rc;
}

}  // extern "C"
