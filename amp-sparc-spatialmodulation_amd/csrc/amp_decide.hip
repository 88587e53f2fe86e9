// amp_decide.hip — MAP hard decision + error counters on the GPU.
//
// Restates Loss.error_rate (loss.py:67-103) for generator_mode='sparc':
//   MAP_decision (loss.py:282-302): per section of M entries, argmax over the flattened
//     (m, k) grid of Re(x_m conj(a_k)) in float64.  The value is formed exactly as numpy's
//     complex multiply forms it (measured: fma(xr, ar, xi*ai)), first index wins ties,
//     an all/partly-NaN section picks its first NaN (np.argmax semantics).
//   mean_square_error / vector_error_rate / frame_error_rate / bit_error_rate
//     (loss.py:105-179) as integer counters and float64 sums.
// Kernel 1 (grid): one lane group per section -> decision, per-section mismatch byte,
//   per-workgroup partial counters.  Kernel 2 (one workgroup): deterministic sums and the
//   channel-use / trial "any mismatch" reductions.
#include <algorithm>

#include "amp_common.h"
#include "amp_decide.h"
#include "amp_host.h"

namespace amp {

constexpr int AMP_DEC_MAX_NA = 64;

struct DecK {
    int B, L, M, Na, Lin, S;
    int ibits;
    long long s_off;    // section offset of these rows in the whole batch (trial-sharded decision)
    const float2* xmap;
    const float2* xmmse;
    const float2* x;
    const long long* sym;
    const long long* idx;
    unsigned char* mism;
    int* dec;
    DecPart* parts;
    int nblk;
    amp_counts* out;
    int rule;            // 0: MAP (sparc), 1: segmented, 2: random
    DecConst c;
};

template <int KK, int G>
__global__ __launch_bounds__(AMP_WG) void map_decide_kernel(DecK P) {
    // one section per group of G = min(M, 64) lanes (coalesced loads of consecutive positions)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M = P.M;
    constexpr int gpw = 64 / G;
    const int gid = lane / G, g = lane % G;
    DecPart q = decpart_zero();
    const long long ibmask = dec_ibmask(P.ibits);
    const int stride = gridDim.x * (AMP_WG / 64) * gpw;
    for (int base = (blockIdx.x * (AMP_WG / 64) + wave) * gpw; base < P.S; base += stride) {   // wave-uniform
        const int s = base + gid;
        const bool act = s < P.S;
        const size_t o0 = (size_t)(act ? s : P.S - 1) * M;
        auto ld = [&](int m, float2& xv, float2& xt, float2& xe) {
            xv = P.xmap[o0 + m]; xt = P.x[o0 + m]; xe = P.xmmse[o0 + m];
        };
        int bi, mm;
        double se;
        if (P.rule == 1)
            decide_section_seg<KK, G>(P.c, M, g, ld, bi, mm, se);
        else
            decide_section<KK, G, false>(P.c, M, g, ld, bi, mm, se);
        if (act && g == 0) {
            P.mism[s] = (unsigned char)mm;
            if (P.dec) P.dec[s] = bi;
            count_section<KK>(P.c, s + P.s_off, M, P.L, P.Na, P.Lin, bi, se, P.sym[s], P.idx[s], ibmask, q);
        }
    }
    long long ier = q.ier, ser = q.ser, iber = q.iber, sber = q.sber;
    double mse = q.mse, msef = q.msef, msem = q.msem, mseL = q.mseL;
    // workgroup reduction (fixed order)
    ier = group_sum(ier, 64); ser = group_sum(ser, 64); iber = group_sum(iber, 64); sber = group_sum(sber, 64);
    mse = group_sum(mse, 64); msef = group_sum(msef, 64); msem = group_sum(msem, 64); mseL = group_sum(mseL, 64);
    __shared__ DecPart sp[AMP_WG / 64];
    if (lane == 0) sp[wave] = DecPart{ier, ser, iber, sber, mse, msef, msem, mseL};
    __syncthreads();
    if (threadIdx.x == 0) {
        DecPart o = sp[0];
        for (int w = 1; w < AMP_WG / 64; ++w) {
            o.ier += sp[w].ier; o.ser += sp[w].ser; o.iber += sp[w].iber; o.sber += sp[w].sber;
            o.mse += sp[w].mse; o.msef += sp[w].msef; o.msem += sp[w].msem; o.mseL += sp[w].mseL;
        }
        P.parts[blockIdx.x] = o;
    }
}


// Random decision (Loss.random_decision, loss.py:252-280; generator_mode='random'): per channel
// use (row of Nt), the Na largest |x_m| (np.argsort()[-Na:]: NaN largest; exact ties in an
// implementation-defined order in numpy, by larger index here), each decided to its nearest
// point (float64, first minimum); the decided positions in ascending order are compared with
// the true sorted indices / labels of that row (loss.py:165-178).  One thread per row: the
// reference runs this only for B = 1 (its reshape drops the batch axis).
__device__ __forceinline__ bool rnd_greater(bool n1, float v1, int m1, bool n2, float v2, int m2) {
    if (n1 != n2) return n1;
    if (n1) return m1 > m2;
    if (v1 != v2) return v1 > v2;
    return m1 > m2;
}

template <int KK>
__global__ __launch_bounds__(AMP_WG) void random_decide_kernel(DecK P, int Nt, int R) {
    constexpr int K = KK;
    constexpr int KU = KUnroll<KK>::value;
    DecPart q = decpart_zero();
    const long long ibmask = dec_ibmask(P.ibits);
    const long long sbmask = (1LL << P.c.sbits) - 1;
    for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < R; row += gridDim.x * blockDim.x) {
        const float2* xm = P.xmap + (size_t)row * Nt;
        const float2* xt = P.x + (size_t)row * Nt;
        const float2* xe = P.xmmse + (size_t)row * Nt;
        int pos[AMP_DEC_MAX_NA];
        bool pn = true;
        float pv = 0.f;
        int pm = 0x7fffffff;
        for (int a = 0; a < P.Na; ++a) {
            bool bn = false;
            float bv = -1.f;
            int bm = -1;
            for (int m = 0; m < Nt; ++m) {
                const float v = hypotf(xm[m].x, xm[m].y);
                const bool vn = v != v;
                if (!rnd_greater(pn, pv, pm, vn, v, m)) continue;     // already chosen
                if (bm < 0 || rnd_greater(vn, v, m, bn, bv, bm)) { bn = vn; bv = v; bm = m; }
            }
            pos[a] = bm;
            pn = bn; pv = bv; pm = bm;
        }
        for (int a = 1; a < P.Na; ++a)                                   // ascending positions
            for (int j = a; j > 0 && pos[j - 1] > pos[j]; --j) { const int t = pos[j]; pos[j] = pos[j - 1]; pos[j - 1] = t; }
        const int lin = row % P.Lin;
        int mism = 0;
        double se = 0.0;
        for (int j = 0; j < P.Na; ++j) {
            const int m = pos[j];
            const double xr = (double)xm[m].x, xi = (double)xm[m].y;
            double d = INFINITY;
            int kh = 0;
#pragma unroll KU
            for (int k = 0; k < K; ++k) {
                const double ds = hypot(xr - P.c.re[k], xi - P.c.im[k]);
                if (ds < d) { d = ds; kh = k; }
            }
            pos[j] = m * K + kh;
            const long long e = (long long)row * P.Na + j;
            const long long ih = (long long)row * Nt + m;
            long long sh = 0;
#pragma unroll KU
            for (int k = 0; k < K; ++k)
                if (k == kh) sh = P.c.gray[k];
            q.ier += (ih != P.idx[e]);
            q.ser += (sh != P.sym[e]);
            q.iber += __popcll((unsigned long long)((ih ^ P.idx[e]) & ibmask));
            q.sber += __popcll((unsigned long long)((sh ^ P.sym[e]) & sbmask));
            if (P.dec) P.dec[e] = pos[j];
        }
        for (int m = 0; m < Nt; ++m) {
            float hr = 0.f, hi = 0.f;
            for (int j = 0; j < P.Na; ++j)
                if (pos[j] / K == m) {
                    const int kh = pos[j] - m * K;
#pragma unroll KU
                    for (int k = 0; k < K; ++k)
                        if (k == kh) { hr = P.c.re32[k]; hi = P.c.im32[k]; }
                }
            mism |= (hr - xt[m].x != 0.f || hi - xt[m].y != 0.f) ? 1 : 0;
            const float dr = xe[m].x - xt[m].x, di = xe[m].y - xt[m].y;
            se += (double)dr * dr + (double)di * di;
        }
        // one mismatch flag per channel use, in the layout map_count_kernel folds
        unsigned char* mrow = P.mism + (size_t)(row / P.Lin) * P.L + (size_t)lin * P.Na;
        for (int a = 0; a < P.Na; ++a) mrow[a] = (a == 0) ? (unsigned char)mism : 0;
        q.mse += se;
        if (lin == 0) q.msef += se;
        if (lin == P.Lin / 2) q.msem += se;
        if (lin == P.Lin - 1) q.mseL += se;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    q.ier = group_sum(q.ier, 64); q.ser = group_sum(q.ser, 64); q.iber = group_sum(q.iber, 64);
    q.sber = group_sum(q.sber, 64);
    q.mse = group_sum(q.mse, 64); q.msef = group_sum(q.msef, 64); q.msem = group_sum(q.msem, 64);
    q.mseL = group_sum(q.mseL, 64);
    __shared__ DecPart sp[AMP_WG / 64];
    if (lane == 0) sp[wave] = q;
    __syncthreads();
    if (threadIdx.x == 0) {
        DecPart o = sp[0];
        for (int w = 1; w < AMP_WG / 64; ++w) decpart_add(o, sp[w]);
        P.parts[blockIdx.x] = o;
    }
}

__global__ __launch_bounds__(1024) void map_count_kernel(DecK P) {
    // channel-use / trial "any mismatch" counts (loss.py:133-136, 150) ...
    long long ver = 0, verf = 0, verm = 0, verL = 0, fer = 0;
    for (int b = threadIdx.x; b < P.B; b += blockDim.x) {
        int trial = 0;
        for (int lin = 0; lin < P.Lin; ++lin) {
            int cu = 0;
            const unsigned char* m = P.mism + (size_t)b * P.L + (size_t)lin * P.Na;
            for (int a = 0; a < P.Na; ++a) cu |= m[a];
            ver += cu;
            if (lin == 0) verf += cu;
            if (lin == P.Lin / 2) verm += cu;
            if (lin == P.Lin - 1) verL += cu;
            trial |= cu;
        }
        fer += trial;
    }
    // ... and the per-workgroup partials of map_decide_kernel, folded in a fixed order
    DecPart t = DecPart{0, 0, 0, 0, 0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < P.nblk; i += blockDim.x) {
        const DecPart q = P.parts[i];
        t.ier += q.ier; t.ser += q.ser; t.iber += q.iber; t.sber += q.sber;
        t.mse += q.mse; t.msef += q.msef; t.msem += q.msem; t.mseL += q.mseL;
    }
    ver = group_sum(ver, 64); verf = group_sum(verf, 64); verm = group_sum(verm, 64); verL = group_sum(verL, 64);
    fer = group_sum(fer, 64);
    t.ier = group_sum(t.ier, 64); t.ser = group_sum(t.ser, 64); t.iber = group_sum(t.iber, 64);
    t.sber = group_sum(t.sber, 64);
    t.mse = group_sum(t.mse, 64); t.msef = group_sum(t.msef, 64); t.msem = group_sum(t.msem, 64);
    t.mseL = group_sum(t.mseL, 64);
    __shared__ long long sc[16][5];
    __shared__ DecPart sp[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        sc[wave][0] = ver; sc[wave][1] = verf; sc[wave][2] = verm; sc[wave][3] = verL; sc[wave][4] = fer;
        sp[wave] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        amp_counts c;
        c.ver = c.verf = c.verm = c.verL = c.fer = 0;
        c.ier = c.ser = c.iber = c.sber = 0;
        c.mse = c.msef = c.msem = c.mseL = 0.0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) {
            c.ver += sc[w][0]; c.verf += sc[w][1]; c.verm += sc[w][2]; c.verL += sc[w][3]; c.fer += sc[w][4];
            c.ier += sp[w].ier; c.ser += sp[w].ser; c.iber += sp[w].iber; c.sber += sp[w].sber;
            c.mse += sp[w].mse; c.msef += sp[w].msef; c.msem += sp[w].msem; c.mseL += sp[w].mseL;
        }
        *P.out = c;
    }
}

static int decide_nblk(const amp_dims* d) {
    const int G = d->M < 64 ? d->M : 64;
    const int per = (AMP_WG / 64) * (64 / G);
    return std::max(1, std::min(cdiv(d->B * d->L, per), 2048));
}

template <int KK>
static void launch_decide_k(const DecK& P, int M, hipStream_t st) {
    const dim3 g(P.nblk), b(AMP_WG);
    switch (M) {
    case 1: hipLaunchKernelGGL((map_decide_kernel<KK, 1>), g, b, 0, st, P); break;
    case 2: hipLaunchKernelGGL((map_decide_kernel<KK, 2>), g, b, 0, st, P); break;
    case 4: hipLaunchKernelGGL((map_decide_kernel<KK, 4>), g, b, 0, st, P); break;
    case 8: hipLaunchKernelGGL((map_decide_kernel<KK, 8>), g, b, 0, st, P); break;
    case 16: hipLaunchKernelGGL((map_decide_kernel<KK, 16>), g, b, 0, st, P); break;
    case 32: hipLaunchKernelGGL((map_decide_kernel<KK, 32>), g, b, 0, st, P); break;
    default: hipLaunchKernelGGL((map_decide_kernel<KK, 64>), g, b, 0, st, P); break;   // M >= 64 (power of 2)
    }
}

static void launch_decide(const DecK& P, int M, hipStream_t st) {
    switch (P.c.K) {
    case 1: launch_decide_k<1>(P, M, st); break;
    case 2: launch_decide_k<2>(P, M, st); break;
    case 4: launch_decide_k<4>(P, M, st); break;
    case 8: launch_decide_k<8>(P, M, st); break;
    case 16: launch_decide_k<16>(P, M, st); break;
    default: launch_decide_k<64>(P, M, st); break;     // check_dims: K in {1, 2, 4, 8, 16, 64}
    }
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_map_decide_workspace_bytes(const amp_dims* d) {
    if (!d) return 0;
    Carve cv(nullptr);
    cv.take<unsigned char>((size_t)d->B * d->L);
    cv.take<DecPart>((size_t)decide_nblk(d));
    return cv.off;
}

static int decide_count(int rule, const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                        const void* x, const void* sym, const void* idx, int32_t ibits_trunc, void* counts,
                        void* decisions, void* ws, size_t ws_bytes, void* stream, long long row0 = 0) {
    int rc = check_dims(d, c, false);
    if (rc) return rc;
    AMP_REQUIRE(xmap && xmmse && x && sym && idx && counts && ws, "amp_map_decide_count: null pointer argument");
    AMP_REQUIRE(ws_bytes >= amp_map_decide_workspace_bytes(d), "amp_map_decide_count: workspace too small");
    AMP_REQUIRE(ibits_trunc >= 0 && ibits_trunc < 64, "amp_map_decide_count: ibits_trunc out of range");
    DecK P;
    P.B = d->B; P.L = d->L; P.M = d->M; P.Na = d->Na; P.Lin = d->Lin; P.S = d->B * d->L;
    P.ibits = ibits_trunc;
    P.s_off = row0 * d->L;
    P.xmap = (const float2*)xmap; P.xmmse = (const float2*)xmmse; P.x = (const float2*)x;
    P.sym = (const long long*)sym; P.idx = (const long long*)idx;
    Carve cv(ws);
    P.mism = cv.take<unsigned char>((size_t)P.S);
    P.nblk = decide_nblk(d);
    P.parts = cv.take<DecPart>((size_t)P.nblk);
    P.out = (amp_counts*)counts;
    P.dec = (int*)decisions;
    P.c = to_decconst(c);
    P.rule = rule;
    hipStream_t st = (hipStream_t)stream;
    launch_decide(P, d->M, st);
    AMP_LAUNCH_CHECK("map_decide");
    hipLaunchKernelGGL(map_count_kernel, dim3(1), dim3(1024), 0, st, P);
    AMP_LAUNCH_CHECK("map_count");
    return AMP_OK;
}

int amp_map_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                         const void* x, const void* sym, const void* idx, int32_t ibits_trunc, void* counts,
                         void* decisions, void* ws, size_t ws_bytes, void* stream) {
    return decide_count(0, d, c, xmap, xmmse, x, sym, idx, ibits_trunc, counts, decisions, ws, ws_bytes, stream);
}

int amp_map_decide_count_rows(const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                              const void* x, const void* sym, const void* idx, int32_t ibits_trunc, int64_t row0,
                              void* counts, void* decisions, void* ws, size_t ws_bytes, void* stream) {
    AMP_REQUIRE(row0 >= 0, "amp_map_decide_count_rows: row0 = %lld", (long long)row0);
    return decide_count(0, d, c, xmap, xmmse, x, sym, idx, ibits_trunc, counts, decisions, ws, ws_bytes, stream,
                        (long long)row0);
}

int amp_segmented_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                               const void* x, const void* sym, const void* idx, int32_t ibits_trunc, void* counts,
                               void* decisions, void* ws, size_t ws_bytes, void* stream) {
    return decide_count(1, d, c, xmap, xmmse, x, sym, idx, ibits_trunc, counts, decisions, ws, ws_bytes, stream);
}

int amp_random_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                            const void* x, const void* sym, const void* idx, int32_t ibits_trunc, void* counts,
                            void* decisions, void* ws, size_t ws_bytes, void* stream) {
    AMP_REQUIRE(d && c && d->B > 0 && d->Nt > 0 && d->Lin > 0 && d->Na >= 1 && d->Na <= AMP_DEC_MAX_NA &&
                    d->Na <= d->Nt && d->L == d->Na * d->Lin && c->K >= 1 && c->K <= AMP_MAX_K &&
                    is_pow2(c->K) && c->K != 32,
                "amp_random_decide_count: bad dims (Na <= %d)", AMP_DEC_MAX_NA);
    AMP_REQUIRE(xmap && xmmse && x && sym && idx && counts && ws, "amp_random_decide_count: null pointer argument");
    AMP_REQUIRE(ws_bytes >= amp_map_decide_workspace_bytes(d), "amp_random_decide_count: workspace too small");
    AMP_REQUIRE(ibits_trunc >= 0 && ibits_trunc < 64, "amp_random_decide_count: ibits_trunc out of range");
    DecK P;
    P.B = d->B; P.L = d->L; P.M = d->M; P.Na = d->Na; P.Lin = d->Lin; P.S = d->B * d->L;
    P.ibits = ibits_trunc;
    P.s_off = 0;
    P.xmap = (const float2*)xmap; P.xmmse = (const float2*)xmmse; P.x = (const float2*)x;
    P.sym = (const long long*)sym; P.idx = (const long long*)idx;
    Carve cv(ws);
    P.mism = cv.take<unsigned char>((size_t)P.S);
    const int R = d->B * d->Lin;
    P.nblk = std::max(1, std::min(cdiv(R, AMP_WG), decide_nblk(d)));
    P.parts = cv.take<DecPart>((size_t)decide_nblk(d));
    P.out = (amp_counts*)counts;
    P.dec = (int*)decisions;
    P.c = to_decconst(c);
    P.rule = 2;
    hipStream_t st = (hipStream_t)stream;
    const dim3 g(P.nblk), b(AMP_WG);
    switch (P.c.K) {
    case 1: hipLaunchKernelGGL(random_decide_kernel<1>, g, b, 0, st, P, d->Nt, R); break;
    case 2: hipLaunchKernelGGL(random_decide_kernel<2>, g, b, 0, st, P, d->Nt, R); break;
    case 4: hipLaunchKernelGGL(random_decide_kernel<4>, g, b, 0, st, P, d->Nt, R); break;
    case 8: hipLaunchKernelGGL(random_decide_kernel<8>, g, b, 0, st, P, d->Nt, R); break;
    case 16: hipLaunchKernelGGL(random_decide_kernel<16>, g, b, 0, st, P, d->Nt, R); break;
    default: hipLaunchKernelGGL(random_decide_kernel<64>, g, b, 0, st, P, d->Nt, R); break;
    }
    AMP_LAUNCH_CHECK("random_decide");
    hipLaunchKernelGGL(map_count_kernel, dim3(1), dim3(1024), 0, st, P);
    AMP_LAUNCH_CHECK("map_count");
    return AMP_OK;
}

}  // extern "C"
