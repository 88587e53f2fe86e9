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
#include "amp_host.h"

namespace amp {

struct DecConst {
    int K, sbits;
    double re[AMP_MAX_K], im[AMP_MAX_K];
    float re32[AMP_MAX_K], im32[AMP_MAX_K];   // complex64 casts of the points (xhat values)
    int gray[AMP_MAX_K];
};

struct alignas(16) DecPart {
    long long ier, ser, iber, sber;
    double mse, msef, msem, mseL;
};

struct DecK {
    int B, L, M, Na, Lin, S;
    int ibits;
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
    DecConst c;
};

__device__ __forceinline__ bool dec_better(double v, int i, bool n, double bv, int bi, bool bn) {
    // does candidate (v, i, n) beat the incumbent (bv, bi, bn)?  NaN first, then larger value,
    // then smaller flat index (np.argmax: first occurrence of the maximum; NaN counts as maximum)
    if (n) return !bn || i < bi;
    if (bn) return false;
    return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(AMP_WG) void map_decide_kernel(DecK P) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M = P.M, K = P.c.K;
    const int G = M < 64 ? M : 64, PPL = M / G, gpw = 64 / G;
    const int gid = lane / G, g = lane - gid * G;
    long long ier = 0, ser = 0, iber = 0, sber = 0;
    double mse = 0, msef = 0, msem = 0, mseL = 0;
    const long long ibmask = (P.ibits >= 63) ? -1LL : ((1LL << P.ibits) - 1);
    const long long sbmask = (1LL << P.c.sbits) - 1;
    const int stride = gridDim.x * (AMP_WG / 64) * gpw;
    for (int base = (blockIdx.x * (AMP_WG / 64) + wave) * gpw; base < P.S; base += stride) {
        const int s = base + gid;
        const bool act = s < P.S;
        const int ss = act ? s : P.S - 1;
        double bv = -INFINITY;
        int bi = 0x7fffffff;
        bool bn = false;
        for (int p = 0; p < PPL; ++p) {
            const int m = g + p * G;
            const float2 xv = P.xmap[(size_t)ss * M + m];
            const double xr = (double)xv.x, xi = (double)xv.y;
            for (int k = 0; k < K; ++k) {
                const double v = __fma_rn(xr, P.c.re[k], __dmul_rn(xi, P.c.im[k]));
                const bool vn = v != v;
                const int f = m * K + k;
                if (dec_better(v, f, vn, bv, bi, bn)) { bv = v; bi = f; bn = vn; }
            }
        }
        for (int o = G >> 1; o > 0; o >>= 1) {
            const double ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            const bool on = __shfl_xor((int)bn, o, 64) != 0;
            if (dec_better(ov, oi, on, bv, bi, bn)) { bv = ov; bi = oi; bn = on; }
        }
        const int mh = bi / K, kh = bi - mh * K;
        // xhat vs x over the section (loss.py:133 count_nonzero(xhat - x)), and the nMSE sum on xmmse
        int mm = 0;
        double se = 0.0;
        for (int p = 0; p < PPL; ++p) {
            const int m = g + p * G;
            const size_t o = (size_t)ss * M + m;
            const float2 xv = P.x[o];
            const float hr = (m == mh) ? P.c.re32[kh] : 0.f, hi = (m == mh) ? P.c.im32[kh] : 0.f;
            mm |= (hr - xv.x != 0.f || hi - xv.y != 0.f) ? 1 : 0;
            const float2 e = P.xmmse[o];
            const float dr = e.x - xv.x, di = e.y - xv.y;
            se += (double)dr * dr + (double)di * di;
        }
        for (int o = G >> 1; o > 0; o >>= 1) {
            mm |= __shfl_xor(mm, o, 64);
            se += __shfl_xor(se, o, 64);
        }
        if (act && g == 0) {
            P.mism[s] = (unsigned char)mm;
            if (P.dec) P.dec[s] = bi;
            const long long ih = (long long)s * M + mh;           // flat index of the chosen entry
            const long long it = P.idx[s];
            const long long sh = P.c.gray[kh];
            const long long st = P.sym[s];
            ier += (ih != it);
            ser += (sh != st);
            iber += __popcll((unsigned long long)((ih ^ it) & ibmask));
            sber += __popcll((unsigned long long)((sh ^ st) & sbmask));
            const int lin = (s % P.L) / P.Na;
            mse += se;
            if (lin == 0) msef += se;
            if (lin == P.Lin / 2) msem += se;
            if (lin == P.Lin - 1) mseL += se;
        }
    }
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

int amp_map_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap, const void* xmmse,
                         const void* x, const void* sym, const void* idx, int32_t ibits_trunc, void* counts,
                         void* decisions, void* ws, size_t ws_bytes, void* stream) {
    int rc = check_dims(d, c, false);
    if (rc) return rc;
    AMP_REQUIRE(xmap && xmmse && x && sym && idx && counts && ws, "amp_map_decide_count: null pointer argument");
    AMP_REQUIRE(ws_bytes >= amp_map_decide_workspace_bytes(d), "amp_map_decide_count: workspace too small");
    AMP_REQUIRE(ibits_trunc >= 0 && ibits_trunc < 64, "amp_map_decide_count: ibits_trunc out of range");
    DecK P;
    P.B = d->B; P.L = d->L; P.M = d->M; P.Na = d->Na; P.Lin = d->Lin; P.S = d->B * d->L;
    P.ibits = ibits_trunc;
    P.xmap = (const float2*)xmap; P.xmmse = (const float2*)xmmse; P.x = (const float2*)x;
    P.sym = (const long long*)sym; P.idx = (const long long*)idx;
    Carve cv(ws);
    P.mism = cv.take<unsigned char>((size_t)P.S);
    P.nblk = decide_nblk(d);
    P.parts = cv.take<DecPart>((size_t)P.nblk);
    P.out = (amp_counts*)counts;
    P.dec = (int*)decisions;
    P.c.K = c->K;
    P.c.sbits = c->symbol_bits;
    for (int i = 0; i < AMP_MAX_K; ++i) {
        const bool v = i < c->K;
        P.c.re[i] = v ? c->re64[i] : 0.0;
        P.c.im[i] = v ? c->im64[i] : 0.0;
        P.c.re32[i] = v ? (float)c->re64[i] : 0.f;
        P.c.im32[i] = v ? (float)c->im64[i] : 0.f;
        P.c.gray[i] = v ? c->gray[i] : 0;
    }
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(map_decide_kernel, dim3(P.nblk), dim3(AMP_WG), 0, st, P);
    AMP_LAUNCH_CHECK("map_decide");
    hipLaunchKernelGGL(map_count_kernel, dim3(1), dim3(1024), 0, st, P);
    AMP_LAUNCH_CHECK("map_count");
    return AMP_OK;
}

}  // extern "C"
