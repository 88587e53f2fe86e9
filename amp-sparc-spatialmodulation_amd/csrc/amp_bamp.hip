// amp_bamp.hip — BAMP detector, device-resident iteration loop.
//
// Restates BAMP.forward (bamp.py:116-143) with its Tracker (bamp.py:12-25) and
// BAMPLayer.forward (bamp.py:48-64):
//   v = |H|^2 var ; z = H xmmse - v (y - z) / u ; u = v + sigma2 ;
//   cov = 1 / (|H|^2^T (1/u)) ; xmap = xmmse + cov (H^H ((y - z)/u)) ;
//   xmmse, var = denoiser(xmap, tau = cov/2)  (bamp.py:66-77)
// and the allclose(var) early exit (bamp.py:140).
// Per iteration: four fp32-MFMA GEMM launches with fused epilogues + one reduction /
// exact-float64 fix-up workgroup (same scheme as amp_vamp.hip).
#include <algorithm>
#include <mutex>

#include "amp_denoise.h"
#include "amp_gemm.h"
#include "amp_gemm_h2.h"
#include "amp_gemm_x3.h"
#include <vector>
#include <cstdio>
#include "amp_host.h"

namespace amp {

constexpr int BRWG = 1024;

// bamp_ka2's epilogue loads issued before the GEMM (A/B builds): measured slower, cfg5 64-QAM
// 18.24 -> 18.52 ms, ISI BAMP 0.1330 -> 0.1345 ms per iteration (same box, gpurun_out r5pf; the
// 48 registers they hold across the reduction cost more than the overlap gains)

struct alignas(16) BampIter {
    int32_t stopped, T, fixed, fixed_all;
    // exact float64 fix-up of iteration T-1 pending (set by bamp_r, done and settled by
    // bamp_fixall): the exact batch max |xi| G, the float32 estimate's slack, the allclose count
    // before the fix-up
    double G, slack;
    uint32_t notclose;
    int32_t active, pad[2];
};

struct BampK {
    int B, N, n, L, M, bn;
    int kapA1, ncpA1, kapA2, ncpA2, kapB1, ncpB1, kapB2, ncpB2;
    int nblk, max_iter;
    float sigma2;       // f32(noise_var): u = v + sigma2 (bamp.py:61)
    const float* Wabs2;    // [ncpA1][kapA1]   v = |H|^2 var
    const float* WH;       // [ncpA2][kapA2]   H xmmse
    const float* Wabs2T;   // [ncpB1][kapB1]   |H|^2^T (1/u)
    const float* WHH;      // [ncpB2][kapB2]   H^H s
    const float* y;        // [B][2n]
    float* v;              // [B][n]
    float* z;              // [B][2n]
    float* invu;           // [B][n]
    float* s;              // [B][2n]  (y - z)/u
    float* cov;            // [B][N]
    float* xmap;           // [B][2N]  caller
    float* xm;             // [B][2N]  caller
    float* var0;           // caller's var (even iterations)
    float* var1;           // workspace  (odd iterations)
    float* secmax;         // [B*L] per-section max logit (fast path)
    float* secabs;         // [B*L] per-section max |logit|
    Partial* parts;        // [max_iter][nblk]
    BampIter* iters;       // [max_iter + 1]
    amp_status* status;
    // block-banded H (Lin > 1 or Lout > 1): per column tile of Wabs2 / WH / Wabs2T / WHH the
    // reduction range holding its nonzero blocks (weight_kband), else null (whole range)
    const int* band[4];
    XState* xs;            // trial-sharded exchange words (amp_bamp_run_sharded)
    Const c;
    int elementwise;                       // random_denoiser (bamp.py:79-88) instead of the block one
    float P0, Ps;
    // fp16x2 GEMMs (amp_gemm_h2.h): the four operators h2-packed into the weight buffers above
    // (real |H|^2 two planes, complex H / H^H four), each GEMM's A rows split into `ap` first
    // bf16x3 GEMMs (amp_gemm_x3.h, x3 = 1): the same scheme with three bf16 pieces per value (real
    // |H|^2 three planes, complex H / H^H six; no exponents)
    int h2, x3, rows_pad;
    int tile_rows;         // row-block-major tile order (xcd_tile_rows: the fp16x2 tiles), else xcd_tile
    unsigned short* ap;    // [4 planes][rows_pad][max(N, n)] fp16, or [6 planes][...] bf16
    int* rexp;             // [rows_pad] row exponents
    // launch engine: rcnt[1] is bamp_fixall's arrival counter (zeroed by bamp_init_kernel)
    unsigned* rcnt;
};

// BAMP's fp16x2 operator scale exponent (the opt-in AMP_GEMM_H2 form): every operator piece is
// scaled by 2^10, so |H|^2 must stay below 64 (|H| < 8; the channel's entries are ~CN(0, 1/Nr));
// larger entries overflow their fp16 piece, the result is then non-finite (NaN detections,
// counted as errors), never silently wrong
constexpr int BH2_EX = 10;

// the fp16x2 GEMMs need whole 64-wide reduction groups and output tiles (a block-banded H reduces
// over each tile's h2_kband range)
static inline bool bamp_h2_shape(const amp_dims* d) {
    return d->N % 64 == 0 && d->n % 64 == 0;
}

// BAMPLayer.random_denoiser (bamp.py:79-88) for one entry, in the reference's dtypes: G(0) in
// float32 (r - 0 stays complex64), G(a_k) in float64 (complex64 - complex128), norm / exp / var
// in float64 (the float32 prior scalars promoted), complex128 / float64 as a reciprocal multiply.
// c64: torch.tensor(config.symbols), complex128 (bamp.py:37).
// KK: the table size as a compile-time bound (points k >= c64.K skipped): the loop is unrolled so
// the by-value kernel-argument table is only read at constant offsets (a runtime-indexed loop made
// the compiler copy the whole table into scratch memory at every kernel entry: ~900 B per lane).
template <int KK>
__device__ __forceinline__ void bamp_bayes_elem(const BampK& P, const Const64& c64, float rr, float ri, float cov,
                                                float& xr, float& xi, float& var) {
    const float a0 = hypotf(rr, ri);
    const float g0 = expf(-(a0 * a0) / cov);
    const double cd = (double)cov;
    double gs = 0.0, sr = 0.0, si = 0.0, s2 = 0.0;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
        if (k >= c64.K) break;
        const double a = hypot((double)rr - c64.re[k], (double)ri - c64.im[k]);
        const double g = exp(-(a * a) / cd);
        const double ak = hypot(c64.re[k], c64.im[k]);
        gs += g;
        sr += c64.re[k] * g;
        si += c64.im[k] * g;
        s2 += (ak * ak) * g;
    }
    double norm = (double)(P.P0 * g0) + (double)P.Ps * gs;
    if (norm == 0.0) norm = 1e-9;                                       // regularize_zero (bamp.py:90-92)
    const double rn = 1.0 / norm;
    const double er = ((double)P.Ps * sr) * rn, ei = ((double)P.Ps * si) * rn;
    const double ae = hypot(er, ei);
    xr = (float)er;
    xi = (float)ei;
    var = (float)(((double)P.Ps * s2) / norm - ae * ae);
}

struct BampWs {
    float *Wabs2, *WH, *Wabs2T, *WHH, *v, *z, *invu, *s, *cov, *var1;
    unsigned short* ap;
    int* rexp;
    int* band[4];
    XState* xs;
    float *secmax, *secabs;
    Partial* parts;
    BampIter* iters;
    unsigned* rcnt;
    size_t bytes;
};

static void bamp_geometry(const amp_dims* d, BampK& P) {
    P.B = d->B; P.N = d->N; P.n = d->n; P.L = d->L; P.M = d->M;
    P.bn = section_bn(d);
    P.kapA1 = round_up(d->N, GBK); P.ncpA1 = round_up(d->n, 128);
    P.kapA2 = round_up(2 * d->N, GBK); P.ncpA2 = round_up(2 * d->n, 128);
    P.kapB1 = round_up(d->n, GBK); P.ncpB1 = round_up(d->N, 128);
    P.kapB2 = round_up(2 * d->n, GBK); P.ncpB2 = round_up(2 * d->N, P.bn);
    P.nblk = cdiv(d->B, GBM) * (P.ncpB2 / P.bn);
}

static BampWs bamp_carve(const amp_dims* d, int max_iter, void* base) {
    BampK P;
    bamp_geometry(d, P);
    Carve cv(base);
    BampWs w;
    // the split forms' shapes also hold the bf16x3 real operators: three 16-bit planes, 1.5x the
    // f32 weight, over the padded outputs the last column tile streams
    const bool x3 = bamp_h2_shape(d);
    w.Wabs2 = cv.take<float>((size_t)P.ncpA1 * P.kapA1 * (x3 ? 3 : 2) / 2);
    w.WH = cv.take<float>((size_t)P.ncpA2 * P.kapA2);
    w.Wabs2T = cv.take<float>((size_t)P.ncpB1 * P.kapB1 * (x3 ? 3 : 2) / 2);
    w.WHH = cv.take<float>((size_t)P.ncpB2 * P.kapB2);
    w.v = cv.take<float>((size_t)d->B * d->n);
    w.z = cv.take<float>((size_t)d->B * 2 * d->n);
    w.invu = cv.take<float>((size_t)d->B * d->n);
    w.s = cv.take<float>((size_t)d->B * 2 * d->n);
    w.cov = cv.take<float>((size_t)d->B * d->N);
    w.var1 = cv.take<float>((size_t)d->B * d->N);
    w.secmax = cv.take<float>((size_t)d->B * d->L);
    w.secabs = cv.take<float>((size_t)d->B * d->L);
    w.parts = cv.take<Partial>((size_t)max_iter * P.nblk);
    w.iters = cv.take<BampIter>((size_t)max_iter + 1);
    w.band[0] = cv.take<int>((size_t)2 * (P.ncpA1 / 128));
    w.band[1] = cv.take<int>((size_t)2 * (P.ncpA2 / 128));
    w.band[2] = cv.take<int>((size_t)2 * (P.ncpB1 / 128));
    w.band[3] = cv.take<int>((size_t)2 * (P.ncpB2 / P.bn));
    w.xs = cv.take<XState>(1);
    w.rcnt = cv.take<unsigned>(16);
    w.ap = nullptr;
    w.rexp = nullptr;
    if (bamp_h2_shape(d)) {
        // the A planes of either split form (fp16x2: four, bf16x3: six)
        const size_t rp = (size_t)round_up(d->B, GBM);
        w.ap = cv.take<unsigned short>(6 * rp * std::max(d->N, d->n));
        w.rexp = cv.take<int>(rp);
    }
    w.bytes = cv.off;
    return w;
}

__device__ __forceinline__ float* bvar(const BampK& P, int t) { return (t & 1) ? P.var1 : P.var0; }
// reduction range of column tile cb of GEMM weight w (0..3: Wabs2, WH, Wabs2T, WHH); whole range
// when the channel is not block-banded
__device__ __forceinline__ int bkb(const BampK& P, int w, int cb) { return P.band[w] ? P.band[w][2 * cb] : 0; }
__device__ __forceinline__ int bke(const BampK& P, int w, int cb) { return P.band[w] ? P.band[w][2 * cb + 1] : -1; }

// KC: the A chunk of the f32 tile (GKC; 256 for the block-banded H, whose short reduction ranges
// need no longer chunks: 33 KB of LDS, four tiles per CU instead of two; the fp16x2 tile only in
// the GKC instantiations).  The chunking does not change the MFMA order: the same bits.
// v = |H|^2 var (bamp.py:59)
template <int KC = GKC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void bamp_ka1(BampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    const GemmTile tile = (KC == GKC && P.tile_rows) ? xcd_tile_rows() : xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * 128;
    if constexpr (X3)
        gemm_tile_x3<128, false>(P.ap, P.rows_pad, P.N, P.Wabs2, row0, col0, lds, bkb(P, 0, tile.cb), bke(P, 0, tile.cb));
    else if (KC == GKC && P.h2)
        gemm_tile_h2<128, false>(P.ap, P.rows_pad, P.rexp, P.N, P.Wabs2, BH2_EX, row0, col0, lds, bkb(P, 0, tile.cb),
                                       bke(P, 0, tile.cb));
    else
        gemm_tile<128, ALoadPlain, KC>(ALoadPlain{bvar(P, t + 1), P.N, P.B, P.N}, P.Wabs2, P.kapA1, row0, col0, lds,
                                       bkb(P, 0, tile.cb), bke(P, 0, tile.cb));
    using C = GemmCfg<128>;
    for (int e = threadIdx.x; e < GBM * 128; e += AMP_WG) {
        const int rho = e >> 7, cc = e & 127;
        const int row = row0 + rho, col = col0 + cc;
        if (row < P.B && col < P.n) P.v[(size_t)row * P.n + col] = lds[rho * C::LDC + cc];
    }
}

// z = H xmmse - v (y - z) / u ; u = v + sigma2 ; s = (y - z) / u   (bamp.py:60-63)
template <int KC = GKC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void bamp_ka2(BampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    const GemmTile tile = (KC == GKC && P.tile_rows) ? xcd_tile_rows() : xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * 128;
    const int twoN = 2 * P.N, twon = 2 * P.n;
    // every global load of this thread's epilogue elements before any store (the z / invu / s
    // stores may alias the next element's loads as far as the compiler knows: one memory latency
    // per element otherwise); each element reads and writes only its own z and invu (so the loads
    // may also go before the GEMM: measured slower, round 5)
    constexpr int IT = GBM * 64 / AMP_WG;
    float2 yv[IT], zv[IT];
    float vv[IT], iuo[IT];
    auto epi_loads = [&] {
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            // unconditional loads at a clamped index (a lane-divergent branch around them
            // serialises their latencies, amp_gemm.h ALoadPlain); out-of-range elements are never stored
            const int e = threadIdx.x + u * AMP_WG;
            const int rho = e >> 6, cp = e & 63;           // complex column pair
            const int row = min(row0 + rho, P.B - 1), i = min((col0 >> 1) + cp, P.n - 1);
            const size_t oc = (size_t)row * twon + 2 * i, o = (size_t)row * P.n + i;
            yv[u] = *reinterpret_cast<const float2*>(P.y + oc);
            zv[u] = *reinterpret_cast<const float2*>(P.z + oc);
            vv[u] = P.v[o];
            iuo[u] = P.invu[o];
        }
    };
    if constexpr (X3)
        gemm_tile_x3<128, true>(P.ap, P.rows_pad, P.N, P.WH, row0, col0, lds, bkb(P, 1, tile.cb), bke(P, 1, tile.cb));
    else if (KC == GKC && P.h2)
        gemm_tile_h2<128, true>(P.ap, P.rows_pad, P.rexp, P.N, P.WH, BH2_EX, row0, col0, lds, bkb(P, 1, tile.cb),
                                       bke(P, 1, tile.cb));
    else
        gemm_tile<128, ALoadPlain, KC>(ALoadPlain{P.xm, twoN, P.B, twoN}, P.WH, P.kapA2, row0, col0, lds,
                                       bkb(P, 1, tile.cb), bke(P, 1, tile.cb));
    using C = GemmCfg<128>;
    epi_loads();
#pragma unroll
    for (int u = 0; u < IT; ++u) {
        const int e = threadIdx.x + u * AMP_WG;
        const int rho = e >> 6, cp = e & 63;
        const int row = row0 + rho, i = (col0 >> 1) + cp;
        if (row < P.B && i < P.n) {
            const size_t oc = (size_t)row * twon + 2 * i, o = (size_t)row * P.n + i;
            const float hr = lds[rho * C::LDC + 2 * cp], hi = lds[rho * C::LDC + 2 * cp + 1];
            const float yr = yv[u].x, yi = yv[u].y;
            const float vi = vv[u], iu_old = iuo[u];
            const float zr = hr - (vi * (yr - zv[u].x)) * iu_old;
            const float zi = hi - (vi * (yi - zv[u].y)) * iu_old;
            const float uu = vi + P.sigma2;
            const float iu = 1.0f / uu;
            *reinterpret_cast<float2*>(P.z + oc) = make_float2(zr, zi);
            P.invu[o] = iu;
            *reinterpret_cast<float2*>(P.s + oc) = make_float2((yr - zr) * iu, (yi - zi) * iu);
        }
    }
}

// cov = 1 / (|H|^2^T (1/u))   (bamp.py:62)
template <int KC = GKC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void bamp_kb1(BampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    const GemmTile tile = (KC == GKC && P.tile_rows) ? xcd_tile_rows() : xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * 128;
    if constexpr (X3)
        gemm_tile_x3<128, false>(P.ap, P.rows_pad, P.n, P.Wabs2T, row0, col0, lds, bkb(P, 2, tile.cb), bke(P, 2, tile.cb));
    else if (KC == GKC && P.h2)
        gemm_tile_h2<128, false>(P.ap, P.rows_pad, P.rexp, P.n, P.Wabs2T, BH2_EX, row0, col0, lds, bkb(P, 2, tile.cb),
                                       bke(P, 2, tile.cb));
    else
        gemm_tile<128, ALoadPlain, KC>(ALoadPlain{P.invu, P.n, P.B, P.n}, P.Wabs2T, P.kapB1, row0, col0, lds,
                                       bkb(P, 2, tile.cb), bke(P, 2, tile.cb));
    using C = GemmCfg<128>;
    for (int e = threadIdx.x; e < GBM * 128; e += AMP_WG) {
        const int rho = e >> 7, cc = e & 127;
        const int row = row0 + rho, col = col0 + cc;
        if (row < P.B && col < P.N) P.cov[(size_t)row * P.N + col] = 1.0f / lds[rho * C::LDC + cc];
    }
}

struct BampDenoisePolicy {
    const float* tile;
    const float* itile;   // LDS [32][ldi]: 1 / (cov / 2) of the tile's positions (bamp_kb2's xmap pass)
    int ldc, ldi, spr, M, N, row0, colc0;
    float* xm;
    float* var_new;
    const float* var_prev;
    float* secmax;
    float* secabs;
    int L;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const float2 v = *reinterpret_cast<const float2*>(tile + rho * ldc + 2 * (sj * M + m));
        rr = v.x; ri = v.y;
        it = itile[rho * ldi + sj * M + m];   // 1 / tau, tau = cov / 2 (bamp.py:68)
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * N + colc0 + sj * M + m;
        *reinterpret_cast<float2*>(xm + 2 * o) = make_float2(xr, xi);
        var_new[o] = var;
        pa.sumvar += (double)var;
        pa.notclose += torch_close(var, var_prev[o]) ? 0u : 1u;     // bamp.py:140
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * L + (colc0 / M) + sj;
        secmax[o] = smax;
        secabs[o] = sabs;
    }
};

// xmap = xmmse + cov (H^H s) ; xmmse, var = denoiser(xmap, cov/2)   (bamp.py:63-64)
template <int BN, int KK, int KC = GKC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void bamp_kb2(BampK P, Const64 c64, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    using C = GemmCfg<BN, KC>;
    const GemmTile tile = (KC == GKC && P.tile_rows) ? xcd_tile_rows() : xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * BN;
    const int twoN = 2 * P.N, twon = 2 * P.n;
    if constexpr (X3)
        gemm_tile_x3<BN, true>(P.ap, P.rows_pad, P.n, P.WHH, row0, col0, lds, bkb(P, 3, tile.cb), bke(P, 3, tile.cb));
    else if (KC == GKC && P.h2)
        gemm_tile_h2<BN, true>(P.ap, P.rows_pad, P.rexp, P.n, P.WHH, BH2_EX, row0, col0, lds, bkb(P, 3, tile.cb),
                               bke(P, 3, tile.cb));
    else
        gemm_tile<BN, ALoadPlain, KC>(ALoadPlain{P.s, twon, P.B, twon}, P.WHH, P.kapB2, row0, col0, lds,
                                      bkb(P, 3, tile.cb), bke(P, 3, tile.cb));
    const int nrows = min(GBM, P.B - row0), ncols = min(BN, twoN - col0);
    float* sit = lds + C::CTILE_FLOATS + 2048;   // past the partial-store scratch
    {
        // the loads of this thread's elements before the xmap stores (which may alias them as far
        // as the compiler knows)
        constexpr int IT = GBM * BN / AMP_WG;
        static_assert(C::CTILE_FLOATS + 2048 + GBM * (BN / 2) <= C::A_FLOATS, "1 / tau tile");
        float xv[IT], cvv[IT];
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            // unconditional loads at a clamped index (see bamp_ka2); out-of-range elements unused
            const int e = threadIdx.x + u * AMP_WG, rho = min(e / BN, nrows - 1), cc = min(e % BN, ncols - 1);
            xv[u] = P.xm[(size_t)(row0 + rho) * twoN + col0 + cc];
            cvv[u] = P.cov[(size_t)(row0 + rho) * P.N + ((col0 + cc) >> 1)];
        }
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int e = threadIdx.x + u * AMP_WG, rho = e / BN, cc = e % BN;
            if (rho < nrows && cc < ncols) {
                const size_t o = (size_t)(row0 + rho) * twoN + col0 + cc;
                const float xp = xv[u] + cvv[u] * lds[rho * C::LDC + cc];
                P.xmap[o] = xp;
                lds[rho * C::LDC + cc] = xp;
                // the denoiser's 1 / tau of this position, read from LDS there instead of a global
                // load per position inside its loop (the same float32 operations)
                if ((cc & 1) == 0) sit[rho * (BN / 2) + (cc >> 1)] = 1.0f / (cvv[u] * 0.5f);
            }
        }
    }
    __syncthreads();
    BampDenoisePolicy pol;
    pol.tile = lds; pol.itile = sit; pol.ldi = BN / 2; pol.ldc = C::LDC; pol.M = P.M; pol.N = P.N; pol.L = P.L;
    pol.spr = (ncols / 2) / P.M; pol.row0 = row0; pol.colc0 = col0 / 2;
    pol.xm = P.xm; pol.var_new = bvar(P, t); pol.var_prev = bvar(P, t + 1); pol.secmax = P.secmax; pol.secabs = P.secabs;
    PartAcc pa;
    if (P.elementwise) {
        // no batch-global shift in random_denoiser: the section statistics stay neutral
        float* vn = bvar(P, t);
        const float* vp = bvar(P, t + 1);
        for (int e = threadIdx.x; e < GBM * (BN / 2); e += AMP_WG) {
            const int rho = e / (BN / 2), cc = e % (BN / 2);
            if (rho < nrows && 2 * cc < ncols) {
                const size_t o = (size_t)(row0 + rho) * P.N + col0 / 2 + cc;
                const float2 v = *reinterpret_cast<const float2*>(lds + rho * C::LDC + 2 * cc);
                float xr, xi, var;
                bamp_bayes_elem<KK>(P, c64, v.x, v.y, P.cov[o], xr, xi, var);
                *reinterpret_cast<float2*>(P.xm + 2 * o) = make_float2(xr, xi);
                vn[o] = var;
                pa.sumvar += (double)var;
                pa.notclose += torch_close(var, vp[o]) ? 0u : 1u;     // bamp.py:140
            }
        }
    } else {
        denoise_sections<true, KK>(pol, nrows * pol.spr, P.M, P.c, pa);
    }
    part_block_store(pa, P.parts + (size_t)t * P.nblk + blockIdx.y * gridDim.x + blockIdx.x, lds + C::CTILE_FLOATS);
}

// Iteration record t+1 (bamp.py:140): early exit when no var moved beyond allclose.
__device__ __forceinline__ void bamp_finish(const BampK& P, int t, uint32_t notclose, int fixed) {
    BampIter nx{};
    nx.stopped = notclose == 0 ? 1 : 0;
    nx.T = t + 1;
    nx.fixed = fixed;
    nx.fixed_all = (fixed < 0) ? 1 : 0;
    P.iters[t + 1] = nx;
    if (nx.stopped || t + 1 == P.max_iter) {
        amp_status s;
        s.T = t + 1; s.nan_state = fixed != 0 ? 1 : 0; s.stopped = nx.stopped;
        s.gemm = P.h2 ? AMP_ARITH_FP16X2 : P.x3 ? AMP_ARITH_BF16X3 : AMP_ARITH_F32;
        s.last_scalar[0] = s.last_scalar[1] = s.last_scalar[2] = s.last_scalar[3] = 0.f;
        *P.status = s;
    }
}

// Reduction and allclose decision (bamp.py:140).  The rare exact-float64 path (a section's
// normaliser out of the float64 range against the batch-global shift, amp_denoise.h) is spread
// over the grid as SCAMP's is: this workgroup only settles the exact batch max |xi| G over the
// candidate sections and leaves a pending record; bamp_fix_sec_body recomputes the out-of-range
// sections (a grid kernel: at 64-QAM on a failing detector most sections of the batch take this
// path every iteration, 314 ms per cfg5 detection when one workgroup recomputed them all), and
// bamp_fin adds the per-block counts and decides the early exit (both in one launch, bamp_fixall,
// in the whole-batch engine; the trial-sharded stages split this work, bamp_xr*).
__global__ __launch_bounds__(BRWG) void bamp_r(BampK P, Const64 c64, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    __shared__ double s_d[BRWG / 64];
    const BampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) P.iters[t + 1] = cur;
        return;
    }
    PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk, P.nblk, lds);
    if (part_allnan(pa)) {
        if (!cur.fixed_all) nan_fill(P.xm, bvar(P, t), (size_t)P.B * P.N);
        if (threadIdx.x == 0) bamp_finish(P, t, 1u, -1);
    } else if (part_danger(pa)) {
        const double slack = logit_slack(pa.maxabs);
        const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
        const float* cov = P.cov;
        const int M = P.M;
        double gm = 0.0;
        for (int sct = threadIdx.x; sct < P.B * P.L; sct += blockDim.x) {
            if ((double)P.secabs[sct] < pa.maxabs - slack) continue;
            const size_t o0 = (size_t)sct * M;
            auto ld = [=](int m, float& rr, float& ri, float& it) {
                const float2 v = xp2[o0 + m];
                rr = v.x; ri = v.y; it = 1.0f / (cov[o0 + m] * 0.5f);
            };
            gm = fmax(gm, section_absmax_f64(ld, M, c64));
        }
        gm = group_max(gm, 64);
        if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            double G = 0.0;
            for (int w = 0; w < BRWG / 64; ++w) G = fmax(G, s_d[w]);
            BampIter nx{};
            nx.stopped = 0; nx.T = t + 1; nx.fixed = 0; nx.fixed_all = 0;
            nx.G = G; nx.slack = slack; nx.notclose = pa.notclose; nx.active = 1;
            P.iters[t + 1] = nx;
        }
    } else if (threadIdx.x == 0) {
        bamp_finish(P, t, pa.notclose, 0);
    }
}

// per-block counts of bamp_fix_sec_body, written over iteration t's partials (consumed by
// bamp_r):
// slot i = {sections fixed, allclose delta} of block i
__device__ __forceinline__ int2* bamp_fix_counts(const BampK& P, int t) {
    return reinterpret_cast<int2*>(P.parts + (size_t)t * P.nblk);
}

__device__ __forceinline__ int bamp_block_sum_int(int v, int* s_i) {
    v = group_sum(v, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_i[threadIdx.x >> 6] = v;
    __syncthreads();
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_i[w];
    return tot;
}

// the out-of-range sections of a pending record, recomputed with the reference's exact float64
// op sequence (exact_section_f64): xmmse, var and the allclose delta against the previous var
__device__ __forceinline__ void bamp_fix_sec_body(const BampK& P, const Const64& c64, int t, const BampIter& pend,
                                                  int* s_i) {
    const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
    float2* x2 = reinterpret_cast<float2*>(P.xm);
    const float* cov = P.cov;
    float* vn = bvar(P, t);
    const float* vp = bvar(P, t + 1);
    const int M = P.M;
    int cnt = 0, dnc = 0;
    for (int sct = blockIdx.x * blockDim.x + threadIdx.x; sct < P.B * P.L; sct += gridDim.x * blockDim.x) {
        if (!((double)P.secmax[sct] - pend.G < AMP_DANGER + pend.slack)) continue;
        const size_t o0 = (size_t)sct * M;
        auto ld = [=](int m, float& rr, float& ri, float& it) {
            const float2 v = xp2[o0 + m];
            rr = v.x; ri = v.y; it = 1.0f / (cov[o0 + m] * 0.5f);
        };
        auto st = [&](int m, float xr, float xi, float var) {
            const size_t o = o0 + m;
            dnc += (torch_close(var, vp[o]) ? 0 : 1) - (torch_close(vn[o], vp[o]) ? 0 : 1);
            x2[o] = make_float2(xr, xi);
            vn[o] = var;
        };
        exact_section_f64<true>(ld, st, M, c64, pend.G);
        ++cnt;
    }
    cnt = bamp_block_sum_int(cnt, s_i);
    dnc = bamp_block_sum_int(dnc, s_i);
    if (threadIdx.x == 0) bamp_fix_counts(P, t)[blockIdx.x] = make_int2(cnt, dnc);
}

// bamp_fix_sec_body, then (last workgroup to arrive) bamp_fin's count and exit decision: one launch
__global__ __launch_bounds__(AMP_WG) void bamp_fixall(BampK P, Const64 c64, int t) {
    __shared__ int s_i[AMP_WG / 64];
    const BampIter pend = P.iters[t + 1];
    if (!pend.active || P.iters[t].stopped) return;
    bamp_fix_sec_body(P, c64, t, pend, s_i);
    if (last_arrival(P.rcnt + 1, gridDim.x)) {
        const int2* c = bamp_fix_counts(P, t);
        int fixed = 0, dnc = 0;
        for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) { fixed += c[i].x; dnc += c[i].y; }
        fixed = bamp_block_sum_int(fixed, s_i);
        dnc = bamp_block_sum_int(dnc, s_i);
        if (threadIdx.x == 0) bamp_finish(P, t, (uint32_t)((int)pend.notclose + dnc), fixed);
    }
}

// Tracker (bamp.py:13-25): xmmse = 0, var(prev) = 1, z = y, u = 0 + sigma2 -> 1/u.
// ---- trial-sharded iteration (amp_bamp_run_sharded; SURVEY §8(e) exact-compat) ----
// bamp_r split at its batch-global values, as the VAMP stages (amp_vamp.hip vamp_xr*): the
// not-close count (bamp.py:140) and max|xi| / min section max (bamp.py:70) after xr1, the rare
// path's exact max|xi| after xr2 and its recomputed sections' deltas after xr3.
__device__ inline void bamp_record(const BampK& P, int t, bool stop, int fixed) {
    BampIter nx{};
    nx.stopped = stop ? 1 : 0;
    nx.T = t + 1;
    nx.fixed = fixed;
    nx.fixed_all = (fixed < 0) ? 1 : 0;
    P.iters[t + 1] = nx;
    if (nx.stopped || t + 1 == P.max_iter) {
        amp_status s;
        s.T = t + 1; s.nan_state = fixed != 0 ? 1 : 0; s.stopped = nx.stopped;
        s.gemm = P.h2 ? AMP_ARITH_FP16X2 : P.x3 ? AMP_ARITH_BF16X3 : AMP_ARITH_F32;
        s.last_scalar[0] = s.last_scalar[1] = s.last_scalar[2] = s.last_scalar[3] = 0.f;
        *P.status = s;
    }
}

__global__ __launch_bounds__(BRWG) void bamp_xr1(BampK P, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    XState* xs = P.xs;
    if (P.iters[t].stopped) {
        if (threadIdx.x == 0) { xs->sum[0] = xs->sum[1] = 0.0; xs->mx[0] = xs->mx[1] = 0.0; }
        return;
    }
    const PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk, P.nblk, lds);
    if (threadIdx.x == 0) {
        xs->sum[0] = 0.0;
        xs->sum[1] = (double)pa.notclose;
        xs->mx[0] = (pa.maxabs <= 1.7976931348623157e308) ? pa.maxabs : INFINITY;   // NaN / inf wins
        xs->mx[1] = (pa.minsecmax == pa.minsecmax) ? -pa.minsecmax : INFINITY;
    }
}

__device__ inline PartAcc bamp_xs_global(const XState& x) {
    PartAcc pa;
    pa.sumvar = 0.0;
    pa.notclose = (uint32_t)x.sum[1];
    pa.maxabs = x.mx[0];
    pa.minsecmax = -x.mx[1];
    return pa;
}

__global__ __launch_bounds__(BRWG) void bamp_xr2(BampK P, Const64 c64, int t) {
    __shared__ double s_d[BRWG / 64];
    XState* xs = P.xs;
    const BampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) { P.iters[t + 1] = cur; xs->mode = 0; xs->gmax[0] = 0.0; }
        return;
    }
    PartAcc pa = bamp_xs_global(*xs);
    if (!part_allnan(pa) && part_danger(pa)) {
        const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
        const float* cov = P.cov;
        const int M = P.M;
        const double G32 = pa.maxabs, slack = logit_slack(G32);
        double gm = 0.0;
        for (int sct = threadIdx.x; sct < P.B * P.L; sct += blockDim.x) {
            if (!((double)P.secabs[sct] >= G32 - slack)) continue;
            const size_t o0 = (size_t)sct * M;
            gm = fmax(gm, section_absmax_f64([=](int m, float& rr, float& ri, float& it) {
                const float2 v = xp2[o0 + m];
                rr = v.x; ri = v.y; it = 1.0f / (cov[o0 + m] * 0.5f);
            }, M, c64));
        }
        gm = group_max(gm, 64);
        if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            double G = 0.0;
            for (int w = 0; w < BRWG / 64; ++w) G = fmax(G, s_d[w]);
            xs->gmax[0] = G;
            xs->mode = 2;
        }
        return;
    }
    int fixed = 0;
    if (part_allnan(pa)) {
        if (!cur.fixed_all) nan_fill(P.xm, bvar(P, t), (size_t)P.B * P.N);
        pa.notclose = 1;
        fixed = -1;
    }
    if (threadIdx.x == 0) {
        bamp_record(P, t, pa.notclose == 0, fixed);
        xs->mode = 0;
        xs->gmax[0] = 0.0;
    }
}

__global__ __launch_bounds__(BRWG) void bamp_xr3(BampK P, Const64 c64, int t) {
    __shared__ double s_d[2][BRWG / 64];
    XState* xs = P.xs;
    if (xs->mode != 2) {
        if (threadIdx.x == 0) xs->fix[0] = xs->fix[1] = xs->fix[2] = 0.0;
        return;
    }
    const PartAcc pa = bamp_xs_global(*xs);
    const double G = xs->gmax[0], slack = logit_slack(pa.maxabs);
    float* vn = bvar(P, t);
    const float* vp = bvar(P, t + 1);
    const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
    const float* cov = P.cov;
    float2* x2 = reinterpret_cast<float2*>(P.xm);
    const int M = P.M;
    int dnc = 0, cnt = 0;
    for (int sct = threadIdx.x; sct < P.B * P.L; sct += blockDim.x) {
        if (!((double)P.secmax[sct] - G < AMP_DANGER + slack)) continue;
        ++cnt;
        const size_t o0 = (size_t)sct * M;
        exact_section_f64<true>(
            [=](int m, float& rr, float& ri, float& it) {
                const float2 v = xp2[o0 + m];
                rr = v.x; ri = v.y; it = 1.0f / (cov[o0 + m] * 0.5f);
            },
            [&](int m, float xr, float xi, float var) {
                const size_t o = o0 + m;
                dnc += (torch_close(var, vp[o]) ? 0 : 1) - (torch_close(vn[o], vp[o]) ? 0 : 1);
                x2[o] = make_float2(xr, xi);
                vn[o] = var;
            },
            M, c64, G);
    }
    dnc = group_sum(dnc, 64);
    cnt = group_sum(cnt, 64);
    if ((threadIdx.x & 63) == 0) { s_d[0][threadIdx.x >> 6] = (double)dnc; s_d[1][threadIdx.x >> 6] = (double)cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0, c = 0.0;
        for (int w = 0; w < BRWG / 64; ++w) { b += s_d[0][w]; c += s_d[1][w]; }
        xs->fix[0] = 0.0; xs->fix[1] = b; xs->fix[2] = c;
    }
}

__global__ void bamp_xr4(BampK P, int t) {
    const XState* xs = P.xs;
    if (xs->mode != 2 || threadIdx.x != 0) return;
    const PartAcc pa = bamp_xs_global(*xs);
    const long long nc = (long long)pa.notclose + (long long)xs->fix[1];
    bamp_record(P, t, nc == 0, (int)xs->fix[2]);
}

__global__ void bamp_init_kernel(BampK P) {
    const size_t BN_ = (size_t)P.B * P.N, Bn = (size_t)P.B * P.n;
    const size_t tot = BN_ > Bn ? BN_ : Bn;
    const float iu = 1.0f / P.sigma2;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
        if (e < BN_) {
            reinterpret_cast<float2*>(P.xm)[e] = make_float2(0.f, 0.f);
            P.var1[e] = 1.0f;
        }
        if (e < Bn) {
            reinterpret_cast<float2*>(P.z)[e] = reinterpret_cast<const float2*>(P.y)[e];
            P.invu[e] = iu;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        P.rcnt[0] = 0u; P.rcnt[1] = 0u;
        BampIter it{};
        it.stopped = 0; it.T = 0; it.fixed = 0; it.fixed_all = 0;
        P.iters[0] = it;
    }
}

__global__ void bamp_output_kernel(BampK P) {
    const int T = P.status->T;
    if (((T - 1) & 1) == 0) return;
    const size_t BN_ = (size_t)P.B * P.N;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < BN_; e += (size_t)gridDim.x * blockDim.x)
        P.var0[e] = P.var1[e];
}

// dynamic LDS of every BAMP GEMM launch: the f32 tile's A block or the split tiles' staged planes,
// whichever is larger (every arithmetic runs from the same instantiation)
constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
constexpr size_t BLDS = cmax(h2_tile_lds<256, true>(), GemmCfg<256>::LDS_BYTES);
// the bf16x3 launches' LDS: the staged planes or the C tile + the epilogue's scratch past it (the
// partial-store scratch; bamp_kb2: + the 1 / tau tile): 48 KB for the complex tiles, three per CU
constexpr size_t XLDS_R = x3_tile_lds<128, false>(2048);
constexpr size_t XLDS_C = x3_tile_lds<128, true>(2048);
template <int BN>
constexpr size_t xlds_kb2() { return x3_tile_lds<BN, true>(2048 + GBM * (BN / 2)); }
static_assert(xlds_kb2<256>() <= BLDS && XLDS_C <= BLDS, "bf16x3 tiles within the attribute");
static_assert(BLDS <= 80 * 1024, "two BAMP GEMM workgroups per CU");
static int bamp_lds_attr(const void* fn) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)BLDS);
    if (e != hipSuccess) {
        set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
        return AMP_E_LAUNCH;
    }
    return AMP_OK;
}
template <int KK>
static int bamp_kb2_attrs() {
    int rc = bamp_lds_attr((const void*)bamp_kb2<128, KK>);
    if (!rc) rc = bamp_lds_attr((const void*)bamp_kb2<256, KK, GKC, true>);
    return rc ? rc : bamp_lds_attr((const void*)bamp_kb2<256, KK>);   // the KC = 256 forms fit the default 64 KB
}

// The f32 tiles stage 256-wide A chunks (33 KB of LDS: four tiles per CU instead of two, the
// chunk loaded one ahead); AMP_BAMP_KC=512 keeps 512 (A/B runs).  The chunking does not change
// the MFMA order: the same bits.
constexpr size_t BSKC_LDS = GemmCfg<128, 256>::LDS_BYTES;
static bool bamp_short_chunks(const BampK& P) {
    static const bool off = [] {
        const char* e = diag_env("AMP_BAMP_KC");
        return e && atoi(e) == 512;
    }();
    return !P.h2 && !P.x3 && !off;
}

template <int KK>
static void launch_kb2_kk(const BampK& P, const Const64& c64, int gr, int t, hipStream_t st) {
    if (P.bn == 128 && bamp_short_chunks(P)) {
        hipLaunchKernelGGL((bamp_kb2<128, KK, 256>), dim3(gr, P.ncpB2 / 128), dim3(AMP_WG), BSKC_LDS, st, P, c64, t);
        return;
    }
    if (P.bn == 128) {
        if (P.x3)
            hipLaunchKernelGGL((bamp_kb2<128, KK, GKC, true>), dim3(gr, P.ncpB2 / 128), dim3(AMP_WG), xlds_kb2<128>(), st,
                               P, c64, t);
        else
            hipLaunchKernelGGL((bamp_kb2<128, KK>), dim3(gr, P.ncpB2 / 128), dim3(AMP_WG), BLDS, st, P, c64, t);
    } else {
        if (P.x3)
            hipLaunchKernelGGL((bamp_kb2<256, KK, GKC, true>), dim3(gr, P.ncpB2 / 256), dim3(AMP_WG), xlds_kb2<256>(), st,
                               P, c64, t);
        else
            hipLaunchKernelGGL((bamp_kb2<256, KK>), dim3(gr, P.ncpB2 / 256), dim3(AMP_WG), BLDS, st, P, c64, t);
    }
}

static void launch_kb2(const BampK& P, const Const64& c64, int gr, int t, hipStream_t st) {
    switch (P.c.K) {
    case 1: launch_kb2_kk<1>(P, c64, gr, t, st); break;
    case 2: launch_kb2_kk<2>(P, c64, gr, t, st); break;
    case 4: launch_kb2_kk<4>(P, c64, gr, t, st); break;
    case 8: launch_kb2_kk<8>(P, c64, gr, t, st); break;
    case 16: launch_kb2_kk<16>(P, c64, gr, t, st); break;
    default: launch_kb2_kk<64>(P, c64, gr, t, st); break;
    }
}

static std::once_flag g_bamp_once;
static int g_bamp_rc = 0;

static int bamp_attrs() {
    std::call_once(g_bamp_once, [] {
        g_bamp_rc = bamp_lds_attr((const void*)bamp_ka1<>);
        if (!g_bamp_rc) g_bamp_rc = bamp_lds_attr((const void*)bamp_ka2<>);
        if (!g_bamp_rc) g_bamp_rc = bamp_lds_attr((const void*)bamp_kb1<>);
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<1>();
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<2>();
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<4>();
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<8>();
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<16>();
        if (!g_bamp_rc) g_bamp_rc = bamp_kb2_attrs<64>();
    });
    return g_bamp_rc;
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_bamp_workspace_bytes(const amp_dims* d, int32_t max_iter) {
    if (!d || max_iter <= 0) return 0;
    return bamp_carve(d, max_iter, nullptr).bytes;
}

}  // extern "C"

namespace amp {

// The parameter block of one BAMP forward from the C-ABI arguments (validated).
static int bamp_setup(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, BampK& P, Const64& c64) {
    int rc = check_dims(d, c);
    if (rc) return rc;
    AMP_REQUIRE(a && a->H && a->y && a->xmap && a->xmmse && a->var && a->status && a->ws,
                "amp_bamp_run: null pointer argument");
    AMP_REQUIRE(a->max_iter > 0, "amp_bamp_run: max_iter must be positive");
    AMP_REQUIRE(d->N % 4 == 0 && d->n % 4 == 0, "amp_bamp_run: N (%d) and n (%d) must be multiples of 4", d->N, d->n);
    const BampWs w = bamp_carve(d, a->max_iter, a->ws);
    AMP_REQUIRE(a->ws_bytes >= w.bytes, "amp_bamp_run: workspace %zu < %zu bytes", a->ws_bytes, w.bytes);
    rc = bamp_attrs();
    if (rc) return rc;
    bamp_geometry(d, P);
    P.max_iter = a->max_iter;
    P.sigma2 = (float)a->noise_var;
    P.Wabs2 = w.Wabs2; P.WH = w.WH; P.Wabs2T = w.Wabs2T; P.WHH = w.WHH;
    P.y = (const float*)a->y; P.v = w.v; P.z = w.z; P.invu = w.invu; P.s = w.s; P.cov = w.cov;
    P.xmap = (float*)a->xmap; P.xm = (float*)a->xmmse; P.var0 = (float*)a->var; P.var1 = w.var1;
    P.secmax = w.secmax; P.secabs = w.secabs; P.parts = w.parts; P.iters = w.iters; P.status = (amp_status*)a->status;
    P.c = to_const(c);
    P.xs = w.xs;
    P.rcnt = w.rcnt;
    {
        // block-banded H: the ranges are formed by the prepare launch sequence (AMP_BAND_GEMM=0: off)
        const char* e = diag_env("AMP_BAND_GEMM");
        const bool band = (d->Lin > 1 || d->Lout > 1) && !(e && e[0] == '0');
        for (int i = 0; i < 4; ++i) P.band[i] = band ? w.band[i] : nullptr;
    }
    AMP_REQUIRE(a->denoiser == 0 || a->denoiser == 1, "amp_bamp_run: denoiser %d", a->denoiser);
    P.elementwise = a->denoiser;
    P.P0 = a->P0;
    P.Ps = a->Ps;
    // GEMM arithmetic, all at the reference's c64 operand precision (bamp.py:59-64) unless fp16x2 is
    // asked for: AMP_GEMM_F32 (f32 MFMA), AMP_GEMM_X3 (bf16x3 tiles, 24-bit operands) or, only when
    // asked for (AMP_GEMM_H2, or AUTO with AMP_BAMP_GEMM=h2), the fp16x2 tile (22-bit operands:
    // narrower than the reference).  AUTO: f32 MFMA (AMP_BAMP_GEMM=x3: bf16x3 where the shape tiles).
    AMP_REQUIRE(a->gemm == AMP_GEMM_AUTO || a->gemm == AMP_GEMM_F32 || a->gemm == AMP_GEMM_H2 || a->gemm == AMP_GEMM_X3,
                "amp_bamp_run: gemm %d (AUTO, F32, X3 or H2)", a->gemm);
    const bool h2ok = bamp_h2_shape(d);
    AMP_REQUIRE((a->gemm != AMP_GEMM_H2 && a->gemm != AMP_GEMM_X3) || h2ok,
                "amp_bamp_run: the split-precision GEMMs need N %% 64 == 0 and n %% 64 == 0 (N = %d, n = %d)", d->N, d->n);
    static const char gemm_env = [] {
        const char* e = diag_env("AMP_BAMP_GEMM");
        return e ? e[0] : '\0';
    }();
    P.h2 = (a->gemm == AMP_GEMM_H2 || (a->gemm == AMP_GEMM_AUTO && h2ok && gemm_env == 'h')) ? 1 : 0;
    P.x3 = (a->gemm == AMP_GEMM_X3 || (a->gemm == AMP_GEMM_AUTO && h2ok && gemm_env == 'x')) ? 1 : 0;
    // tile order: the fp16x2 tiles walk row blocks (each XCD serves the whole 4 MB operator from its
    // L2); the bf16x3 operator (6 MB at cfg5) does not fit, so its tiles walk column blocks (each
    // XCD keeps its share of the operator resident).  AMP_BAMP_X3_ROWS=1: row-major (A/B runs).
    static const bool x3_rows = [] {
        const char* e = diag_env("AMP_BAMP_X3_ROWS");
        return e && e[0] == '1';
    }();
    P.tile_rows = P.h2 || (P.x3 && x3_rows) ? 1 : 0;
    P.rows_pad = round_up(d->B, GBM);
    P.ap = w.ap;
    P.rexp = w.rexp;
    c64 = to_const64(c);
    return AMP_OK;
}

// Tracker (bamp.py:13-25): the four weights and the initial state.
static int bamp_prepare_impl(const BampK& P, const amp_bamp_args* a, hipStream_t st) {
    int rc;
    const float2* H = (const float2*)a->H;
    if (P.x3) {
        // the four operators as bf16x3 planes in ONE launch: |H|^2 (O = n, J = N), H (O = n, J = N),
        // |H|^2^T (O = N, J = n), H^H (O = N, J = n)
        CWeightJob j[4];
        j[0] = CWeightJob{H, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.Wabs2, P.N, P.n, WPACKX3_ABS2, 0};
        j[1] = CWeightJob{H, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.WH, P.N, P.n, WPACKX3, 0};
        j[2] = CWeightJob{H, 1, P.N, 0, nullptr, P.N, P.n, (float*)P.Wabs2T, P.n, P.N, WPACKX3_ABS2, 0};
        j[3] = CWeightJob{H, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.WHH, P.n, P.N, WPACKX3, 0};
        if ((rc = build_cweights(j, 4, nullptr, 0, st))) return rc;
    } else if (P.h2) {
        // the four operators as fp16x2 planes (exponent BH2_EX) in ONE launch: |H|^2 (O = n, J = N),
        // H (O = n, J = N), |H|^2^T (O = N, J = n), H^H (O = N, J = n)
        CWeightJob j[4];
        j[0] = CWeightJob{H, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.Wabs2, P.N, P.n, WPACKH2_ABS2, BH2_EX};
        j[1] = CWeightJob{H, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.WH, P.N, P.n, WPACKH2, BH2_EX};
        j[2] = CWeightJob{H, 1, P.N, 0, nullptr, P.N, P.n, (float*)P.Wabs2T, P.n, P.N, WPACKH2_ABS2, BH2_EX};
        j[3] = CWeightJob{H, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.WHH, P.n, P.N, WPACKH2, BH2_EX};
        if ((rc = build_cweights(j, 4, nullptr, 0, st))) return rc;
    } else {
    // weights, once per forward (Tracker: adj, abs2, abs2T, bamp.py:17-19)
    if ((rc = build_abs2_weight(H, P.N, 1, P.n, P.N, (float*)P.Wabs2, P.kapA1, P.ncpA1, st))) return rc;
    if ((rc = build_cweight(H, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.WH, P.kapA2, P.ncpA2, st))) return rc;
    if ((rc = build_abs2_weight(H, 1, P.N, P.N, P.n, (float*)P.Wabs2T, P.kapB1, P.ncpB1, st))) return rc;
    if ((rc = build_cweight(H, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.WHH, P.kapB2, P.ncpB2, st))) return rc;
    }
    if (P.band[0] && (P.h2 || P.x3)) {
        // per column tile: real |H|^2 (fp16x2 two planes, bf16x3 three; 8 16-tiles per 128
        // outputs), complex H (four / six planes, 4)
        const int pr = P.x3 ? 3 : 2, pc = P.x3 ? 6 : 4;
        if ((rc = h2_kband(P.Wabs2, pr, P.N / 32, 8, P.ncpA1 / 128, P.n / 16, const_cast<int*>(P.band[0]), st))) return rc;
        if ((rc = h2_kband(P.WH, pc, P.N / 32, 4, P.ncpA2 / 128, P.n / 16, const_cast<int*>(P.band[1]), st))) return rc;
        if ((rc = h2_kband(P.Wabs2T, pr, P.n / 32, 8, P.ncpB1 / 128, P.N / 16, const_cast<int*>(P.band[2]), st))) return rc;
        if ((rc = h2_kband(P.WHH, pc, P.n / 32, P.bn / 32, P.ncpB2 / P.bn, P.N / 16, const_cast<int*>(P.band[3]), st))) return rc;
    } else if (P.band[0]) {
        const float* wts[4] = {P.Wabs2, P.WH, P.Wabs2T, P.WHH};
        const int kaps[4] = {P.kapA1, P.kapA2, P.kapB1, P.kapB2}, ncps[4] = {P.ncpA1, P.ncpA2, P.ncpB1, P.ncpB2};
        const int bns[4] = {128, 128, 128, P.bn};
        for (int i = 0; i < 4; ++i)
            if ((rc = weight_kband(wts[i], kaps[i], ncps[i], bns[i], const_cast<int*>(P.band[i]), st))) return rc;
    }
    const size_t tot = std::max((size_t)P.B * P.N, (size_t)P.B * P.n);
    const int g = (int)std::min<size_t>((tot + 255) / 256, 2048);
    hipLaunchKernelGGL(bamp_init_kernel, dim3(g), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("bamp_init");
    return AMP_OK;
}

// the four GEMM launches of one BAMPLayer.forward (bamp.py:59-64), each preceded on the fp16x2
// path by the split of its A rows (var, xmmse, 1/u, s) into the plane buffer
static void bamp_split(const BampK& P, const float* a, int lda, int K, bool cpx, int t, hipStream_t st) {
    const int* stop = &P.iters[t].stopped;
    // a workgroup per row when four rows per workgroup would leave CUs idle on long rows
    const int wpr = (P.rows_pad / 4 < 2 * device_cu_count() && K >= 1024) ? 4 : 1;
    const dim3 grid(P.rows_pad * wpr / 4);
    if (P.x3) {
        if (cpx)
            hipLaunchKernelGGL(x3_split_rows_kernel<true>, grid, dim3(256), 0, st, a, lda, P.B, P.rows_pad, K, P.ap,
                               stop, wpr);
        else
            hipLaunchKernelGGL(x3_split_rows_kernel<false>, grid, dim3(256), 0, st, a, lda, P.B, P.rows_pad, K, P.ap,
                               stop, wpr);
        return;
    }
    if (cpx)
        hipLaunchKernelGGL(h2_split_rows_kernel<true>, grid, dim3(256), 0, st, a, lda, P.B, P.rows_pad, K, P.ap,
                           P.rexp, stop, wpr);
    else
        hipLaunchKernelGGL(h2_split_rows_kernel<false>, grid, dim3(256), 0, st, a, lda, P.B, P.rows_pad, K, P.ap,
                           P.rexp, stop, wpr);
}

static void bamp_gemms(const BampK& P, const Const64& c64, int t, hipStream_t st) {
    const int gr = cdiv(P.B, GBM);
    // the host reads bvar(P, t + 1) as the device does: (t + 1) & 1 picks var1, else var0
    if (P.h2 || P.x3) bamp_split(P, ((t + 1) & 1) ? P.var1 : P.var0, P.N, P.N, false, t, st);
    const bool skc = bamp_short_chunks(P);
    if (skc) hipLaunchKernelGGL((bamp_ka1<256>), dim3(gr, P.ncpA1 / 128), dim3(AMP_WG), BSKC_LDS, st, P, t);
    else if (P.x3) hipLaunchKernelGGL((bamp_ka1<GKC, true>), dim3(gr, P.ncpA1 / 128), dim3(AMP_WG), XLDS_R, st, P, t);
    else hipLaunchKernelGGL((bamp_ka1<>), dim3(gr, P.ncpA1 / 128), dim3(AMP_WG), BLDS, st, P, t);
    if (P.h2 || P.x3) bamp_split(P, P.xm, 2 * P.N, P.N, true, t, st);
    if (skc) hipLaunchKernelGGL((bamp_ka2<256>), dim3(gr, P.ncpA2 / 128), dim3(AMP_WG), BSKC_LDS, st, P, t);
    else if (P.x3) hipLaunchKernelGGL((bamp_ka2<GKC, true>), dim3(gr, P.ncpA2 / 128), dim3(AMP_WG), XLDS_C, st, P, t);
    else hipLaunchKernelGGL((bamp_ka2<>), dim3(gr, P.ncpA2 / 128), dim3(AMP_WG), BLDS, st, P, t);
    if (P.h2 || P.x3) bamp_split(P, P.invu, P.n, P.n, false, t, st);
    if (skc) hipLaunchKernelGGL((bamp_kb1<256>), dim3(gr, P.ncpB1 / 128), dim3(AMP_WG), BSKC_LDS, st, P, t);
    else if (P.x3) hipLaunchKernelGGL((bamp_kb1<GKC, true>), dim3(gr, P.ncpB1 / 128), dim3(AMP_WG), XLDS_R, st, P, t);
    else hipLaunchKernelGGL((bamp_kb1<>), dim3(gr, P.ncpB1 / 128), dim3(AMP_WG), BLDS, st, P, t);
    if (P.h2 || P.x3) bamp_split(P, P.s, 2 * P.n, P.n, true, t, st);
    launch_kb2(P, c64, gr, t, st);
}

// One BAMPLayer.forward (bamp.py:48-64) + the allclose test of bamp.py:140 (no-op once stopped).
// bamp_fixall is a no-op unless bamp_r left a pending record (nfix blocks' counts fit the
// iteration's nblk partial slots).
static int bamp_iterate_impl(const BampK& P, const Const64& c64, int t, hipStream_t st) {
    bamp_gemms(P, c64, t, st);
    hipLaunchKernelGGL(bamp_r, dim3(1), dim3(BRWG), 0, st, P, c64, t);
    const int nfix = fix_grid(P.nblk, P.B * P.L);
    hipLaunchKernelGGL(bamp_fixall, dim3(nfix), dim3(AMP_WG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("bamp iteration");
    return AMP_OK;
}

static int bamp_iterate_sharded(const BampK& P, const Const64& c64, int t, hipStream_t st, bool& hook_failed) {
    bamp_gemms(P, c64, t, st);
    hipLaunchKernelGGL(bamp_xr1, dim3(1), dim3(BRWG), 0, st, P, t);
    AMP_LAUNCH_CHECK("bamp_xr1");
    // every hook call is made on every rank even after one failed: the ranks' collectives stay
    // matched and a failed rank's poisoned words reach the others (amp_sparc.h)
    hook_failed |= call_allreduce_hook(P.xs->sum, 2, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hook_failed |= call_allreduce_hook(P.xs->mx, 2, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(bamp_xr2, dim3(1), dim3(BRWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("bamp_xr2");
    hook_failed |= call_allreduce_hook(P.xs->gmax, 1, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(bamp_xr3, dim3(1), dim3(BRWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("bamp_xr3");
    hook_failed |= call_allreduce_hook(P.xs->fix, 3, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hipLaunchKernelGGL(bamp_xr4, dim3(1), dim3(64), 0, st, P, t);
    AMP_LAUNCH_CHECK("bamp_xr4");
    return AMP_OK;
}

// the caller's var holds the last executed iteration's (ping-pong buffers)
static int bamp_finalize_impl(const BampK& P, hipStream_t st) {
    hipLaunchKernelGGL(bamp_output_kernel, dim3((int)std::min<size_t>(((size_t)P.B * P.N + 255) / 256, 2048)),
                       dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("bamp_output");
    return AMP_OK;
}

}  // namespace amp

extern "C" {

int amp_bamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, int32_t B_global,
                         void* stream) {
    BampK P;
    Const64 c64;
    int rc = bamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(allreduce_hook_set(), "amp_bamp_run_sharded: no all-reduce hook registered (amp_set_allreduce_hook)");
    AMP_REQUIRE(B_global >= d->B, "amp_bamp_run_sharded: B_global = %d < this rank's B = %d", B_global, d->B);
    AMP_REQUIRE(a->denoiser == 0, "amp_bamp_run_sharded: the element-wise denoiser (mode 'random', B = 1) has no "
                "batch-global values to share");
    hipStream_t st = (hipStream_t)stream;
    rc = bamp_prepare_impl(P, a, st);
    bool hook_failed = false;
    for (int t = 0; t < P.max_iter && !rc; ++t) rc = bamp_iterate_sharded(P, c64, t, st, hook_failed);
    if (!rc && hook_failed) rc = hook_failure("bamp");
    return rc ? rc : bamp_finalize_impl(P, st);
}

int amp_bamp_run(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream) {
    BampK P;
    Const64 c64;
    int rc = bamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if ((rc = bamp_prepare_impl(P, a, st))) return rc;
    for (int t = 0; t < P.max_iter; ++t)
        if ((rc = bamp_iterate_impl(P, c64, t, st))) return rc;
    return bamp_finalize_impl(P, st);
}

int amp_bamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream) {
    BampK P;
    Const64 c64;
    int rc = bamp_setup(d, c, a, P, c64);
    return rc ? rc : bamp_prepare_impl(P, a, (hipStream_t)stream);
}

int amp_bamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, int32_t t, void* stream) {
    BampK P;
    Const64 c64;
    int rc = bamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(t >= 0 && t < a->max_iter, "amp_bamp_iterate: t = %d outside [0, %d)", t, a->max_iter);
    return bamp_iterate_impl(P, c64, t, (hipStream_t)stream);
}

int amp_bamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream) {
    BampK P;
    Const64 c64;
    int rc = bamp_setup(d, c, a, P, c64);
    return rc ? rc : bamp_finalize_impl(P, (hipStream_t)stream);
}

// BAMPLayer.random_denoiser (bamp.py:79-88) as a standalone element-wise op (layer-level API).
__global__ __launch_bounds__(AMP_WG) void bamp_random_denoise_kernel(BampK P, Const64 c64, long long count,
                                                                     const float2* r, const float* cov, float2* xm,
                                                                     float* var) {
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < count;
         e += (long long)gridDim.x * blockDim.x) {
        float xr, xi, v;
        bamp_bayes_elem<AMP_MAX_K>(P, c64, r[e].x, r[e].y, cov[e], xr, xi, v);
        xm[e] = make_float2(xr, xi);
        var[e] = v;
    }
}

int amp_bamp_random_denoise(const amp_constellation* c, int64_t count, const void* r, const void* cov, float P0,
                            float Ps, void* xmmse, void* var, void* stream) {
    AMP_REQUIRE(c && c->K >= 1 && c->K <= AMP_MAX_K, "amp_bamp_random_denoise: bad constellation size %d",
                c ? c->K : 0);
    AMP_REQUIRE(count >= 0, "amp_bamp_random_denoise: count < 0");
    if (count == 0) return AMP_OK;
    AMP_REQUIRE(r && cov && xmmse && var, "amp_bamp_random_denoise: null pointer argument");
    BampK P{};
    P.c = to_const(c);
    P.P0 = P0;
    P.Ps = Ps;
    const Const64 c64 = to_const64(c);
    const int g = (int)std::max(1LL, std::min(((long long)count + AMP_WG - 1) / AMP_WG, 8192LL));
    hipLaunchKernelGGL(bamp_random_denoise_kernel, dim3(g), dim3(AMP_WG), 0, (hipStream_t)stream, P, c64, (long long)count,
                       (const float2*)r, (const float*)cov, (float2*)xmmse, (float*)var);
    AMP_LAUNCH_CHECK("bamp_random_denoise");
    return AMP_OK;
}

}  // extern "C"
