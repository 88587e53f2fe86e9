// amp_scamp.hip — SCAMP (spatially coupled SPARC AMP), device-resident iteration loop.
//
// Restates SCAMP.forward (scamp.py:77-107), Tracker (scamp.py:8-25) and
// SCAMPLayer.forward (scamp.py:43-59):
//   gamma = W psi / Lc ; b = gamma / phi ; z = y - A xmmse + b z ; phi = sigma2 + gamma ;
//   tau = L / (W^T (1/phi)) / Mr ; xmap = xmmse + tau (A^H (z / phi)) ;
//   xmmse = denoiser(xmap, tau/2) (mean only, scamp.py:61-68) ;
//   psi = 1 - sum_{block} |xmmse|^2 / Na ; early exit on allclose(psi) (scamp.py:105).
// Per iteration: two fp32-MFMA GEMM launches with fused epilogues + one reduction /
// exact-float64 fix-up workgroup.  The second GEMM's column tile holds whole coupling
// blocks (2*Nt columns) so psi is formed in its epilogue.
#include <algorithm>
#include <atomic>
#include <mutex>

#include "amp_gemm_x3.h"
#include "amp_scamp.h"

namespace amp {

// z = y - A xmmse + b z ; phi = sigma2 + gamma ; s = z / phi   (scamp.py:45-51, 57)
// X3: the bf16x3 tile (amp_gemm_x3.h) in an instantiation of its own, so the f32 tiles keep their
// register budget (one instantiation holding both ran the f32 ISI shape 25 % slower)
template <int KC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void scamp_ka(ScampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    const GemmTile tile = xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * 128;
    const int twoN = 2 * P.N, twon = 2 * P.n;
    const int kb = P.bandA ? P.bandA[2 * tile.cb] : 0, ke = P.bandA ? P.bandA[2 * tile.cb + 1] : -1;
    if constexpr (X3)
        gemm_tile_x3<128, true>(P.lap, P.rows_pad, P.N, P.WA, row0, col0, lds, kb, ke);
    else
        gemm_tile<128, ALoadPlain, KC>(ALoadPlain{P.xm, twoN, P.B, twoN}, P.WA, P.kapA, row0, col0, lds, kb, ke);
    using C = GemmCfg<128, KC>;
    const float* psi = spsi(P, t + 1);               // psi of iteration t-1 (ones at t = 0)
    const float* phi_old = sphi(P, t + 1);           // +inf at t = 0 (scamp.py:19)
    float* phi_new = sphi(P, t);
    // gamma of each (trial, output block) the tile touches, formed once (the same float32 sum as
    // scamp_gamma) instead of once per element: Lin MACs of global loads per element had made the
    // epilogue, not the GEMM, the cost of a Lin > 1 tile
    // The rows' psi and the W rows come into LDS first (coalesced), so the serial float32 sums
    // read LDS, not a chain of dependent global loads.
    const int lo0 = (col0 >> 1) / P.Nr, nlo = (min((col0 >> 1) + 63, P.n - 1)) / P.Nr - lo0 + 1;
    const int Lin = P.Lin;
    float* sg = lds + C::CTILE_FLOATS;                 // [GBM][nlo] gamma
    float* sp = sg + GBM * nlo;                        // [GBM][Lin] psi rows
    float* sw = sp + GBM * Lin;                        // [nlo][Lin] W rows lo0 ..
    const bool per_block = C::CTILE_FLOATS + GBM * nlo + GBM * Lin + nlo * Lin <= C::A_FLOATS;
    if (per_block) {
        for (int e = threadIdx.x; e < GBM * Lin; e += AMP_WG) {
            const int row = row0 + e / Lin;
            sp[e] = row < P.B ? psi[(size_t)row0 * Lin + e] : 0.f;
        }
        for (int e = threadIdx.x; e < nlo * Lin; e += AMP_WG) sw[e] = P.W[(size_t)lo0 * Lin + e];
        __syncthreads();
        for (int e = threadIdx.x; e < GBM * nlo; e += AMP_WG) {
            const int rho = e / nlo, j = e - rho * nlo;
            float g = 0.f;                             // scamp_gamma's sum, in its order
            for (int lc = 0; lc < Lin; ++lc) g += sw[j * Lin + lc] * sp[rho * Lin + lc];
            sg[e] = g / (float)Lin;
        }
        __syncthreads();
    }
    // Every global load of this thread's elements is issued before any store: the stores to z / s
    // may alias the next element's loads as far as the compiler knows, and a load-compute-store loop
    // waited a full memory latency per element (each element reads and writes only its own z).
    constexpr int IT = GBM * 64 / AMP_WG;
    float2 yv[IT], zv[IT];
    float po[IT];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
        // unconditional loads at a clamped index (a lane-divergent branch around them serialises
        // their latencies, amp_gemm.h ALoadPlain); out-of-range elements are never stored
        const int e = threadIdx.x + u * AMP_WG;
        const int rho = e >> 6, cp = e & 63;
        const int row = min(row0 + rho, P.B - 1), i = min((col0 >> 1) + cp, P.n - 1);
        const size_t oc = (size_t)row * twon + 2 * i;
        yv[u] = *reinterpret_cast<const float2*>(P.y + oc);
        zv[u] = *reinterpret_cast<const float2*>(P.z + oc);
        po[u] = phi_old[(size_t)row * P.Lout + i / P.Nr];
    }
#pragma unroll
    for (int u = 0; u < IT; ++u) {
        const int e = threadIdx.x + u * AMP_WG;
        const int rho = e >> 6, cp = e & 63;
        const int row = row0 + rho, i = (col0 >> 1) + cp;
        if (row < P.B && i < P.n) {
            const int lo = i / P.Nr;
            const float gma = per_block ? sg[rho * nlo + lo - lo0] : scamp_gamma(P, psi + (size_t)row * P.Lin, lo);
            const float b = gma / po[u];
            const size_t oc = (size_t)row * twon + 2 * i;
            const float ar = lds[rho * C::LDC + 2 * cp], ai = lds[rho * C::LDC + 2 * cp + 1];
            const float zr = (yv[u].x - ar) + b * zv[u].x;
            const float zi = (yv[u].y - ai) + b * zv[u].y;
            const float ph = P.sigma2 + gma;
            const float iph = 1.0f / ph;
            *reinterpret_cast<float2*>(P.z + oc) = make_float2(zr, zi);
            *reinterpret_cast<float2*>(P.s + oc) = make_float2(zr * iph, zi * iph);
            if (i % P.Nr == 0) phi_new[(size_t)row * P.Lout + lo] = ph;
        }
    }
}

struct ScampDenoisePolicy {
    const float* tile;
    const float* tau_tile;   // LDS [32][Lin] tau of the tile's rows and blocks lc0 .. lc0 + Lin - 1
    int ldc, spr, M, N, Nt, L, row0, colc0, Lin, lc0;
    float* xm;
    float* secmax;
    float* secabs;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const int cc = sj * M + m;
        const float2 v = *reinterpret_cast<const float2*>(tile + rho * ldc + 2 * cc);
        rr = v.x; ri = v.y;
        it = 1.0f / (tau_tile[rho * Lin + (colc0 + cc) / Nt - lc0] * 0.5f);   // tau_use / 2 (scamp.py:63)
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float, PartAcc&) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * N + colc0 + sj * M + m;
        *reinterpret_cast<float2*>(xm + 2 * o) = make_float2(xr, xi);
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        const int rho = sec / spr, sj = sec - rho * spr;
        const size_t o = (size_t)(row0 + rho) * L + (colc0 / M) + sj;
        secmax[o] = smax;
        secabs[o] = sabs;
    }
};

// tau = L / (W^T (1/phi)) / Mr ; xmap = xmmse + tau (A^H s) ; xmmse = denoiser ; psi   (scamp.py:53-59)
template <int BN, int KK, int KC = GKC, bool X3 = false>
__global__ __launch_bounds__(AMP_WG) void scamp_kb(ScampK P, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (P.iters[t].stopped) return;
    using C = GemmCfg<BN, KC>;
    const GemmTile tile = xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * BN;
    const int twoN = 2 * P.N, twon = 2 * P.n;
    const int kb = P.bandB ? P.bandB[2 * tile.cb] : 0, ke = P.bandB ? P.bandB[2 * tile.cb + 1] : -1;
    if constexpr (X3)
        gemm_tile_x3<BN, true>(P.lap, P.rows_pad, P.n, P.WAH, row0, col0, lds, kb, ke);
    else
        gemm_tile<BN, ALoadPlain, KC>(ALoadPlain{P.s, twon, P.B, twon}, P.WAH, P.kapB, row0, col0, lds, kb, ke);
    const int nrows = min(GBM, P.B - row0), ncols = min(BN, twoN - col0);
    const int lc0 = (col0 / 2) / P.Nt, nlc = max(1, (ncols / 2) / P.Nt);   // coupling blocks in this tile
    // tau of the blocks this tile covers only (blocks lc0 .. lc0 + ntc - 1): each is written to
    // P.tau by the tile that holds its first column
    const int ntc = (col0 / 2 + ncols / 2 - 1) / P.Nt - lc0 + 1;
    float* tau_t = lds + C::CTILE_FLOATS;                                    // [32][ntc]
    const float* phi = sphi(P, t);
    // the rows' 1 / phi and the W columns lc0 .. into LDS first (coalesced): the serial float32
    // sums then read LDS instead of a chain of dependent global loads
    const int Lout = P.Lout;
    float* siph = tau_t + GBM * ntc;                                         // [32][Lout] 1 / phi
    float* swc = siph + GBM * Lout;                                          // [ntc][Lout] W columns
    const bool staged = C::CTILE_FLOATS + GBM * ntc + GBM * Lout + ntc * Lout <= C::A_FLOATS;
    if (staged) {
        for (int e = threadIdx.x; e < GBM * Lout; e += AMP_WG)
            siph[e] = e / Lout < nrows ? 1.0f / phi[(size_t)row0 * Lout + e] : 0.f;
        for (int e = threadIdx.x; e < ntc * Lout; e += AMP_WG) {
            const int j = e / Lout, lo = e - j * Lout;
            swc[e] = P.W[lo * P.Lin + lc0 + j];
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < GBM * ntc; e += AMP_WG) {
        const int rho = e / ntc, lc = lc0 + e - rho * ntc;
        float tv = 0.f;
        if (rho < nrows) {
            float acc = 0.f;   // (W^T (1/phi))[lc] in float32
            if (staged)
                for (int lo = 0; lo < Lout; ++lo) acc += swc[(lc - lc0) * Lout + lo] * siph[rho * Lout + lo];
            else
                for (int lo = 0; lo < P.Lout; ++lo)
                    acc += P.W[lo * P.Lin + lc] * (1.0f / phi[(size_t)(row0 + rho) * P.Lout + lo]);
            tv = ((1.0f / acc) * (float)P.L) / (float)P.Nr;          // L / x = recip(x) * L ; / Mr
            if (lc * P.Nt >= col0 / 2) P.tau[(size_t)(row0 + rho) * P.Lin + lc] = tv;
        }
        tau_t[e] = tv;
    }
    __syncthreads();
    {
        // xmmse of every element of this thread first (the xmap stores may alias them as far as
        // the compiler knows: one load latency per element otherwise)
        constexpr int IT = GBM * BN / AMP_WG;
        float xv[IT];
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            // unconditional loads at a clamped index (see scamp_ka); out-of-range elements unused
            const int e = threadIdx.x + u * AMP_WG, rho = min(e / BN, nrows - 1), cc = min(e % BN, ncols - 1);
            xv[u] = P.xm[(size_t)(row0 + rho) * twoN + col0 + cc];
        }
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int e = threadIdx.x + u * AMP_WG, rho = e / BN, cc = e % BN;
            if (rho < nrows && cc < ncols) {
                const size_t o = (size_t)(row0 + rho) * twoN + col0 + cc;
                const float tv = tau_t[rho * ntc + ((col0 + cc) >> 1) / P.Nt - lc0];
                const float xp = xv[u] + tv * lds[rho * C::LDC + cc];
                P.xmap[o] = xp;
                lds[rho * C::LDC + cc] = xp;
            }
        }
    }
    __syncthreads();
    ScampDenoisePolicy pol;
    pol.tile = lds; pol.tau_tile = tau_t; pol.ldc = C::LDC; pol.M = P.M; pol.N = P.N; pol.Nt = P.Nt; pol.L = P.L;
    pol.spr = (ncols / 2) / P.M; pol.row0 = row0; pol.colc0 = col0 / 2; pol.Lin = ntc; pol.lc0 = lc0;
    pol.xm = P.xm; pol.secmax = P.secmax; pol.secabs = P.secabs;
    PartAcc pa;
    denoise_sections<false, KK>(pol, nrows * pol.spr, P.M, P.c, pa);
    __syncthreads();
    // psi = 1 - sum_block |xmmse|^2 / Na (scamp.py:59) from the freshly written tile
    const float* psi_prev = spsi(P, t + 1);
    float* psi_new = spsi(P, t);
    unsigned nc = 0;
    for (int e = threadIdx.x; e < (P.psi_split ? 0 : GBM * nlc); e += AMP_WG) {
        const int rho = e / nlc, b = e % nlc;
        if (rho >= nrows) continue;
        const int lc = lc0 + b;
        const float2* xr = reinterpret_cast<const float2*>(P.xm) + (size_t)(row0 + rho) * P.N + (size_t)lc * P.Nt;
        double ssum = 0.0;
        for (int m = 0; m < P.Nt; ++m) {
            const float2 v = xr[m];
            const float a = (float)sqrt((double)v.x * v.x + (double)v.y * v.y);   // torch abs (hypot)
            ssum += (double)(a * a);
        }
        const float ps = 1.0f - (float)ssum / (float)P.Na;
        const size_t o = (size_t)(row0 + rho) * P.Lin + lc;
        nc += torch_close(ps, psi_prev[o]) ? 0u : 1u;                // scamp.py:105
        psi_new[o] = ps;
    }
    pa.notclose += nc;
    part_block_store(pa, P.parts + (size_t)t * P.nblk + blockIdx.y * gridDim.x + blockIdx.x, lds);
}

// psi (scamp.py:59) and its allclose count (scamp.py:105) when the A^H tile holds only part of
// a coupling block: one thread per (trial, block), after every tile of the iteration is written.
__device__ __forceinline__ unsigned block_sum_u32(unsigned v, unsigned* s_u) {
    v = group_sum(v, 64);
    if ((threadIdx.x & 63) == 0) s_u[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_u[w];
    return tot;
}

__global__ __launch_bounds__(AMP_WG) void scamp_psi(ScampK P, int t) {
    // one wavefront per (trial, coupling block): lanes stride the block's Nt entries
    __shared__ unsigned s_u[AMP_WG / 64];
    if (P.iters[t].stopped) return;
    const float* psi_prev = spsi(P, t + 1);
    float* psi_new = spsi(P, t);
    const int lane = threadIdx.x & 63;
    const int nwave = gridDim.x * (AMP_WG / 64);
    unsigned nc = 0;
    for (int blk = blockIdx.x * (AMP_WG / 64) + (threadIdx.x >> 6); blk < P.B * P.Lin; blk += nwave) {
        const float2* xr = reinterpret_cast<const float2*>(P.xm) + (size_t)blk * P.Nt;
        double ssum = 0.0;
        for (int m = lane; m < P.Nt; m += 64) {
            const float2 v = xr[m];
            const float a = (float)sqrt((double)v.x * v.x + (double)v.y * v.y);   // torch abs (hypot)
            ssum += (double)(a * a);
        }
        ssum = group_sum(ssum, 64);
        if (lane == 0) {
            const float ps = 1.0f - (float)ssum / (float)P.Na;
            nc += torch_close(ps, psi_prev[blk]) ? 0u : 1u;
            psi_new[blk] = ps;
        }
    }
    nc = block_sum_u32(nc, s_u);
    if (threadIdx.x == 0) P.psi_nc[(size_t)t * P.psi_nblk + blockIdx.x] = nc;
}

// Rare path (float64 fix-up) spread over the grid.  scamp_r reduces the partials and, when some
// section may leave the float64 range, settles the exact batch max |xi| G (one workgroup: few
// candidate sections); scamp_fix_sec recomputes the out-of-range sections with the reference's
// exact arithmetic, scamp_fix_psi_fin their coupling blocks' psi (and the allclose delta), each a
// grid kernel, and the last workgroup of the second adds the per-block counts and decides the
// early exit.  Without a pending fix-up both return at once.  The trial-sharded stages run
// scamp_fix_sec / scamp_fix_psi and settle the counts across ranks.  (Before: one
// workgroup recomputed every such section, 267 us per iteration at cfg3's NaN onset.)
__device__ __forceinline__ void scamp_finish(const ScampK& P, int t, uint32_t notclose, int fixed, int fixed_all) {
    ScampIter nx;
    nx.stopped = notclose == 0 ? 1 : 0;
    nx.T = t + 1;
    nx.fixed = fixed;
    nx.fixed_all = fixed_all;
    nx.G = 0.0; nx.slack = 0.0; nx.notclose = notclose; nx.active = 0; nx.pad[0] = nx.pad[1] = 0;
    P.iters[t + 1] = nx;
    if (nx.stopped || t + 1 == P.max_iter) {
        amp_status s;
        s.T = t + 1; s.nan_state = fixed != 0 ? 1 : 0; s.stopped = nx.stopped;
        s.gemm = P.lx3 ? AMP_ARITH_BF16X3 : AMP_ARITH_F32;
        s.last_scalar[0] = s.last_scalar[1] = s.last_scalar[2] = s.last_scalar[3] = 0.f;
        *P.status = s;
    }
}

__global__ __launch_bounds__(SRWG) void scamp_r(ScampK P, Const64 c64, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    __shared__ double s_d[SRWG / 64];
    const ScampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) P.iters[t + 1] = cur;
        return;
    }
    PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk, P.nblk, lds);
    if (P.psi_split) {
        __shared__ unsigned s_u[SRWG / 64];
        unsigned nc = 0;
        for (int i = threadIdx.x; i < P.psi_nblk; i += blockDim.x) nc += P.psi_nc[(size_t)t * P.psi_nblk + i];
        pa.notclose += block_sum_u32(nc, s_u);
    }
    if (part_allnan(pa)) {
        if (!cur.fixed_all) {
            nan_fill(P.xm, nullptr, (size_t)P.B * P.N);
            float* psi_new = spsi(P, t);
            for (int e = threadIdx.x; e < P.B * P.Lin; e += blockDim.x) psi_new[e] = __int_as_float(0x7fc00000);
        }
        if (threadIdx.x == 0) scamp_finish(P, t, 1u, -1, 1);
    } else if (part_danger(pa)) {
        // exact float64 batch max |xi| over the candidate sections (those within the float32
        // estimate's slack of the float32 batch max)
        const double slack = logit_slack(pa.maxabs);
        const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
        const float* tau = P.tau;
        const int M = P.M, L = P.L, N = P.N, Nt = P.Nt, Lin = P.Lin;
        double gm = 0.0;
        for (int sct = threadIdx.x; sct < P.B * L; sct += blockDim.x) {
            if ((double)P.secabs[sct] < pa.maxabs - slack) continue;
            const size_t o0 = (size_t)sct * M;
            const int b = sct / L, lc = (int)((o0 % (size_t)N) / Nt);
            const float tv = tau[(size_t)b * Lin + lc];
            auto ld = [=](int m, float& rr, float& ri, float& it) {
                const float2 v = xp2[o0 + m];
                rr = v.x; ri = v.y; it = 1.0f / (tv * 0.5f);
            };
            gm = fmax(gm, section_absmax_f64(ld, M, c64));
        }
        gm = group_max(gm, 64);
        if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            double G = 0.0;
            for (int w = 0; w < SRWG / 64; ++w) G = fmax(G, s_d[w]);
            ScampIter nx;
            nx.stopped = 0; nx.T = t + 1; nx.fixed = 0; nx.fixed_all = 0;
            nx.G = G; nx.slack = slack; nx.notclose = pa.notclose; nx.active = 1; nx.pad[0] = nx.pad[1] = 0;
            P.iters[t + 1] = nx;
        }
    } else if (threadIdx.x == 0) {
        scamp_finish(P, t, pa.notclose, 0, 0);
    }
}

// per-block integer counts of the fix-up kernels, written over iteration t's partials (already
// consumed by scamp_r): slot i = {sections fixed, allclose delta} of block i
__device__ __forceinline__ int2* scamp_fix_counts(const ScampK& P, int t) {
    return reinterpret_cast<int2*>(P.parts + (size_t)t * P.nblk);
}

__device__ __forceinline__ int block_sum_int(int v, int* s_i) {
    v = group_sum(v, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_i[threadIdx.x >> 6] = v;
    __syncthreads();
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_i[w];
    return tot;
}

__global__ __launch_bounds__(AMP_WG) void scamp_fix_sec(ScampK P, Const64 c64, int t) {
    __shared__ int s_i[AMP_WG / 64];
    const ScampIter pend = P.iters[t + 1];
    if (!pend.active || P.iters[t].stopped) return;
    const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
    float2* x2 = reinterpret_cast<float2*>(P.xm);
    const int M = P.M, L = P.L, N = P.N, Nt = P.Nt, Lin = P.Lin;
    int cnt = 0;
    for (int sct = blockIdx.x * blockDim.x + threadIdx.x; sct < P.B * L; sct += gridDim.x * blockDim.x) {
        if (!((double)P.secmax[sct] - pend.G < AMP_DANGER + pend.slack)) continue;
        const size_t o0 = (size_t)sct * M;
        const int b = sct / L, lc = (int)((o0 % (size_t)N) / Nt);
        const float tv = P.tau[(size_t)b * Lin + lc];
        auto ld = [=](int m, float& rr, float& ri, float& it) {
            const float2 v = xp2[o0 + m];
            rr = v.x; ri = v.y; it = 1.0f / (tv * 0.5f);
        };
        auto st = [=](int m, float xr, float xi, float) { x2[o0 + m] = make_float2(xr, xi); };
        exact_section_f64<false>(ld, st, M, c64, pend.G);
        ++cnt;
    }
    cnt = block_sum_int(cnt, s_i);
    if (threadIdx.x == 0) scamp_fix_counts(P, t)[blockIdx.x].x = cnt;
}

__device__ __forceinline__ void scamp_fix_psi_body(const ScampK& P, int t, const ScampIter& pend, int* s_i) {
    const float* psi_prev = spsi(P, t + 1);
    float* psi_new = spsi(P, t);
    const int spb = P.Nt / P.M;   // sections per coupling block
    int dnc = 0;
    for (int blk = blockIdx.x * blockDim.x + threadIdx.x; blk < P.B * P.Lin; blk += gridDim.x * blockDim.x) {
        bool hit = false;
        for (int j = 0; j < spb && !hit; ++j)
            hit = (double)P.secmax[(size_t)blk * spb + j] - pend.G < AMP_DANGER + pend.slack;
        if (!hit) continue;
        const float2* xr = reinterpret_cast<const float2*>(P.xm) + (size_t)blk * P.Nt;
        double ssum = 0.0;
        for (int m = 0; m < P.Nt; ++m) {
            const float a = (float)sqrt((double)xr[m].x * xr[m].x + (double)xr[m].y * xr[m].y);
            ssum += (double)(a * a);
        }
        const float ps = 1.0f - (float)ssum / (float)P.Na;
        dnc += (torch_close(ps, psi_prev[blk]) ? 0 : 1) - (torch_close(psi_new[blk], psi_prev[blk]) ? 0 : 1);
        psi_new[blk] = ps;
    }
    dnc = block_sum_int(dnc, s_i);
    if (threadIdx.x == 0) scamp_fix_counts(P, t)[blockIdx.x].y = dnc;
}

__global__ __launch_bounds__(AMP_WG) void scamp_fix_psi(ScampK P, int t) {
    __shared__ int s_i[AMP_WG / 64];
    const ScampIter pend = P.iters[t + 1];
    if (!pend.active || P.iters[t].stopped) return;
    scamp_fix_psi_body(P, t, pend, s_i);
}

// scamp_fix_psi, then (last workgroup to arrive) scamp_fin's count and exit decision over both
// fix-up launches' per-block counts: one launch fewer per iteration.  scamp_fix_sec stays a launch
// of its own (one thread per section: the exact float64 recompute is the rare path's cost).
__global__ __launch_bounds__(AMP_WG) void scamp_fix_psi_fin(ScampK P, int t) {
    __shared__ int s_i[AMP_WG / 64];
    const ScampIter pend = P.iters[t + 1];
    if (!pend.active || P.iters[t].stopped) return;
    scamp_fix_psi_body(P, t, pend, s_i);
    if (last_arrival(P.rcnt + 1, gridDim.x)) {
        const int2* c = scamp_fix_counts(P, t);
        int fixed = 0, d = 0;
        for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) { fixed += c[i].x; d += c[i].y; }
        fixed = block_sum_int(fixed, s_i);
        d = block_sum_int(d, s_i);
        if (threadIdx.x == 0) scamp_finish(P, t, (uint32_t)((int)pend.notclose + d), fixed, 0);
    }
}

// ---- trial-sharded iteration (amp_scamp_run_sharded; SURVEY §8(e) exact-compat) ----
// scamp_r / scamp_fin split at their batch-global values, as the VAMP and BAMP stages: the
// denoiser's max|xi| / min section max (scamp.py:64) and the psi allclose count (scamp.py:105)
// after sxr1, the rare path's exact max|xi| after sxr2 (scamp_fix_sec / scamp_fix_psi then
// recompute this rank's sections and psi), the fix-up counts after sxr4.
__global__ __launch_bounds__(SRWG) void scamp_sxr1(ScampK P, int t) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    __shared__ unsigned s_u[SRWG / 64];
    XState* xs = P.xs;
    if (P.iters[t].stopped) {
        if (threadIdx.x == 0) { xs->sum[0] = xs->sum[1] = 0.0; xs->mx[0] = xs->mx[1] = 0.0; }
        return;
    }
    PartAcc pa = part_reduce_all(P.parts + (size_t)t * P.nblk, P.nblk, lds);
    if (P.psi_split) {
        unsigned nc = 0;
        for (int i = threadIdx.x; i < P.psi_nblk; i += blockDim.x) nc += P.psi_nc[(size_t)t * P.psi_nblk + i];
        pa.notclose += block_sum_u32(nc, s_u);
    }
    if (threadIdx.x == 0) {
        xs->sum[0] = 0.0;
        xs->sum[1] = (double)pa.notclose;
        xs->mx[0] = (pa.maxabs <= 1.7976931348623157e308) ? pa.maxabs : INFINITY;   // NaN / inf wins
        xs->mx[1] = (pa.minsecmax == pa.minsecmax) ? -pa.minsecmax : INFINITY;
    }
}

__global__ __launch_bounds__(SRWG) void scamp_sxr2(ScampK P, Const64 c64, int t) {
    __shared__ double s_d[SRWG / 64];
    XState* xs = P.xs;
    const ScampIter cur = P.iters[t];
    if (cur.stopped) {
        if (threadIdx.x == 0) { P.iters[t + 1] = cur; xs->mode = 0; xs->gmax[0] = 0.0; }
        return;
    }
    PartAcc pa;
    pa.notclose = (uint32_t)xs->sum[1];
    pa.maxabs = xs->mx[0];
    pa.minsecmax = -xs->mx[1];
    if (part_allnan(pa)) {
        if (!cur.fixed_all) {
            nan_fill(P.xm, nullptr, (size_t)P.B * P.N);
            float* psi_new = spsi(P, t);
            for (int e = threadIdx.x; e < P.B * P.Lin; e += blockDim.x) psi_new[e] = __int_as_float(0x7fc00000);
        }
        if (threadIdx.x == 0) { scamp_finish(P, t, 1u, -1, 1); xs->mode = 0; xs->gmax[0] = 0.0; }
    } else if (part_danger(pa)) {
        // this rank's exact float64 max |xi| over its candidate sections (scamp_r's first stage)
        const double slack = logit_slack(pa.maxabs);
        const float2* xp2 = reinterpret_cast<const float2*>(P.xmap);
        const float* tau = P.tau;
        const int M = P.M, L = P.L, N = P.N, Nt = P.Nt, Lin = P.Lin;
        double gm = 0.0;
        for (int sct = threadIdx.x; sct < P.B * L; sct += blockDim.x) {
            if ((double)P.secabs[sct] < pa.maxabs - slack) continue;
            const size_t o0 = (size_t)sct * M;
            const int b = sct / L, lc = (int)((o0 % (size_t)N) / Nt);
            const float tv = tau[(size_t)b * Lin + lc];
            gm = fmax(gm, section_absmax_f64([=](int m, float& rr, float& ri, float& it) {
                const float2 v = xp2[o0 + m];
                rr = v.x; ri = v.y; it = 1.0f / (tv * 0.5f);
            }, M, c64));
        }
        gm = group_max(gm, 64);
        if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = gm;
        __syncthreads();
        if (threadIdx.x == 0) {
            double G = 0.0;
            for (int w = 0; w < SRWG / 64; ++w) G = fmax(G, s_d[w]);
            xs->gmax[0] = G;
            xs->mode = 2;
            ScampIter nx;   // pending record: G is set to the global value by scamp_sxr3
            nx.stopped = 0; nx.T = t + 1; nx.fixed = 0; nx.fixed_all = 0;
            nx.G = G; nx.slack = slack; nx.notclose = pa.notclose; nx.active = 1; nx.pad[0] = nx.pad[1] = 0;
            P.iters[t + 1] = nx;
        }
    } else if (threadIdx.x == 0) {
        scamp_finish(P, t, pa.notclose, 0, 0);
        xs->mode = 0;
        xs->gmax[0] = 0.0;
    }
}

__global__ void scamp_sxr3(ScampK P, int t) {   // the global exact G into the pending record
    if (threadIdx.x == 0 && P.xs->mode == 2) P.iters[t + 1].G = P.xs->gmax[0];
}

__global__ __launch_bounds__(AMP_WG) void scamp_sxr4(ScampK P, int t, int nfix) {   // this rank's fix-up counts
    __shared__ int s_i[AMP_WG / 64];
    XState* xs = P.xs;
    if (xs->mode != 2) {
        if (threadIdx.x == 0) xs->fix[0] = xs->fix[1] = xs->fix[2] = 0.0;
        return;
    }
    const int2* c = scamp_fix_counts(P, t);
    int fixed = 0, dnc = 0;
    for (int i = threadIdx.x; i < nfix; i += blockDim.x) { fixed += c[i].x; dnc += c[i].y; }
    fixed = block_sum_int(fixed, s_i);
    dnc = block_sum_int(dnc, s_i);
    if (threadIdx.x == 0) { xs->fix[0] = 0.0; xs->fix[1] = (double)dnc; xs->fix[2] = (double)fixed; }
}

__global__ void scamp_sxr5(ScampK P, int t) {
    const XState* xs = P.xs;
    if (threadIdx.x != 0 || xs->mode != 2) return;
    const long long nc = (long long)xs->sum[1] + (long long)xs->fix[1];
    scamp_finish(P, t, (uint32_t)nc, (int)xs->fix[2], 0);
}

// Tracker (scamp.py:9-25): z = y, psi = 1, phi = inf, xmmse = 0
__global__ void scamp_init_kernel(ScampK P) {
    const size_t BN_ = (size_t)P.B * P.N, Bn = (size_t)P.B * P.n, BL = (size_t)P.B * P.Lout;
    const size_t tot = std::max(std::max(BN_, Bn), BL);
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
        if (e < BN_) reinterpret_cast<float2*>(P.xm)[e] = make_float2(0.f, 0.f);
        if (e < Bn) reinterpret_cast<float2*>(P.z)[e] = reinterpret_cast<const float2*>(P.y)[e];
        if (e < (size_t)P.B * P.Lin) P.psi1[e] = 1.0f;
        if (e < BL) P.phi[BL + e] = INFINITY;        // phi buffer of "iteration -1"
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        P.rcnt[0] = 0u; P.rcnt[1] = 0u;
        ScampIter it;
        it.stopped = 0; it.T = 0; it.fixed = 0; it.fixed_all = 0;
        it.G = 0.0; it.slack = 0.0; it.notclose = 0; it.active = 0; it.pad[0] = it.pad[1] = 0;
        P.iters[0] = it;
    }
}

__global__ void scamp_output_kernel(ScampK P) {
    const int T = P.status->T;
    if (((T - 1) & 1) == 0) return;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < (size_t)P.B * P.Lin;
         e += (size_t)gridDim.x * blockDim.x)
        P.psi0[e] = P.psi1[e];
}

static std::once_flag g_scamp_once;
static int g_scamp_rc = 0;

template <int KK>
static int scamp_kb_attrs() {
    int rc = set_lds_attr<128>((const void*)scamp_kb<128, KK>);
    if (!rc) rc = set_lds_attr<256>((const void*)scamp_kb<256, KK, GKC, true>);
    return rc ? rc : set_lds_attr<256>((const void*)scamp_kb<256, KK>);
}

// Block-banded A (the ISI operators): every tile reduces over a few coupling blocks only, so the
// 256-wide A chunk (half the LDS: four tiles per CU instead of two) costs no extra chunks there.
// AMP_SCAMP_KC=512 keeps the 512-wide chunk (A/B runs).
constexpr size_t SKC_LDS = GemmCfg<128, 256>::LDS_BYTES;   // the short-chunk tiles' LDS

static bool scamp_short_chunks(const ScampK& P) {
    static const bool off = [] {
        const char* e = diag_env("AMP_SCAMP_KC");
        return e && atoi(e) == 512;
    }();
    return P.bandA != nullptr && !off;
}

// the bf16x3 tiles run in the 128-wide short-chunk instantiations (their epilogues' LDS budget is
// the 256-chunk A block) with the staged planes' 48 KB, the 256-wide kb in its GKC instantiation
constexpr size_t SX3_LDS = x3_tile_lds<128, true>(GemmCfg<128, 256>::A_FLOATS - GemmCfg<128, 256>::CTILE_FLOATS);
static_assert(x3_tile_lds<256, true>(0) <= GemmCfg<256>::LDS_BYTES, "bf16x3 planes within the 256-wide tile's LDS");

// A rows -> six bf16 planes for the next bf16x3 GEMM (no-op launch once the loop has stopped)
static void scamp_split(const ScampK& P, const float* a, int lda, int K, int t, hipStream_t st) {
    const int wpr = (P.rows_pad / 4 < 2 * device_cu_count() && K >= 1024) ? 4 : 1;
    hipLaunchKernelGGL(x3_split_rows_kernel<true>, dim3(P.rows_pad * wpr / 4), dim3(256), 0, st, a, lda, P.B,
                       P.rows_pad, K, P.lap, &P.iters[t].stopped, wpr);
}

template <int KK>
static void launch_kb_kk(const ScampK& P, int gr, size_t ldsB, int t, hipStream_t st) {
    if (P.bn == 128 && P.lx3)
        hipLaunchKernelGGL((scamp_kb<128, KK, 256, true>), dim3(gr, P.ncpB / 128), dim3(AMP_WG), SX3_LDS, st, P, t);
    else if (P.lx3)
        hipLaunchKernelGGL((scamp_kb<256, KK, GKC, true>), dim3(gr, P.ncpB / 256), dim3(AMP_WG), ldsB, st, P, t);
    else if (P.bn == 128 && scamp_short_chunks(P))
        hipLaunchKernelGGL((scamp_kb<128, KK, 256>), dim3(gr, P.ncpB / 128), dim3(AMP_WG), SKC_LDS,
                           st, P, t);
    else if (P.bn == 128)
        hipLaunchKernelGGL((scamp_kb<128, KK>), dim3(gr, P.ncpB / 128), dim3(AMP_WG), ldsB, st, P, t);
    else
        hipLaunchKernelGGL((scamp_kb<256, KK>), dim3(gr, P.ncpB / 256), dim3(AMP_WG), ldsB, st, P, t);
}

static void launch_ka(const ScampK& P, int gr, int t, hipStream_t st) {
    if (P.lx3) {
        scamp_split(P, P.xm, 2 * P.N, P.N, t, st);
        hipLaunchKernelGGL((scamp_ka<256, true>), dim3(gr, P.ncpA / 128), dim3(AMP_WG), SX3_LDS, st, P, t);
    } else if (scamp_short_chunks(P))
        hipLaunchKernelGGL(scamp_ka<256>, dim3(gr, P.ncpA / 128), dim3(AMP_WG), SKC_LDS, st, P, t);
    else
        hipLaunchKernelGGL(scamp_ka<GKC>, dim3(gr, P.ncpA / 128), dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, P, t);
}

static void launch_kb(const ScampK& P, int gr, size_t ldsB, int t, hipStream_t st) {
    if (P.lx3) scamp_split(P, P.s, 2 * P.n, P.n, t, st);
    switch (P.c.K) {
    case 1: launch_kb_kk<1>(P, gr, ldsB, t, st); break;
    case 2: launch_kb_kk<2>(P, gr, ldsB, t, st); break;
    case 4: launch_kb_kk<4>(P, gr, ldsB, t, st); break;
    case 8: launch_kb_kk<8>(P, gr, ldsB, t, st); break;
    case 16: launch_kb_kk<16>(P, gr, ldsB, t, st); break;
    default: launch_kb_kk<64>(P, gr, ldsB, t, st); break;
    }
}

static int scamp_attrs() {
    std::call_once(g_scamp_once, [] {
        g_scamp_rc = set_lds_attr<128>((const void*)scamp_ka<GKC>);
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<1>();
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<2>();
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<4>();
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<8>();
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<16>();
        if (!g_scamp_rc) g_scamp_rc = scamp_kb_attrs<64>();
    });
    return g_scamp_rc;
}

}  // namespace amp

using namespace amp;

extern "C" {

size_t amp_scamp_workspace_bytes(const amp_dims* d, int32_t max_iter) {
    if (!d || max_iter <= 0) return 0;
    return scamp_carve(d, max_iter, nullptr).bytes;
}

}  // extern "C"

namespace amp {

// AMP_SCAMP_GEMM=f32: AMP_GEMM_AUTO keeps the f32-MFMA persistent GEMMs (A/B runs)
static bool scamp_gemm_f32_requested() {
    static const bool v = [] {
        const char* e = diag_env("AMP_SCAMP_GEMM");
        return e && e[0] == 'f';
    }();
    return v;
}

// AMP_SCAMP_GEMM=h2: AMP_GEMM_AUTO picks the fp16x2 persistent GEMMs instead of bf16x3 (A/B runs)
static bool scamp_gemm_h2_requested() {
    static const bool v = [] {
        const char* e = diag_env("AMP_SCAMP_GEMM");
        return e && e[0] == 'h';
    }();
    return v;
}

// Block-banded A (Lin > 1 or Lout > 1): the GEMMs skip the reduction blocks of each column tile
// that hold only zeros (weight_kband over the packed weights, once per forward).  Off with
// AMP_BAND_GEMM=0 (A/B runs).
static bool band_gemm_enabled() {
    static const bool on = [] {
        const char* e = diag_env("AMP_BAND_GEMM");
        return !(e && e[0] == '0');
    }();
    return on;
}

static int scamp_setup(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, ScampK& P,
                       Const64& c64) {
    int rc = check_dims(d, c);
    if (rc) return rc;
    AMP_REQUIRE(a && a->W && a->A && a->y && a->xmap && a->xmmse && a->psi && a->status && a->ws,
                "amp_scamp_run: null pointer argument");
    AMP_REQUIRE(a->max_iter > 0, "amp_scamp_run: max_iter must be positive");
    AMP_REQUIRE(is_pow2(d->Nt) && 2 * d->Nt <= 256, "amp_scamp_run: Nt = %d must be a power of two <= 128", d->Nt);
    AMP_REQUIRE(d->Lin <= SMAXLIN, "amp_scamp_run: Lin = %d > %d", d->Lin, SMAXLIN);
    const ScampWs w = scamp_carve(d, a->max_iter, a->ws);
    AMP_REQUIRE(a->ws_bytes >= w.bytes, "amp_scamp_run: workspace %zu < %zu bytes", a->ws_bytes, w.bytes);
    rc = scamp_attrs();
    if (rc) return rc;
    scamp_geometry(d, P);
    P.max_iter = a->max_iter;
    P.sigma2 = (float)a->noise_var;
    P.W = (const float*)a->W;
    P.WA = w.WA; P.WAH = w.WAH;
    // block-banded A: the ranges are formed by the prepare launch sequence (every later call of
    // the layer-level API reads them from the workspace)
    const bool band = (d->Lin > 1 || d->Lout > 1) && band_gemm_enabled();
    P.bandA = band ? w.bandA : nullptr;
    P.bandB = band ? w.bandB : nullptr;
    P.xs = w.xs;
    P.y = (const float*)a->y; P.z = w.z; P.s = w.s; P.phi = w.phi; P.tau = w.tau;
    P.xmap = (float*)a->xmap; P.xm = (float*)a->xmmse; P.psi0 = (float*)a->psi; P.psi1 = w.psi1;
    P.secmax = w.secmax; P.secabs = w.secabs; P.parts = w.parts; P.iters = w.iters; P.status = (amp_status*)a->status;
    P.psi_nc = w.psi_nc; P.psi_nblk = scamp_psi_nblk(d); P.psi_split = (P.bn / 2 < P.Nt) ? 1 : 0;
    P.nwg = cdiv(d->B, 16);
    P.gen = 0;
    P.Wq1 = w.Wq1; P.Wq2 = w.Wq2; P.pparts = w.pparts; P.pxch = w.pxch; P.pbar = w.pbar;
    P.Wx1 = w.Wx1; P.Wx2 = w.Wx2;
    P.dec_on = 0; P.ibits = 0; P.xtrue = nullptr; P.sym = nullptr; P.idx = nullptr; P.counts = nullptr;
    P.host_rec = nullptr;
    P.fold_in = fold_in_kernel() ? 1 : 0;
    P.dwg = w.dwg;
    P.trace = nullptr;
    P.rcnt = w.pbar + 8;
    P.c = to_const(c);
    c64 = to_const64(c);
    AMP_REQUIRE(a->gemm >= AMP_GEMM_AUTO && a->gemm <= AMP_GEMM_H2, "amp_scamp: gemm %d", a->gemm);
    const bool fits = scamp_persist_x3_fits(d), lx3ok = scamp_lx3_shape(d);
    AMP_REQUIRE(a->gemm != AMP_GEMM_H2 || fits, "amp_scamp: the split-precision engine's LDS carve exceeds 160 KB");
    AMP_REQUIRE(a->gemm != AMP_GEMM_X3 || fits || lx3ok,
                "amp_scamp: bf16x3 needs the persistent engine's LDS carve within 160 KB or, on the launch engine, "
                "N %% 64 == 0 and n %% 64 == 0 (N = %d, n = %d)", d->N, d->n);
    // launch engine: bf16x3 tiles when asked for (AMP_GEMM_X3) or, under AUTO, with
    // AMP_SCAMP_LAUNCH_GEMM=x3; f32 MFMA tiles otherwise
    static const bool lx3_env = [] {
        const char* e = diag_env("AMP_SCAMP_LAUNCH_GEMM");
        return e && e[0] == 'x';
    }();
    P.lx3 = lx3ok && (a->gemm == AMP_GEMM_X3 || (a->gemm == AMP_GEMM_AUTO && lx3_env)) ? 1 : 0;
    P.rows_pad = round_up(d->B, GBM);
    P.lap = w.lap;
    // 0 f32 MFMA, 1 bf16x3, 2 fp16x2.  AUTO keeps bf16x3 for SCAMP: with fp16x2 one cfg3 golden
    // (QPSK, 7 dB, seed 1) never meets the psi allclose exit (T 20 vs the reference's 6, VER / SER
    // equal): at nMSE 1e-9 psi is ~1e-9 and torch.allclose's atol 1e-8 decides, which the
    // fp16x2 products' 2^-22 terms move.  AMP_SCAMP_GEMM=f32 / h2 for A/B runs.
    P.x3 = a->gemm == AMP_GEMM_H2 ? 2 : a->gemm == AMP_GEMM_X3 ? (fits ? 1 : 0) : a->gemm == AMP_GEMM_F32 || !fits ? 0
         : scamp_gemm_f32_requested() ? 0 : scamp_gemm_h2_requested() ? 2 : 1;
    return AMP_OK;
}

// The persistent engine's operators (16x16x4-packed A and A^H) and zeroed barrier words, in one
// launch; a fresh generation for the granule tags.
static int scamp_persist_prepare(ScampK& P, const amp_scamp_args* a, hipStream_t st) {
    static std::atomic<unsigned> gen{0};
    P.gen = ++gen;
    CWeightJob j[2];
    if (P.x3) {
        const int pk = P.x3 == 2 ? WPACKH2 : WPACKX3;
        //   A x     (scamp.py:47)   X[o][j] = A[o][j],        o < n, j < N   (bf16x3 / fp16x2 planes)
        j[0] = CWeightJob{(const float2*)a->A, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.Wx1, P.N, P.n, pk, SH2_EX};
        //   A^H s   (scamp.py:57)   X[o][j] = conj(A[j][o]),  o < N, j < n
        j[1] = CWeightJob{(const float2*)a->A, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.Wx2, P.n, P.N, pk, SH2_EX};
        return build_cweights(j, 2, P.pbar, 64, st);
    }
    //   A x       (scamp.py:47)   X[o][j] = A[o][j],        o < n, j < N
    j[0] = CWeightJob{(const float2*)a->A, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.Wq1, 2 * P.N, 2 * P.n, WPACK16};
    //   A^H s     (scamp.py:57)   X[o][j] = conj(A[j][o]),  o < N, j < n
    j[1] = CWeightJob{(const float2*)a->A, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.Wq2, 2 * P.n, 2 * P.N, WPACK16};
    return build_cweights(j, 2, P.pbar, 64, st);
}

// Tracker (scamp.py:9-25): the two weights and the initial state.
static int scamp_prepare_impl(const ScampK& P, const amp_scamp_args* a, hipStream_t st) {
    int rc;
    const float2* A = (const float2*)a->A;
    if (P.lx3) {
        // bf16x3 planes (x3_index) in the f32 weights' buffers (12 of their 16 bytes per entry):
        // A x (O = n, J = N), A^H s (O = N, J = n)
        CWeightJob j[2];
        j[0] = CWeightJob{A, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.WA, P.N, P.n, WPACKX3, 0};
        j[1] = CWeightJob{A, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.WAH, P.n, P.N, WPACKX3, 0};
        if ((rc = build_cweights(j, 2, nullptr, 0, st))) return rc;
        if (P.bandA) {
            if ((rc = h2_kband(P.WA, 6, P.N / 32, 4, P.ncpA / 128, P.n / 16, const_cast<int*>(P.bandA), st))) return rc;
            if ((rc = h2_kband(P.WAH, 6, P.n / 32, P.bn / 32, P.ncpB / P.bn, P.N / 16, const_cast<int*>(P.bandB), st)))
                return rc;
        }
    } else {
    if ((rc = build_cweight(A, P.N, 1, 0, nullptr, P.n, P.N, (float*)P.WA, P.kapA, P.ncpA, st))) return rc;
    if ((rc = build_cweight(A, 1, P.N, 1, nullptr, P.N, P.n, (float*)P.WAH, P.kapB, P.ncpB, st))) return rc;
    }
    if (P.bandA && !P.lx3) {
        if ((rc = weight_kband(P.WA, P.kapA, P.ncpA, 128, const_cast<int*>(P.bandA), st))) return rc;
        if ((rc = weight_kband(P.WAH, P.kapB, P.ncpB, P.bn, const_cast<int*>(P.bandB), st))) return rc;
    }
    const size_t tot = std::max(std::max((size_t)P.B * P.N, (size_t)P.B * P.n), (size_t)P.B * P.Lout);
    hipLaunchKernelGGL(scamp_init_kernel, dim3((int)std::min<size_t>((tot + 255) / 256, 2048)), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("scamp_init");
    return AMP_OK;
}

// One SCAMPLayer.forward (scamp.py:43-59) + the allclose(psi) test of scamp.py:105: the two GEMM
// launches (+ scamp_psi when a tile holds part of a coupling block), the batch reduction and the
// rare path's fix-up with its exit decision (scamp_fix_sec, scamp_fix_psi_fin: they return at once
// unless scamp_r left a pending record).  The reduction keeps a launch of its own: folded into the last workgroup of
// the GEMM launch it needs an agent-scope release per workgroup (an L2 write-back on every XCD),
// which cost more than the launch (scamp_psi 6.9 -> 40 us at the ISI shape).
static int scamp_iterate_impl(const ScampK& P, const Const64& c64, int t, hipStream_t st) {
    const int gr = cdiv(P.B, GBM);
    const size_t ldsB = (P.bn == 128 ? GemmCfg<128>::LDS_BYTES : GemmCfg<256>::LDS_BYTES);
    // fix-up grid: one slot per block in iteration t's partials (consumed by then)
    const int nfix = fix_grid(P.nblk, P.B * P.L);
    launch_ka(P, gr, t, st);
    launch_kb(P, gr, ldsB, t, st);
    if (P.psi_split)
        hipLaunchKernelGGL(scamp_psi, dim3(P.psi_nblk), dim3(AMP_WG), 0, st, P, t);
    hipLaunchKernelGGL(scamp_r, dim3(1), dim3(SRWG), 0, st, P, c64, t);
    hipLaunchKernelGGL(scamp_fix_sec, dim3(nfix), dim3(AMP_WG), 0, st, P, c64, t);
    hipLaunchKernelGGL(scamp_fix_psi_fin, dim3(nfix), dim3(AMP_WG), 0, st, P, t);
    AMP_LAUNCH_CHECK("scamp iteration");
    return AMP_OK;
}

static int scamp_iterate_sharded(const ScampK& P, const Const64& c64, int t, hipStream_t st, bool& hook_failed) {
    const int gr = cdiv(P.B, GBM);
    const size_t ldsB = (P.bn == 128 ? GemmCfg<128>::LDS_BYTES : GemmCfg<256>::LDS_BYTES);
    const int nfix = fix_grid(P.nblk, P.B * P.L);
    launch_ka(P, gr, t, st);
    launch_kb(P, gr, ldsB, t, st);
    if (P.psi_split) hipLaunchKernelGGL(scamp_psi, dim3(P.psi_nblk), dim3(AMP_WG), 0, st, P, t);
    hipLaunchKernelGGL(scamp_sxr1, dim3(1), dim3(SRWG), 0, st, P, t);
    AMP_LAUNCH_CHECK("scamp_sxr1");
    // every hook call is made on every rank even after one failed: the ranks' collectives stay
    // matched and a failed rank's poisoned words reach the others (amp_sparc.h)
    hook_failed |= call_allreduce_hook(P.xs->sum, 2, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hook_failed |= call_allreduce_hook(P.xs->mx, 2, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(scamp_sxr2, dim3(1), dim3(SRWG), 0, st, P, c64, t);
    AMP_LAUNCH_CHECK("scamp_sxr2");
    hook_failed |= call_allreduce_hook(P.xs->gmax, 1, AMP_ALLREDUCE_MAX, st) != AMP_OK;
    hipLaunchKernelGGL(scamp_sxr3, dim3(1), dim3(64), 0, st, P, t);
    hipLaunchKernelGGL(scamp_fix_sec, dim3(nfix), dim3(AMP_WG), 0, st, P, c64, t);
    hipLaunchKernelGGL(scamp_fix_psi, dim3(nfix), dim3(AMP_WG), 0, st, P, t);
    hipLaunchKernelGGL(scamp_sxr4, dim3(1), dim3(AMP_WG), 0, st, P, t, nfix);
    AMP_LAUNCH_CHECK("scamp_sxr4");
    hook_failed |= call_allreduce_hook(P.xs->fix, 3, AMP_ALLREDUCE_SUM, st) != AMP_OK;
    hipLaunchKernelGGL(scamp_sxr5, dim3(1), dim3(64), 0, st, P, t);
    AMP_LAUNCH_CHECK("scamp_sxr5");
    return AMP_OK;
}

static int scamp_finalize_impl(const ScampK& P, hipStream_t st) {
    hipLaunchKernelGGL(scamp_output_kernel, dim3(64), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("scamp_output");
    return AMP_OK;
}

__global__ __launch_bounds__(1024) void vamp_decide_fold(const DecWG* w, int n, amp_counts* out);   // amp_vamp_persist.hip

}  // namespace amp

extern "C" {

int amp_scamp_select_engine(const amp_dims* d, int32_t engine) {
    if (!d) return AMP_E_ARG;
    const bool elig = scamp_persist_eligible(d, device_cu_count());
    if (engine == AMP_ENGINE_PERSISTENT) return elig ? AMP_ENGINE_PERSISTENT : AMP_E_ARG;
    if (engine == AMP_ENGINE_AUTO && elig) return AMP_ENGINE_PERSISTENT;
    return engine == AMP_ENGINE_AUTO || engine == AMP_ENGINE_LAUNCHES ? AMP_ENGINE_LAUNCHES : AMP_E_ARG;
}

int amp_scamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a,
                          int32_t B_global, void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(allreduce_hook_set(), "amp_scamp_run_sharded: no all-reduce hook registered (amp_set_allreduce_hook)");
    AMP_REQUIRE(B_global >= d->B, "amp_scamp_run_sharded: B_global = %d < this rank's B = %d", B_global, d->B);
    hipStream_t st = (hipStream_t)stream;
    if ((rc = scamp_prepare_impl(P, a, st))) return rc;
    bool hook_failed = false;
    for (int t = 0; t < P.max_iter && !rc; ++t) rc = scamp_iterate_sharded(P, c64, t, st, hook_failed);
    if (!rc && hook_failed) rc = hook_failure("scamp");
    return rc ? rc : scamp_finalize_impl(P, st);
}

int amp_scamp_run(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    AMP_REQUIRE(a->engine >= AMP_ENGINE_AUTO && a->engine <= AMP_ENGINE_PERSISTENT, "amp_scamp_run: engine %d",
                a->engine);
    const bool elig = scamp_persist_eligible(d, device_cu_count());
    AMP_REQUIRE(a->engine != AMP_ENGINE_PERSISTENT || elig,
                "amp_scamp_run: persistent engine needs (2N, 2n) in {(128, 256), (256, 512), (256, 256)}, M <= 64 "
                "and ceil(B/16) = %d <= %d CUs", cdiv(d->B, 16), device_cu_count());
    if (a->engine == AMP_ENGINE_PERSISTENT || (a->engine == AMP_ENGINE_AUTO && elig)) {
        AMP_REQUIRE(a->gemm != AMP_GEMM_X3 || scamp_persist_x3_fits(d),
                    "amp_scamp_run: the persistent bf16x3 engine's LDS carve exceeds 160 KB");
        if ((rc = scamp_persist_prepare(P, a, st))) return rc;
        DecConst dc;
        static_cast<Const64&>(dc) = c64;   // no decision in this launch: only the float64 table is read
        return scamp_persist_launch(P, dc, st);
    }
    if ((rc = scamp_prepare_impl(P, a, st))) return rc;
    for (int t = 0; t < P.max_iter; ++t)
        if ((rc = scamp_iterate_impl(P, c64, t, st))) return rc;
    return scamp_finalize_impl(P, st);
}

// Diagnostic: one persistent-engine forward whose workgroups stamp s_memtime at every phase
// boundary: trace[(wg * max_iter + t) * 10 + phase] (phases: amp_scamp_persist_kernel.h).
int amp_scamp_persist_trace(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* trace,
                            void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(trace && scamp_persist_eligible(d, device_cu_count()), "amp_scamp_persist_trace: not eligible / null trace");
    hipStream_t st = (hipStream_t)stream;
    if ((rc = scamp_persist_prepare(P, a, st))) return rc;
    P.trace = (unsigned long long*)trace;
    DecConst dc;
    static_cast<Const64&>(dc) = c64;
    return scamp_persist_launch(P, dc, st);
}

int amp_scamp_detect_count(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a,
                           const amp_vamp_decide_args* dec, void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(dec && dec->x && dec->sym && dec->idx && dec->counts, "amp_scamp_detect_count: null pointer argument");
    AMP_REQUIRE(dec->ibits_trunc >= 0 && dec->ibits_trunc < 64, "amp_scamp_detect_count: ibits_trunc out of range");
    AMP_REQUIRE(d->Lin * d->Na * d->M == d->N, "amp_scamp_detect_count: inconsistent dims");
    AMP_REQUIRE(a->engine != AMP_ENGINE_LAUNCHES && scamp_persist_eligible(d, device_cu_count()),
                "amp_scamp_detect_count: needs the persistent engine ((2N, 2n) in {(128, 256), (256, 512), "
                "(256, 256)}, M <= 64, ceil(B/16) = %d <= %d CUs)", cdiv(d->B, 16), device_cu_count());
    hipStream_t st = (hipStream_t)stream;
    if ((rc = scamp_persist_prepare(P, a, st))) return rc;
    P.dec_on = 1;
    P.ibits = dec->ibits_trunc;
    P.xtrue = (const float2*)dec->x;
    P.sym = (const long long*)dec->sym;
    P.idx = (const long long*)dec->idx;
    P.counts = (amp_counts*)dec->counts;
    P.host_rec = P.fold_in ? (unsigned char*)dec->host_record : nullptr;
    DecConst dc = to_decconst(c);
    static_cast<Const64&>(dc) = c64;
    if ((rc = scamp_persist_launch(P, dc, st))) return rc;   // the counter records folded inside it ...
    if (P.fold_in) return AMP_OK;
    hipLaunchKernelGGL(vamp_decide_fold, dim3(1), dim3(256), 0, st, (const DecWG*)P.dwg, P.nwg, P.counts);   // ... or here
    AMP_LAUNCH_CHECK("vamp_decide_fold (scamp)");
    return AMP_OK;
}

int amp_scamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    return rc ? rc : scamp_prepare_impl(P, a, (hipStream_t)stream);
}

int amp_scamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, int32_t t,
                      void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    if (rc) return rc;
    AMP_REQUIRE(t >= 0 && t < a->max_iter, "amp_scamp_iterate: t = %d outside [0, %d)", t, a->max_iter);
    return scamp_iterate_impl(P, c64, t, (hipStream_t)stream);
}

int amp_scamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream) {
    ScampK P;
    Const64 c64;
    int rc = scamp_setup(d, c, a, P, c64);
    return rc ? rc : scamp_finalize_impl(P, (hipStream_t)stream);
}

}  // extern "C"
