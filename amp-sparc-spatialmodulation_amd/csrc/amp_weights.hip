// amp_weights.hip — expanded-weight builders, the plain-store GEMM, error state.
#include <stdarg.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

#include "amp_gemm.h"
#include <hip/hip_ext.h>

#include "amp_host.h"
#include "amp_gemm_h2.h"
#include "amp_persist.h"

namespace amp {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_dims(const amp_dims* d, const amp_constellation* c, bool tiled) {
    AMP_REQUIRE(d && c, "null dims/constellation");
    AMP_REQUIRE(d->B > 0 && d->Nt > 0 && d->Na > 0 && d->Nr > 0 && d->Lin > 0 && d->Lout > 0, "non-positive dimension");
    AMP_REQUIRE(d->Nt % d->Na == 0, "Na must divide Nt (config.py:133)");
    AMP_REQUIRE(d->M == d->Nt / d->Na && d->L == d->Na * d->Lin && d->N == d->Nt * d->Lin && d->n == d->Nr * d->Lout,
                "inconsistent derived dimensions");
    AMP_REQUIRE(is_pow2(d->M), "section size M = Nt/Na = %d must be a power of two", d->M);
    AMP_REQUIRE(c->K >= 1 && c->K <= AMP_MAX_K && is_pow2(c->K) && c->K != 32,
                "constellation size K = %d must be 1, 2, 4, 8, 16 or 64", c->K);
    AMP_REQUIRE(c->K <= 16 || d->M <= 64, "64-point constellations need M = Nt/Na <= 64 (M = %d)", d->M);
    if (!tiled) return AMP_OK;   // the decision / standalone denoiser have no GEMM tiling
    AMP_REQUIRE(2 * d->M <= 256, "section size M = %d > 128 not supported by the fused detectors", d->M);
    AMP_REQUIRE(d->N % 2 == 0 && d->n % 2 == 0, "N (%d) and n (%d) must be even", d->N, d->n);
    const int bn = section_bn(d);
    AMP_REQUIRE(2 * d->N <= bn || (2 * d->N) % bn == 0, "2N = %d must be <= %d or a multiple of it", 2 * d->N, bn);
    return AMP_OK;
}

__device__ __forceinline__ size_t widx(int n, int k, int kap, int packed) {
    return packed == WPACK32 ? wpack_index(n, k, kap) : packed == WPACK16 ? wpack16_index(n, k, kap)
                                                                           : (size_t)n * kap + k;
}

// Wt[2o][2j] = Re X, Wt[2o][2j+1] = -Im X, Wt[2o+1][2j] = Im X, Wt[2o+1][2j+1] = Re X,
// X[o][j] = rowscale[o] * op(src[o*so + j*sj]), op = conj if `conj`; zero padding up to [ncp][kap].
// packed: WPACK32 / WPACK16 = the MFMA-packed layouts the GEMM engines stream (amp_gemm.h),
// WPACK_NONE = row-major.
// rowscale multiplies like the reference's `s.view(-1,1) * Uh` (f32 x c64 -> per-component products).
__global__ void build_cweight_kernel(const float2* __restrict__ src, long so, long sj, int conj,
                                     const float* __restrict__ rowscale, int O, int J, float* __restrict__ wt,
                                     int kap, int ncp, int packed) {
    const long total = (long)(ncp / 2) * (kap / 2);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int o = (int)(e / (kap / 2)), j = (int)(e % (kap / 2));
        float xr = 0.f, xi = 0.f;
        if (o < O && j < J) {
            const float2 v = src[o * so + j * sj];
            xr = v.x;
            xi = conj ? -v.y : v.y;
            if (rowscale) {
                const float s = rowscale[o];
                xr = s * xr;
                xi = s * xi;
            }
        }
        wt[widx(2 * o, 2 * j, kap, packed)] = xr;
        wt[widx(2 * o, 2 * j + 1, kap, packed)] = -xi;
        wt[widx(2 * o + 1, 2 * j, kap, packed)] = xi;
        wt[widx(2 * o + 1, 2 * j + 1, kap, packed)] = xr;
    }
}

// Wt[o][j] = |src[o*so + j*sj]|^2 with torch's complex abs (correctly rounded hypot) then an
// f32 square (bamp.py:18 `H.abs()**2`).
__global__ void build_abs2_kernel(const float2* __restrict__ src, long so, long sj, int O, int J,
                                  float* __restrict__ wt, int kap, int ncp) {   // always packed
    const long total = (long)ncp * kap;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int o = (int)(e / kap), j = (int)(e % kap);
        float v = 0.f;
        if (o < O && j < J) {
            const float2 z = src[o * so + j * sj];
            const float a = (float)sqrt((double)z.x * z.x + (double)z.y * z.y);
            v = a * a;
        }
        wt[wpack_index(o, j, kap)] = v;
    }
}

// row-major [ncp][kap] -> MFMA-packed
__global__ void pack_weight_kernel(const float* __restrict__ src, float* __restrict__ dst, int kap, int ncp) {
    const long total = (long)ncp * kap;
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x)
        dst[wpack_index((int)(e / kap), (int)(e % kap), kap)] = src[e];
}

int build_cweight(const float2* src, long so, long sj, int conj, const float* rowscale, int O, int J, float* wt,
                  int kap, int ncp, hipStream_t st, int packed) {
    AMP_REQUIRE(packed == WPACK_NONE || (kap % GBK == 0 && ncp % 128 == 0) ||
                    (packed == WPACK16 && kap % 16 == 0 && ncp % 16 == 0),
                "build_cweight: kap %d / ncp %d not tiled", kap, ncp);
    const long total = (long)(ncp / 2) * (kap / 2);
    const int grid = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(build_cweight_kernel, dim3(grid), dim3(256), 0, st, src, so, sj, conj, rowscale, O, J, wt,
                       kap, ncp, packed);
    AMP_LAUNCH_CHECK("build_cweight");
    return AMP_OK;
}

struct CWeightJobs {
    CWeightJob j[CW_MAX_JOBS];
    unsigned* zero;
    int nzero;
};

__global__ void build_cweights_kernel(CWeightJobs P) {
    const CWeightJob J = P.j[blockIdx.y];
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < P.nzero; i += blockDim.x) P.zero[i] = 0u;
    if (J.packed == WPACKX3) {
        // bf16x3 planes of X itself (no real expansion): kap = J, ncp = O (complex counts).  Lane l
        // of (tile ct, group g) holds X[16 ct + (l & 15)][32 g + 8 (l >> 4) .. + 7] (x3_index) as one
        // 16-byte chunk per plane; thread e takes the element pair e & 3 of chunk e >> 2 (lane
        // (e >> 2) & 63 of block e >> 8) and writes its 4-byte word of every plane: consecutive
        // threads write consecutive words (1 KB per plane per 256 threads), and the launch has
        // enough threads to cover the load latency (one per chunk was latency-bound: 7.4 us)
        unsigned* w3 = reinterpret_cast<unsigned*>(J.wt);
        const int gpt = J.kap >> 5;                               // groups per 16-column tile
        const long tot = (long)(J.ncp >> 4) * gpt * 256;
        for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
            const int part = (int)(e & 3), l = (int)((e >> 2) & 63);
            const long blk = e >> 8;
            const int ct = (int)(blk / gpt), g = (int)(blk - (long)ct * gpt);
            const int o = 16 * ct + (l & 15), j0 = 32 * g + 8 * (l >> 4) + 2 * part;
            float xr[2], xi[2];
            const float s = (J.rowscale && o < J.O) ? J.rowscale[o] : 1.0f;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = j0 + q;
                float a = 0.f, b = 0.f;
                if (o < J.O && j < J.J) {
                    const float2 v = J.src[o * J.so + j * J.sj];
                    a = v.x;
                    b = J.conj ? -v.y : v.y;
                    if (J.rowscale) {
                        a = s * a;
                        b = s * b;
                    }
                }
                xr[q] = a;
                xi[q] = b;
            }
            unsigned c[6];
            split3x2(xr[0], xr[1], c[0], c[1], c[2]);
            split3x2(xi[0], xi[1], c[3], c[4], c[5]);
            unsigned* dst = w3 + ((size_t)blk * 6 * 64 + l) * 4 + part;
#pragma unroll
            for (int f = 0; f < 6; ++f) dst[f * 256] = c[f];   // plane f: 64 chunks of 4 words
        }
        return;
    }
    if (J.packed == WPACKI8) {
        // int8x4 digit planes of X (amp_persist.h gemm_i8): kap = J, ncp = O (complex counts).  One
        // block per output column o: the column's max |value| (re and im) sets its exponent e_o,
        // every value becomes rint(x 2^(30 - e_o)) and its four balanced base-256 digits.
        signed char* w8 = reinterpret_cast<signed char*>(J.wt);
        int* ecol = reinterpret_cast<int*>(w8 + i8_exp_offset(J.ncp, J.kap));
        __shared__ float s_m[256 / 64];
        for (int o = blockIdx.x; o < J.ncp; o += gridDim.x) {
            auto val = [&](int j, float& xr, float& xi) {
                xr = 0.f; xi = 0.f;
                if (o < J.O && j < J.J) {
                    const float2 v = J.src[o * J.so + j * J.sj];
                    xr = v.x;
                    xi = J.conj ? -v.y : v.y;
                    if (J.rowscale) {
                        const float sc = J.rowscale[o];
                        xr = sc * xr;
                        xi = sc * xi;
                    }
                }
            };
            float m = 0.f;
            for (int j = threadIdx.x; j < J.kap; j += blockDim.x) {
                float xr, xi;
                val(j, xr, xi);
                m = i8_absmax(i8_absmax(m, xr), xi);
            }
            for (int sh = 32; sh >= 1; sh >>= 1) m = fmaxf(m, __shfl_xor(m, sh));
            __syncthreads();
            if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
            __syncthreads();
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmaxf(m, s_m[w]);
            // a non-finite operator column: its digits are zero and its exponent makes the column
            // factor inf (the GEMM's results are then non-finite, never silently wrong)
            const int e = i8_row_exp(m);
            if (threadIdx.x == 0) ecol[o] = e == 0x7fffffff ? 200 : e;
            for (int j = threadIdx.x; j < J.kap; j += blockDim.x) {
                float xr, xi;
                val(j, xr, xi);
                const int vr = i8_fix(xr, e), vi = i8_fix(xi, e);
                w8[i8_index(o, j, 0, J.kap)] = (signed char)((vr + 0x808080) >> 24);
                w8[i8_index(o, j, 1, J.kap)] = (signed char)((vr + 0x8080) >> 16);
                w8[i8_index(o, j, 2, J.kap)] = (signed char)((vr + 0x80) >> 8);
                w8[i8_index(o, j, 3, J.kap)] = (signed char)vr;
                w8[i8_index(o, j, 4, J.kap)] = (signed char)((vi + 0x808080) >> 24);
                w8[i8_index(o, j, 5, J.kap)] = (signed char)((vi + 0x8080) >> 16);
                w8[i8_index(o, j, 6, J.kap)] = (signed char)((vi + 0x80) >> 8);
                w8[i8_index(o, j, 7, J.kap)] = (signed char)vi;
            }
        }
        return;
    }
    if (J.packed == WPACKH2) {
        // fp16x2 planes of X 2^ex (amp_persist.h gemm_h2): kap = J, ncp = O (complex counts).
        // |x| 2^ex >= 65520 leaves fp16's range: the piece is then inf, so the GEMM's result is
        // non-finite (never silently wrong); VAMP's SVD factors have |x| <= 1 (ex = 14), SCAMP's
        // channel entries are ~CN(0, 1/Nr) (ex = 10: |x| < 64).
        unsigned short* w2 = reinterpret_cast<unsigned short*>(J.wt);
        const long tot = (long)J.ncp * J.kap;
        for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
            const int o = (int)(e / J.kap), j = (int)(e % J.kap);
            float xr = 0.f, xi = 0.f;
            if (o < J.O && j < J.J) {
                const float2 v = J.src[o * J.so + j * J.sj];
                xr = v.x;
                xi = J.conj ? -v.y : v.y;
                if (J.rowscale) {
                    const float s = J.rowscale[o];
                    xr = s * xr;
                    xi = s * xi;
                }
            }
            unsigned p[4];
            split2(xr, J.ex, p[0], p[1]);
            split2(xi, J.ex, p[2], p[3]);
#pragma unroll
            for (int f = 0; f < 4; ++f) w2[h2_index(o, j, f, J.kap)] = (unsigned short)p[f];
        }
        return;
    }
    if (J.packed == WPACKH2_ABS2) {
        // fp16x2 planes of the real |X|^2 (torch's complex abs, the correctly rounded hypot, then
        // an f32 square: bamp.py:18 `H.abs()**2`), scaled by 2^ex (gemm_tile_h2, amp_gemm_h2.h)
        unsigned short* w2 = reinterpret_cast<unsigned short*>(J.wt);
        const long tot = (long)J.ncp * J.kap;
        for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
            const int o = (int)(e / J.kap), j = (int)(e % J.kap);
            float v = 0.f;
            if (o < J.O && j < J.J) {
                const float2 z = J.src[o * J.so + j * J.sj];
                const float a = (float)sqrt((double)z.x * z.x + (double)z.y * z.y);
                v = a * a;
            }
            unsigned p0, p1;
            split2(v, J.ex, p0, p1);
            w2[h2r_index(o, j, 0, J.kap)] = (unsigned short)p0;
            w2[h2r_index(o, j, 1, J.kap)] = (unsigned short)p1;
        }
        return;
    }
    if (J.packed == WPACKX3_ABS2) {
        // bf16x3 planes of the real |X|^2 (torch's complex abs, the correctly rounded hypot, then an
        // f32 square: bamp.py:18 `H.abs()**2`) for gemm_tile_x3 (amp_gemm_x3.h)
        unsigned short* w3 = reinterpret_cast<unsigned short*>(J.wt);
        const long tot = (long)J.ncp * J.kap;
        for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
            const int o = (int)(e / J.kap), j = (int)(e % J.kap);
            float v = 0.f;
            if (o < J.O && j < J.J) {
                const float2 z = J.src[o * J.so + j * J.sj];
                const float a = (float)sqrt((double)z.x * z.x + (double)z.y * z.y);
                v = a * a;
            }
            unsigned p[3];
            split3(v, p[0], p[1], p[2]);
#pragma unroll
            for (int f = 0; f < 3; ++f) w3[x3r_index(o, j, f, J.kap)] = (unsigned short)p[f];
        }
        return;
    }
    const long total = (long)(J.ncp / 2) * (J.kap / 2);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int o = (int)(e / (J.kap / 2)), j = (int)(e % (J.kap / 2));
        float xr = 0.f, xi = 0.f;
        if (o < J.O && j < J.J) {
            const float2 v = J.src[o * J.so + j * J.sj];
            xr = v.x;
            xi = J.conj ? -v.y : v.y;
            if (J.rowscale) {
                const float s = J.rowscale[o];
                xr = s * xr;
                xi = s * xi;
            }
        }
        J.wt[widx(2 * o, 2 * j, J.kap, J.packed)] = xr;
        J.wt[widx(2 * o, 2 * j + 1, J.kap, J.packed)] = -xi;
        J.wt[widx(2 * o + 1, 2 * j, J.kap, J.packed)] = xi;
        J.wt[widx(2 * o + 1, 2 * j + 1, J.kap, J.packed)] = xr;
    }
}

int build_cweights(const CWeightJob* jobs, int njobs, unsigned* zero, int nzero, hipStream_t st) {
    AMP_REQUIRE(njobs >= 1 && njobs <= CW_MAX_JOBS, "build_cweights: %d jobs", njobs);
    CWeightJobs P;
    long most = 0;
    for (int i = 0; i < njobs; ++i) {
        const CWeightJob& J = jobs[i];
        const bool planar = J.packed == WPACKX3 || J.packed == WPACKH2 || J.packed == WPACKH2_ABS2 ||
                            J.packed == WPACKI8 || J.packed == WPACKX3_ABS2;
        AMP_REQUIRE((planar ? J.J <= J.kap && J.O <= J.ncp : 2 * J.J <= J.kap && 2 * J.O <= J.ncp) &&
                        (J.packed == WPACK_NONE || (J.packed == WPACK32 && J.kap % GBK == 0 && J.ncp % 128 == 0) ||
                         (J.packed == WPACK16 && J.kap % 16 == 0 && J.ncp % 16 == 0) ||
                         (planar && J.kap % (J.packed == WPACKI8 ? 64 : 32) == 0 && J.ncp % 16 == 0)),
                    "build_cweights: job %d kap %d / ncp %d not tiled for layout %d", i, J.kap, J.ncp, J.packed);
        P.j[i] = J;
        most = std::max(most, planar ? (long)J.ncp * J.kap : (long)(J.ncp / 2) * (J.kap / 2));
    }
    P.zero = zero;
    P.nzero = zero ? nzero : 0;
    const int grid = (int)std::min<long>((most + 255) / 256, 2048);
    hipLaunchKernelGGL(build_cweights_kernel, dim3(grid, njobs), dim3(256), 0, st, P);
    AMP_LAUNCH_CHECK("build_cweights");
    return AMP_OK;
}

int build_abs2_weight(const float2* src, long so, long sj, int O, int J, float* wt, int kap, int ncp,
                      hipStream_t st) {
    AMP_REQUIRE(kap % GBK == 0 && ncp % 128 == 0, "build_abs2_weight: kap %d / ncp %d not tiled", kap, ncp);
    const long total = (long)ncp * kap;
    const int grid = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(build_abs2_kernel, dim3(grid), dim3(256), 0, st, src, so, sj, O, J, wt, kap, ncp);
    AMP_LAUNCH_CHECK("build_abs2_weight");
    return AMP_OK;
}

template <int BN>
int set_lds_attr(const void* fn) {
    static_assert(GemmCfg<BN>::LDS_BYTES <= 160 * 1024, "LDS budget");
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GemmCfg<BN>::LDS_BYTES);
    if (e != hipSuccess) {
        set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
        return AMP_E_LAUNCH;
    }
    return AMP_OK;
}
template int set_lds_attr<128>(const void*);
template int set_lds_attr<256>(const void*);

// Plain GEMM: C[rows][ldc] = A[rows][lda](ka valid) . Wt^T, columns [0, nc) stored.
template <int BN>
__global__ __launch_bounds__(AMP_WG) void gemm_store_kernel(const float* __restrict__ a, int lda, int rows, int ka,
                                                            const float* __restrict__ wt, int kap,
                                                            float* __restrict__ c, int ldc, int nc) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const GemmTile tile = xcd_tile();
    const int row0 = tile.rb * GBM, col0 = tile.cb * BN;
    gemm_tile<BN>(ALoadPlain{a, lda, rows, ka}, wt, kap, row0, col0, lds);
    using C = GemmCfg<BN>;
    for (int e = threadIdx.x; e < GBM * BN; e += AMP_WG) {
        const int rho = e / BN, cc = e % BN;
        const int row = row0 + rho, col = col0 + cc;
        if (row < rows && col < nc) c[(size_t)row * ldc + col] = lds[rho * C::LDC + cc];
    }
}

// Grid (column tile, reduction slice): each wave takes (column group, reduction group) blocks of
// the packed layout (64 float4 = one lane each, wcol in gemm_tile) within its slice and keeps the
// first / last group holding a nonzero value (NaN / inf count as nonzero: they must reach the
// product); the slices meet in band[] through atomic min / max (vector atomics), bracketed by an
// init and a conversion launch.  (One workgroup per tile had taken 225 us per operator at the
// ISI shape: 17 workgroups walking 8 MB.)
__global__ __launch_bounds__(256) void weight_kband_init(int* __restrict__ band, int ntiles, int G) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntiles) { band[2 * t] = G; band[2 * t + 1] = -1; }
}

__global__ __launch_bounds__(256) void weight_kband_kernel(const float4* __restrict__ wp, int G, int cgs, int gps,
                                                           int* __restrict__ band) {
    __shared__ int s_lo, s_hi;
    if (threadIdx.x == 0) { s_lo = G; s_hi = -1; }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cg0 = blockIdx.x * cgs;
    const int ga = blockIdx.y * gps, gn = min(gps, G - ga);
    int lo = G, hi = -1;
    for (int b = wave; b < cgs * gn; b += blockDim.x >> 6) {   // wave-uniform
        const int cg = cg0 + b / gn, g = ga + b % gn;
        const float4 v = wp[((size_t)cg * G + g) * 64 + lane];
        const bool nz = (v.x != 0.f) | (v.y != 0.f) | (v.z != 0.f) | (v.w != 0.f) | (v.x != v.x) | (v.y != v.y) |
                        (v.z != v.z) | (v.w != v.w);
        if (__any(nz)) { lo = min(lo, g); hi = max(hi, g); }
    }
    if (lane == 0) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
    __syncthreads();
    if (threadIdx.x == 0 && s_hi >= 0) {
        atomicMin(&band[2 * blockIdx.x], s_lo);
        atomicMax(&band[2 * blockIdx.x + 1], s_hi);
    }
}

__global__ __launch_bounds__(256) void weight_kband_fin(int* __restrict__ band, int ntiles) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const int lo = band[2 * t], hi = band[2 * t + 1];
    const int gpk = GBK / 8;                               // reduction groups per GBK
    band[2 * t] = hi < 0 ? 0 : (lo / gpk) * GBK;
    band[2 * t + 1] = hi < 0 ? 0 : ((hi + gpk) / gpk) * GBK;
}

int weight_kband(const float* wp, int kap, int ncp, int BN, int* band, hipStream_t st) {
    AMP_REQUIRE(kap % GBK == 0 && ncp % BN == 0 && BN % 32 == 0, "weight_kband: kap %d / ncp %d / BN %d", kap, ncp,
                BN);
    const int nt = ncp / BN, G = kap / 8;
    const int gps = 64;                                    // reduction groups per slice: 64 KB per tile-slice
    hipLaunchKernelGGL(weight_kband_init, dim3(cdiv(nt, 256)), dim3(256), 0, st, band, nt, G);
    hipLaunchKernelGGL(weight_kband_kernel, dim3(nt, cdiv(G, gps)), dim3(256), 0, st, (const float4*)wp, G, BN / 32,
                       gps, band);
    hipLaunchKernelGGL(weight_kband_fin, dim3(cdiv(nt, 256)), dim3(256), 0, st, band, nt);
    AMP_LAUNCH_CHECK("weight_kband");
    return AMP_OK;
}

// [lo, hi] 32-groups -> [kb, ke) in reduction elements, whole 64-element pairs
__global__ __launch_bounds__(256) void h2_kband_fin(int* __restrict__ band, int ntiles) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const int lo = band[2 * t], hi = band[2 * t + 1];
    band[2 * t] = hi < 0 ? 0 : 32 * (lo & ~1);
    band[2 * t + 1] = hi < 0 ? 0 : 32 * ((hi | 1) + 1);
}

// h2_kband_kernel over a plane-packed operator (PL 16-bit planes: fp16x2 2 / 4, bf16x3 3 / 6; G
// 32-groups per 16-output tile, tpt 16-output tiles per GEMM column tile, ntiles column tiles, n16
// packed 16-output tiles): [kb, ke) per column tile.
int h2_kband(const void* wq, int PL, int G, int tpt, int ntiles, int n16, int* band, hipStream_t st) {
    AMP_REQUIRE(G % 2 == 0 && (PL == 2 || PL == 3 || PL == 4 || PL == 6), "h2_kband: G %d / PL %d", G, PL);
    const int gps = 64;
    hipLaunchKernelGGL(weight_kband_init, dim3(cdiv(ntiles, 256)), dim3(256), 0, st, band, ntiles, G);
    if (PL == 6)
        hipLaunchKernelGGL(h2_kband_kernel<6>, dim3(ntiles, cdiv(G, gps)), dim3(256), 0, st, (const u32x4*)wq, G, tpt,
                           gps, n16, band);
    else if (PL == 3)
        hipLaunchKernelGGL(h2_kband_kernel<3>, dim3(ntiles, cdiv(G, gps)), dim3(256), 0, st, (const u32x4*)wq, G, tpt,
                           gps, n16, band);
    else if (PL == 4)
        hipLaunchKernelGGL(h2_kband_kernel<4>, dim3(ntiles, cdiv(G, gps)), dim3(256), 0, st, (const u32x4*)wq, G, tpt,
                           gps, n16, band);
    else
        hipLaunchKernelGGL(h2_kband_kernel<2>, dim3(ntiles, cdiv(G, gps)), dim3(256), 0, st, (const u32x4*)wq, G, tpt,
                           gps, n16, band);
    hipLaunchKernelGGL(h2_kband_fin, dim3(cdiv(ntiles, 256)), dim3(256), 0, st, band, ntiles);
    AMP_LAUNCH_CHECK("h2_kband");
    return AMP_OK;
}

int fix_grid(int nblk, int work) {
    static const bool uncapped = [] {   // AMP_FIX_GRID=0: one workgroup per 256 sections (A/B runs)
        const char* e = diag_env("AMP_FIX_GRID");
        return e && e[0] == '0';
    }();
    const int g = std::max(1, std::min(nblk, cdiv(work, AMP_WG)));
    return uncapped ? g : std::min(g, 2 * device_cu_count());
}

int gemm_store(const float* a, int lda, int rows, int ka, const float* wt, int kap, int ncp, float* c, int ldc,
               int nc, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        int rc = set_lds_attr<128>((const void*)gemm_store_kernel<128>);
        if (rc) return rc;
        attr = true;
    }
    dim3 grid(cdiv(rows, GBM), ncp / 128);
    hipLaunchKernelGGL(gemm_store_kernel<128>, grid, dim3(AMP_WG), GemmCfg<128>::LDS_BYTES, st, a, lda, rows, ka, wt,
                       kap, c, ldc, nc);
    AMP_LAUNCH_CHECK("gemm_store");
    return AMP_OK;
}

static amp_allreduce_fn g_hook = nullptr;
static void* g_hook_ctx = nullptr;

bool allreduce_hook_set() { return g_hook != nullptr; }

int call_allreduce_hook(double* buf, int count, int op, hipStream_t st) {
    const int rc = g_hook((void*)buf, count, op, (void*)st, g_hook_ctx);
    return rc ? AMP_E_LAUNCH : AMP_OK;
}

int hook_failure(const char* what) {
    set_error("amp_%s_run_sharded: the all-reduce hook failed on this rank (every later call was still made)",
              what);
    return AMP_E_LAUNCH;
}

}  // namespace amp

namespace amp {
// The CU range of every stream amp_stream_create_cu_range made (until amp_stream_destroy), and per
// shard exchange buffer the ranges its current generation's grids were launched on: what
// amp_vamp_detect_count_shard checks before it launches a grid that spins on its partners.
static std::mutex g_cu_mu;
static std::map<hipStream_t, std::pair<int, int>> g_cu_streams;
static std::map<const void*, std::pair<unsigned, std::vector<std::pair<int, int>>>> g_shard_ranges;

bool cu_range_of(hipStream_t st, int* cu0, int* cu1) {
    std::lock_guard<std::mutex> lk(g_cu_mu);
    const auto it = g_cu_streams.find(st);
    if (it == g_cu_streams.end()) return false;
    *cu0 = it->second.first;
    *cu1 = it->second.second;
    return true;
}

void shard_forget(const void* xbuf) {
    std::lock_guard<std::mutex> lk(g_cu_mu);
    g_shard_ranges.erase(xbuf);
}

bool shard_claim_range(const void* xbuf, unsigned gen, int cu0, int cu1) {
    std::lock_guard<std::mutex> lk(g_cu_mu);
    auto& e = g_shard_ranges[xbuf];
    if (e.first != gen) {
        e.first = gen;
        e.second.clear();
    }
    for (const auto& r : e.second)
        if (cu0 < r.second && r.first < cu1) return false;
    e.second.emplace_back(cu0, cu1);
    return true;
}
}  // namespace amp

extern "C" {

int amp_set_allreduce_hook(amp_allreduce_fn fn, void* ctx) {
    amp::g_hook = fn;
    amp::g_hook_ctx = ctx;
    return AMP_OK;
}

const char* amp_last_error(void) { return amp::g_err; }

// A stream whose kernels run only on the CUs [cu0, cu1) (hipExtStreamCreateWithCUMask; its own
// hardware queue): co-resident persistent grids of one batch's shards (amp_vamp_detect_count_shard)
// each on its own part of the chip, so one grid's launch never waits behind another's in a queue.
int amp_stream_create_cu_range(int32_t cu0, int32_t cu1, void** stream) {
    AMP_REQUIRE(stream && cu0 >= 0 && cu1 > cu0 && cu1 <= amp::device_cu_count(),
                "amp_stream_create_cu_range: CUs [%d, %d) of %d", cu0, cu1, amp::device_cu_count());
    uint32_t mask[32] = {0};
    const int words = (amp::device_cu_count() + 31) / 32;
    AMP_REQUIRE(words <= 32, "amp_stream_create_cu_range: %d CUs", amp::device_cu_count());
    for (int c = cu0; c < cu1; ++c) mask[c >> 5] |= 1u << (c & 31);
    hipStream_t st = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask);
    AMP_REQUIRE(e == hipSuccess, "amp_stream_create_cu_range: %s", hipGetErrorString(e));
    {
        std::lock_guard<std::mutex> lk(amp::g_cu_mu);
        amp::g_cu_streams[st] = {cu0, cu1};
    }
    *stream = st;
    return AMP_OK;
}

int amp_stream_destroy(void* stream) {
    {
        std::lock_guard<std::mutex> lk(amp::g_cu_mu);
        amp::g_cu_streams.erase((hipStream_t)stream);
    }
    const hipError_t e = hipStreamDestroy((hipStream_t)stream);
    AMP_REQUIRE(e == hipSuccess, "amp_stream_destroy: %s", hipGetErrorString(e));
    return AMP_OK;
}

const char* amp_build_info(void) {
    return "amp_sparc gfx950: fp32 MFMA v_mfma_f32_32x32x2_f32 GEMM engine (BM=32, A block in LDS, "
           "MFMA-packed weights streamed from L2, BN=128/256), "
           "fused LMMSE/Onsager/section-denoiser epilogues";
}

// Test/diagnostic entry point: C[rows][ldc] = A[rows][lda] . Wt[ncp][kap]^T with a row-major Wt
// (first ka columns of A valid, first nc columns of C stored); packs Wt into a stream-ordered
// temporary first.  Requirements: lda % 4 == 0, ka % 4 == 0, kap % 64 == 0, ncp % 128 == 0.
int amp_gemm_nt_f32(const void* a, int32_t lda, int32_t rows, int32_t ka, const void* wt, int32_t kap, int32_t ncp,
                    void* c, int32_t ldc, int32_t nc, void* stream) {
    AMP_REQUIRE(lda % 4 == 0 && ka % 4 == 0 && kap % amp::GBK == 0 && ncp % 128 == 0 && ka <= kap && nc <= ncp,
                "amp_gemm_nt_f32: bad shape (lda %d ka %d kap %d ncp %d nc %d)", lda, ka, kap, ncp, nc);
    hipStream_t st = (hipStream_t)stream;
    float* wp = nullptr;
    hipError_t e = hipMallocAsync((void**)&wp, (size_t)kap * ncp * sizeof(float), st);
    AMP_REQUIRE(e == hipSuccess, "amp_gemm_nt_f32: hipMallocAsync: %s", hipGetErrorString(e));
    const long total = (long)ncp * kap;
    hipLaunchKernelGGL(amp::pack_weight_kernel, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0,
                       st, (const float*)wt, wp, kap, ncp);
    int rc = amp::gemm_store((const float*)a, lda, rows, ka, wp, kap, ncp, (float*)c, ldc, nc, st);
    (void)hipFreeAsync(wp, st);
    return rc;
}

// Test/diagnostic entry point for the complex weight expansion (see build_cweight_kernel).
int amp_build_cweight(const void* src, int64_t so, int64_t sj, int32_t conj, const void* rowscale, int32_t O,
                      int32_t J, void* wt, int32_t kap, int32_t ncp, void* stream) {
    return amp::build_cweight((const float2*)src, so, sj, conj, (const float*)rowscale, O, J, (float*)wt, kap, ncp,
                              (hipStream_t)stream, amp::WPACK_NONE);
}

}  // extern "C"
