// Split-precision complex GEMM microbenchmark (persistent-engine shape): 256 workgroups x 4
// waves, each workgroup C[16 x O] = A[16 x K] . X^T (complex, K = O = 256 at cfg4), repeated
// REPS times from LDS-resident A pieces and L2-streamed weight pieces.
//   bf16x3: a = a0 + a1 + a2 (bf16 pieces), 6 products a0b0 a0b1 a1b0 a0b2 a1b1 a2b0 on
//   v_mfma_f32_16x16x32_bf16; complex-planar operands (Re / Im planes, the weight's unique
//   values only: Cr = Ar.Xr - Ai.Xi, Ci = Ar.Xi + Ai.Xr).
// hipcc -O3 --offload-arch=gfx950 -o /tmp/gx3 tools/ubench/gemm_x3_ubench.hip && /tmp/gx3
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KC = 256, OC = 256, REPS = 20, NWG = 256;
constexpr int LDA = KC + 8;   // bf16 elements per LDS row (16-byte pad)

__device__ __forceinline__ bf16x8 as_bf(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

template <int NT, int G, int R, int AUX = 0, int MODE = 0, bool PF = false>
__device__ __forceinline__ void gemm_x3(const unsigned short* sA, const void* wq, int ct0, f32x4 (&cr)[NT],
                                        f32x4 (&ci)[NT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < NT; ++t) { cr[t] = f32x4{0, 0, 0, 0}; ci[t] = f32x4{0, 0, 0, 0}; }
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 6 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    u32x4 ring[R][NT][6];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < 6; ++f) ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + d) * 6 + f) * 1024, AUX);
    const unsigned short* ap = sA + (lane & 15) * LDA + 8 * (lane >> 4);
    u32x4 an[6];
#pragma unroll
    for (int f = 0; f < 6; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % R;
        u32x4 a[6];
#pragma unroll
        for (int f = 0; f < 6; ++f) a[f] = an[f];
        if (PF && g + 1 < G) {
#pragma unroll
            for (int f = 0; f < 6; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA + 32 * (g + 1));
        } else if (!PF) {
#pragma unroll
            for (int f = 0; f < 6; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA + 32 * g);
        }
        u32x4 na[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) na[f] = a[3 + f] ^ u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4* w = ring[d][t];
            if constexpr (MODE == 1) {
                for (int f = 0; f < 6; ++f) cr[t][f & 3] += __builtin_bit_cast(float, w[f].x ^ a[f].y);
                continue;
            }
            // smallest terms first
#define MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(x), as_bf(y), acc, 0, 0, 0)
            MF(cr[t], a[0], w[2]); MF(ci[t], a[0], w[5]);
            MF(cr[t], a[1], w[1]); MF(ci[t], a[1], w[4]);
            MF(cr[t], a[2], w[0]); MF(ci[t], a[2], w[3]);
            MF(cr[t], na[0], w[5]); MF(ci[t], a[3], w[2]);
            MF(cr[t], na[1], w[4]); MF(ci[t], a[4], w[1]);
            MF(cr[t], na[2], w[3]); MF(ci[t], a[5], w[0]);
            MF(cr[t], a[0], w[1]); MF(ci[t], a[0], w[4]);
            MF(cr[t], a[1], w[0]); MF(ci[t], a[1], w[3]);
            MF(cr[t], na[0], w[4]); MF(ci[t], a[3], w[1]);
            MF(cr[t], na[1], w[3]); MF(ci[t], a[4], w[0]);
            MF(cr[t], a[0], w[0]); MF(ci[t], a[0], w[3]);
            MF(cr[t], na[0], w[3]); MF(ci[t], a[3], w[0]);
#undef MF
        }
        if (MODE != 2 && g + R < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int f = 0; f < 6; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + R) * 6 + f) * 1024, AUX);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int AUX = 0, int MODE = 0, bool PF = false>
__global__ __launch_bounds__(256, 1) void kx3(const unsigned short* apieces, const void* wq, float* out,
                                               unsigned long long* cyc) {
    __shared__ unsigned short sA[6 * 16 * LDA];
    for (int e = threadIdx.x; e < 6 * 16 * KC; e += 256) {
        const int f = e / (16 * KC), rem = e % (16 * KC), row = rem / KC, k = rem % KC;
        sA[(f * 16 + row) * LDA + k] = apieces[e];
    }
    __syncthreads();
    constexpr int NT = OC / 16 / 4, G = KC / 32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 cr[NT], ci[NT];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        gemm_x3<NT, G, R, AUX, MODE, PF>(sA, wq, wave * NT, cr, ci);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0) {
        for (int t = 0; t < NT; ++t)
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r, o = 16 * (wave * NT + t) + (lane & 15);
                out[(row * OC + o) * 2] = cr[t][r];
                out[(row * OC + o) * 2 + 1] = ci[t][r];
            }
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static unsigned short bf16_rn(float x) {
    unsigned u;
    memcpy(&u, &x, 4);
    const unsigned r = 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)((u + r) >> 16);
}
static float bf2f(unsigned short h) {
    unsigned u = (unsigned)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static void split3(float x, unsigned short p[3]) {
    p[0] = bf16_rn(x);
    const float r1 = x - bf2f(p[0]);
    p[1] = bf16_rn(r1);
    const float r2 = r1 - bf2f(p[1]);
    p[2] = bf16_rn(r2);
}

template <int R, int AUX = 0, int MODE = 0, bool PF = false>
static void run(int nwg, const std::vector<unsigned short>& ap, const std::vector<unsigned short>& wp,
                const std::vector<double>& ref, const std::vector<float>& f32c) {
    unsigned short *dA;
    void* dW;
    float* dO;
    unsigned long long* dc;
    hipMalloc(&dA, ap.size() * 2);
    hipMalloc(&dW, wp.size() * 2);
    hipMalloc(&dO, 16 * OC * 2 * 4);
    hipMalloc(&dc, NWG * 8);
    hipMemcpy(dA, ap.data(), ap.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW, wp.data(), wp.size() * 2, hipMemcpyHostToDevice);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kx3<R, AUX, MODE, PF>), dim3(nwg), dim3(256), 0, 0, dA, dW, dO, dc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(NWG, 0);
    hipMemcpy(c.data(), dc, nwg * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    std::vector<float> o(16 * OC * 2);
    hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
    double ex3 = 0, ef = 0, nrm = 0;
    for (size_t i = 0; i < o.size(); ++i) {
        ex3 = std::max(ex3, fabs(o[i] - ref[i]));
        ef = std::max(ef, fabs(f32c[i] - ref[i]));
        nrm = std::max(nrm, fabs(ref[i]));
    }
    printf("bf16x3 PF=%d MODE=%d nwg=%d AUX=%d R=%d: cycles per GEMM median %.0f  max %.0f   max|err| x3 %.3e  f32-seq %.3e  (max|C| %.3f)\n", (int)PF, MODE, nwg, AUX, R,
           (double)c[NWG - nwg + nwg / 2] / REPS, (double)c[NWG - 1] / REPS, ex3, ef, nrm);
    hipFree(dA); hipFree(dW); hipFree(dO); hipFree(dc);
}

int main() {
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> A(16 * KC * 2), X(OC * KC * 2);
    for (auto& v : A) v = rnd();
    for (auto& v : X) v = rnd() * 0.0625f;
    // A pieces: planar [Ar0 Ar1 Ar2 Ai0 Ai1 Ai2][16][KC]
    std::vector<unsigned short> ap(6 * 16 * KC);
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < KC; ++k) {
            unsigned short p[3], q[3];
            split3(A[(r * KC + k) * 2], p);
            split3(A[(r * KC + k) * 2 + 1], q);
            for (int s = 0; s < 3; ++s) {
                ap[(s * 16 + r) * KC + k] = p[s];
                ap[((3 + s) * 16 + r) * KC + k] = q[s];
            }
        }
    // weight pieces: [ct][g][f: Xr0 Xr1 Xr2 Xi0 Xi1 Xi2][lane][8], B[k][col] = X[col][k]
    const int G = KC / 32;
    std::vector<unsigned short> wp((size_t)(OC / 16) * G * 6 * 64 * 8);
    for (int o = 0; o < OC; ++o)
        for (int k = 0; k < KC; ++k) {
            unsigned short p[3], q[3];
            split3(X[(o * KC + k) * 2], p);
            split3(X[(o * KC + k) * 2 + 1], q);
            const int ct = o >> 4, g = k >> 5, kk = k & 31, lane = (o & 15) + 16 * (kk >> 3), j = kk & 7;
            for (int s = 0; s < 3; ++s) {
                wp[((((size_t)ct * G + g) * 6 + s) * 64 + lane) * 8 + j] = p[s];
                wp[((((size_t)ct * G + g) * 6 + 3 + s) * 64 + lane) * 8 + j] = q[s];
            }
        }
    std::vector<double> ref(16 * OC * 2);
    std::vector<float> f32c(16 * OC * 2);
    for (int r = 0; r < 16; ++r)
        for (int o = 0; o < OC; ++o) {
            double sr = 0, si = 0;
            float fr = 0, fi = 0;
            for (int k = 0; k < KC; ++k) {
                const float ar = A[(r * KC + k) * 2], ai = A[(r * KC + k) * 2 + 1];
                const float xr = X[(o * KC + k) * 2], xi = X[(o * KC + k) * 2 + 1];
                sr += (double)ar * xr - (double)ai * xi;
                si += (double)ar * xi + (double)ai * xr;
                fr = fmaf(ar, xr, fr); fr = fmaf(-ai, xi, fr);
                fi = fmaf(ar, xi, fi); fi = fmaf(ai, xr, fi);
            }
            ref[(r * OC + o) * 2] = sr; ref[(r * OC + o) * 2 + 1] = si;
            f32c[(r * OC + o) * 2] = fr; f32c[(r * OC + o) * 2 + 1] = fi;
        }
    run<2, 0, 0, false>(256, ap, wp, ref, f32c);
    run<2, 0, 2, false>(256, ap, wp, ref, f32c);
    run<1, 0, 0, true>(256, ap, wp, ref, f32c);
    run<2, 0, 0, true>(256, ap, wp, ref, f32c);
    run<3, 0, 0, true>(256, ap, wp, ref, f32c);
    run<2, 0, 2, true>(256, ap, wp, ref, f32c);
    return 0;
}
