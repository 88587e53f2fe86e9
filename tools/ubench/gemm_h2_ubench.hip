// Split-precision complex GEMM microbenchmark, fp16x2 against bf16x3 (persistent-engine shape:
// 256 workgroups x 4 waves, each workgroup C[16 x O] = A[16 x K] . X^T, complex, K = O = 256 at
// cfg4, repeated REPS times from LDS-resident A pieces and L2-streamed weight pieces).
//   fp16x2: a 2^ea = h0 + h1, x 2^ex = g0 + g1 (fp16 pieces, RN; 22 significant bits), three
//   products h0g0 h0g1 h1g0 on v_mfma_f32_16x16x32_f16 (dropped h1g1 <= 2^-22 |ax|), the result
//   scaled back by 2^-(ea + ex) (exact); 4 planes of 16-bit pieces instead of 6: 8 bytes per
//   complex weight entry instead of 12, 12 MFMAs per complex tile-group instead of 24.
// hipcc -O3 --offload-arch=gfx950 -o /tmp/gh2 tools/ubench/gemm_h2_ubench.hip && /tmp/gh2
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int KC = 256, OC = 256, REPS = 20, NWG = 256;
constexpr int LDA = KC + 8;   // 16-bit elements per LDS row (16-byte pad)
constexpr int ESC_A = 13, ESC_X = 16;   // power-of-two scales of the pieces (A in [-1,1], X in [-1/16, 1/16])

__device__ __forceinline__ f16x8 as_h(u32x4 v) { return __builtin_bit_cast(f16x8, v); }

template <int NT, int G, int R>
__device__ __forceinline__ void gemm_h2(const unsigned short* sA, const void* wq, int ct0, f32x4 (&cr)[NT],
                                        f32x4 (&ci)[NT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < NT; ++t) { cr[t] = f32x4{0, 0, 0, 0}; ci[t] = f32x4{0, 0, 0, 0}; }
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 4 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    u32x4 ring[R][NT][4];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < 4; ++f) ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + d) * 4 + f) * 1024, 0);
    const unsigned short* ap = sA + (lane & 15) * LDA + 8 * (lane >> 4);
    u32x4 an[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % R;
        u32x4 a[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) a[f] = an[f];
        if (g + 1 < G) {
#pragma unroll
            for (int f = 0; f < 4; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA + 32 * (g + 1));
        }
        u32x4 na[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) na[f] = a[2 + f] ^ u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4* w = ring[d][t];   // w[0] Xr g0, w[1] Xr g1, w[2] Xi g0, w[3] Xi g1
#define MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h(x), as_h(y), acc, 0, 0, 0)
            // Cr = Ar.Xr - Ai.Xi ; Ci = Ar.Xi + Ai.Xr   (a[0] Ar h0, a[1] Ar h1, a[2] Ai h0, a[3] Ai h1)
            MF(cr[t], a[0], w[1]);  MF(ci[t], a[0], w[3]);
            MF(cr[t], a[1], w[0]);  MF(ci[t], a[1], w[2]);
            MF(cr[t], na[0], w[3]); MF(ci[t], a[2], w[1]);
            MF(cr[t], na[1], w[2]); MF(ci[t], a[3], w[0]);
            MF(cr[t], a[0], w[0]);  MF(ci[t], a[0], w[2]);
            MF(cr[t], na[0], w[2]); MF(ci[t], a[2], w[0]);
#undef MF
        }
        if (g + R < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + R) * 4 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R>
__global__ __launch_bounds__(256, 1) void kh2(const unsigned short* apieces, const void* wq, float* out,
                                               unsigned long long* cyc) {
    __shared__ unsigned short sA[4 * 16 * LDA];
    for (int e = threadIdx.x; e < 4 * 16 * KC; e += 256) {
        const int f = e / (16 * KC), rem = e % (16 * KC), row = rem / KC, k = rem % KC;
        sA[(f * 16 + row) * LDA + k] = apieces[e];
    }
    __syncthreads();
    constexpr int NT = OC / 16 / 4, G = KC / 32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 cr[NT], ci[NT];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        gemm_h2<NT, G, R>(sA, wq, wave * NT, cr, ci);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const float sc = ldexpf(1.0f, -(ESC_A + ESC_X));
    if (blockIdx.x == 0) {
        for (int t = 0; t < NT; ++t)
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r, o = 16 * (wave * NT + t) + (lane & 15);
                out[(row * OC + o) * 2] = cr[t][r] * sc;
                out[(row * OC + o) * 2 + 1] = ci[t][r] * sc;
            }
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static unsigned short h16(float x) {
    _Float16 h = (_Float16)x;
    unsigned short u;
    memcpy(&u, &h, 2);
    return u;
}
static float hf(unsigned short u) {
    _Float16 h;
    memcpy(&h, &u, 2);
    return (float)h;
}
static void split2(float x, int e, unsigned short p[2]) {
    const float s = ldexpf(x, e);
    p[0] = h16(s);
    p[1] = h16(s - hf(p[0]));
}

template <int R>
static void run(const std::vector<unsigned short>& ap, const std::vector<unsigned short>& wp,
                const std::vector<double>& ref, const std::vector<float>& f32c) {
    unsigned short* dA;
    void* dW;
    float* dO;
    unsigned long long* dc;
    hipMalloc(&dA, ap.size() * 2);
    hipMalloc(&dW, wp.size() * 2);
    hipMalloc(&dO, 16 * OC * 2 * 4);
    hipMalloc(&dc, NWG * 8);
    hipMemcpy(dA, ap.data(), ap.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW, wp.data(), wp.size() * 2, hipMemcpyHostToDevice);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kh2<R>), dim3(NWG), dim3(256), 0, 0, dA, dW, dO, dc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(NWG, 0);
    hipMemcpy(c.data(), dc, NWG * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    std::vector<float> o(16 * OC * 2);
    hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
    double eh = 0, ef = 0, nrm = 0, sh = 0, sf = 0;
    for (size_t i = 0; i < o.size(); ++i) {
        eh = std::max(eh, fabs(o[i] - ref[i]));
        ef = std::max(ef, fabs(f32c[i] - ref[i]));
        sh += (o[i] - ref[i]) * (o[i] - ref[i]);
        sf += (f32c[i] - ref[i]) * (f32c[i] - ref[i]);
        nrm = std::max(nrm, fabs(ref[i]));
    }
    printf("fp16x2 R=%d: cycles per GEMM median %.0f max %.0f   max|err| h2 %.3e f32-seq %.3e   rms h2 %.3e f32-seq %.3e (max|C| %.3f)\n",
           R, (double)c[NWG / 2] / REPS, (double)c[NWG - 1] / REPS, eh, ef, sqrt(sh / o.size()), sqrt(sf / o.size()), nrm);
    hipFree(dA); hipFree(dW); hipFree(dO); hipFree(dc);
}

int main() {
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> A(16 * KC * 2), X(OC * KC * 2);
    for (auto& v : A) v = rnd();
    for (auto& v : X) v = rnd() * 0.0625f;
    // A pieces: planar [Ar h0 h1, Ai h0 h1][16][KC]
    std::vector<unsigned short> ap(4 * 16 * KC);
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < KC; ++k) {
            unsigned short p[2], q[2];
            split2(A[(r * KC + k) * 2], ESC_A, p);
            split2(A[(r * KC + k) * 2 + 1], ESC_A, q);
            for (int s = 0; s < 2; ++s) {
                ap[(s * 16 + r) * KC + k] = p[s];
                ap[((2 + s) * 16 + r) * KC + k] = q[s];
            }
        }
    // weight pieces: [ct][g][f: Xr g0 g1, Xi g0 g1][lane][8], B[k][col] = X[col][k]
    const int G = KC / 32;
    std::vector<unsigned short> wp((size_t)(OC / 16) * G * 4 * 64 * 8);
    for (int o = 0; o < OC; ++o)
        for (int k = 0; k < KC; ++k) {
            unsigned short p[2], q[2];
            split2(X[(o * KC + k) * 2], ESC_X, p);
            split2(X[(o * KC + k) * 2 + 1], ESC_X, q);
            const int ct = o >> 4, g = k >> 5, kk = k & 31, lane = (o & 15) + 16 * (kk >> 3), j = kk & 7;
            for (int s = 0; s < 2; ++s) {
                wp[((((size_t)ct * G + g) * 4 + s) * 64 + lane) * 8 + j] = p[s];
                wp[((((size_t)ct * G + g) * 4 + 2 + s) * 64 + lane) * 8 + j] = q[s];
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
    run<1>(ap, wp, ref, f32c);
    run<2>(ap, wp, ref, f32c);
    run<3>(ap, wp, ref, f32c);
    return 0;
}
