// Split-precision complex GEMM microbenchmark: int8x4 (block fixed point on the integer matrix
// cores) against the persistent engine's shape (256 workgroups x 4 waves, each workgroup
// C[16 x O] = A[16 x K] . X^T, complex, K = O = 256 at cfg4, REPS times from LDS-resident A slices
// and L2-streamed operator slices).
//   Every A row carries its own power-of-two scale 2^ea (max |value| of the row < 2^ea), every
//   operator column its own 2^ex; the scaled value v 2^(30 - e) is rounded to a 31-bit integer and
//   written as four balanced base-256 digits s0 .. s3 (s0 the top one, |s0| <= 64, the others in
//   [-128, 127]).  A product keeps the digit pairs i + j <= 3 — ten per real product, exact in
//   int32 (v_mfma_i32_16x16x64_i8, K = 64 per instruction) — summed per level s = i + j in its own
//   accumulator, the levels combined in f32 at the end (Horner, smallest first) and the scales
//   taken off exactly.  Operands: 31-bit fixed point per row / column; dropped terms (i + j >= 4)
//   < 2^-30 of (row max . column max).  8 bytes per complex operator entry (bf16x3: 12), 40 MFMAs
//   per complex tile and 64-deep group (bf16x3: 48 for the same depth).
//   -Ai is sliced on its own (balanced digits are not closed under negation), so the A operand
//   is twelve int8 planes (Ar, Ai, -Ai): 48 KB at cfg4, the bf16x3 planes' size.
// hipcc -O3 --offload-arch=gfx950 -o /tmp/gi8 tools/ubench/gemm_i8_ubench.hip && /tmp/gi8
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../amp-sparc-spatialmodulation_amd/csrc/amp_persist.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int KC = 256, OC = 256, REPS = 20, NWG = 256;
constexpr int LDA = KC + 16;   // bytes per LDS row of one plane (16-byte pad)

template <int NT, int G, int R, bool TILEREFILL>
__device__ __forceinline__ void gemm_i8(const signed char* sA, const void* wq, int ct0, i32x4 (&acc)[NT][2][4]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[t][c][s] = i32x4{0, 0, 0, 0};
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 8 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    u32x4 ring[R][NT][8];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int f = 0; f < 8; ++f) ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + d) * 8 + f) * 1024, 0);
    // A fragment of group g: row lane & 15, k = 64 g + 16 (lane >> 4) + j; read one group ahead
    const signed char* ap = sA + (lane & 15) * LDA + 16 * (lane >> 4);
    u32x4 an[12];
#pragma unroll
    for (int f = 0; f < 12; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int d = g % R;
        u32x4 a[12];   // Ar s0..s3, Ai s0..s3, -Ai s0..s3
#pragma unroll
        for (int f = 0; f < 12; ++f) a[f] = an[f];
        if (g + 1 < G) {
#pragma unroll
            for (int f = 0; f < 12; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA + 64 * (g + 1));
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4* w = ring[d][t];   // w[0..3] Xr s0..s3, w[4..7] Xi s0..s3
#define MI(acc_, x, y) acc_ = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, x), __builtin_bit_cast(i32x4, y), acc_, 0, 0, 0)
#pragma unroll
            for (int s = 3; s >= 0; --s)
#pragma unroll
                for (int i = 0; i <= s; ++i) {
                    const int j = s - i;
                    MI(acc[t][0][s], a[i], w[j]);          // Ar Xr
                    MI(acc[t][0][s], a[8 + i], w[4 + j]);  // (-Ai) Xi
                    MI(acc[t][1][s], a[i], w[4 + j]);      // Ar Xi
                    MI(acc[t][1][s], a[4 + i], w[j]);      // Ai Xr
                }
#undef MI
            // this tile's slot of the ring refilled for group g + R right behind its MFMAs
            if (TILEREFILL && g + R < G) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int f = 0; f < 8; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + R) * 8 + f) * 1024, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (!TILEREFILL && g + R < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int f = 0; f < 8; ++f)
                    ring[d][t][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((t * G + g + R) * 8 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Tile-outer form (the engine's): complex column tile t runs all its K groups before tile t + 1,
// so only ONE tile's level accumulators are live (P = Ar.Xr, Q = Ai.Xi, C = Ar.Xi + Ai.Xr, four
// levels each: 48 registers) and the result leaves as f32 (Cr = P - Q exact in int32: every level
// sum < 2^25).  The A operand is eight planes (Ar, Ai; no -Ai), re-read from LDS per tile.  The
// operator streams through a ring of D (tile, group) slots in (t, g) order.
template <int NT, int G, int D>
__device__ __forceinline__ void gemm_i8t(const signed char* sA, const void* wq, int ct0, const int* aexp,
                                         const int* xexp, f32x4 (&cr)[NT], f32x4 (&ci)[NT]) {
    const int lane = threadIdx.x & 63;
    const int ct0u = __builtin_amdgcn_readfirstlane(ct0);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (char*)const_cast<void*>(wq) + (size_t)ct0u * G * 8 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    const int vo = lane * 16;
    constexpr int NS = NT * G;                 // (tile, group) steps, t-major
    u32x4 ring[D][8];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int f = 0; f < 8; ++f) ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, (d * 8 + f) * 1024, 0);
    const signed char* ap = sA + (lane & 15) * LDA + 16 * (lane >> 4);
    u32x4 an[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA);
    i32x4 P[4], Q[4], C[4];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
        const int t = st / G, g = st % G, d = st % D;
        if (g == 0) {
#pragma unroll
            for (int s = 0; s < 4; ++s) { P[s] = i32x4{0, 0, 0, 0}; Q[s] = P[s]; C[s] = P[s]; }
        }
        u32x4 a[8];
#pragma unroll
        for (int f = 0; f < 8; ++f) a[f] = an[f];
        if (st + 1 < NS) {
            const int g1 = (st + 1) % G;
#pragma unroll
            for (int f = 0; f < 8; ++f) an[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * LDA + 64 * g1);
        }
        const u32x4* w = ring[d];   // w[0..3] Xr s0..s3, w[4..7] Xi s0..s3
#define MI(acc_, x, y) acc_ = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, x), __builtin_bit_cast(i32x4, y), acc_, 0, 0, 0)
#pragma unroll
        for (int s = 3; s >= 0; --s)
#pragma unroll
            for (int i = 0; i <= s; ++i) {
                const int j = s - i;
                MI(P[s], a[i], w[j]);          // Ar Xr
                MI(Q[s], a[4 + i], w[4 + j]);  // Ai Xi
                MI(C[s], a[i], w[4 + j]);      // Ar Xi
                MI(C[s], a[4 + i], w[j]);      // Ai Xr
            }
#undef MI
        __builtin_amdgcn_sched_barrier(0);
        if (st + D < NS) {
#pragma unroll
            for (int f = 0; f < 8; ++f)
                ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((st + D) * 8 + f) * 1024, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (g == G - 1) {
            const int o = 16 * (ct0 + t) + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = aexp[4 * (lane >> 4) + r] + xexp[o] - 12;
                float vr = (float)(P[3][r] - Q[3][r]), vi = (float)C[3][r];
                vr = fmaf(vr, 0x1p-8f, (float)(P[2][r] - Q[2][r])); vi = fmaf(vi, 0x1p-8f, (float)C[2][r]);
                vr = fmaf(vr, 0x1p-8f, (float)(P[1][r] - Q[1][r])); vi = fmaf(vi, 0x1p-8f, (float)C[1][r]);
                vr = fmaf(vr, 0x1p-8f, (float)(P[0][r] - Q[0][r])); vi = fmaf(vi, 0x1p-8f, (float)C[0][r]);
                cr[t][r] = __builtin_amdgcn_ldexpf(vr, e);
                ci[t][r] = __builtin_amdgcn_ldexpf(vi, e);
            }
        }
    }
}

template <int D>
__global__ __launch_bounds__(256, 1) void ki8t(const signed char* apieces, const int* aexp, const void* wq,
                                               const int* xexp, float* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) signed char sA[8 * 16 * LDA];
    __shared__ int s_ae[16];
    for (int e = threadIdx.x; e < 8 * 16 * KC; e += 256) {
        const int f = e / (16 * KC), rem = e % (16 * KC), row = rem / KC, k = rem % KC;
        sA[(f * 16 + row) * LDA + k] = apieces[e];
    }
    if (threadIdx.x < 16) s_ae[threadIdx.x] = aexp[threadIdx.x];
    __syncthreads();
    constexpr int NT = OC / 16 / 4, G = KC / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 cr[NT], ci[NT];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        gemm_i8t<NT, G, D>(sA, wq, wave * NT, s_ae, xexp, cr, ci);
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

__device__ __forceinline__ float i8_combine(const i32x4 (&l)[4], int r) {
    float v = (float)l[3][r];
    v = fmaf(v, 0x1p-8f, (float)l[2][r]);
    v = fmaf(v, 0x1p-8f, (float)l[1][r]);
    return fmaf(v, 0x1p-8f, (float)l[0][r]);
}

template <int R, bool TR>
__global__ __launch_bounds__(256, 1) void ki8(const signed char* apieces, const int* aexp, const void* wq,
                                               const int* xexp, float* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) signed char sA[12 * 16 * LDA];
    for (int e = threadIdx.x; e < 12 * 16 * KC; e += 256) {
        const int f = e / (16 * KC), rem = e % (16 * KC), row = rem / KC, k = rem % KC;
        sA[(f * 16 + row) * LDA + k] = apieces[e];
    }
    __syncthreads();
    constexpr int NT = OC / 16 / 4, G = KC / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    i32x4 acc[NT][2][4];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        gemm_i8<NT, G, R, TR>(sA, wq, wave * NT, acc);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0) {
        for (int t = 0; t < NT; ++t)
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r, o = 16 * (wave * NT + t) + (lane & 15);
                const int e = aexp[row] + xexp[o] - 12;   // 2^(ea - 30) 2^(ex - 30) 2^48
                out[(row * OC + o) * 2] = ldexpf(i8_combine(acc[t][0], r), e);
                out[(row * OC + o) * 2 + 1] = ldexpf(i8_combine(acc[t][1], r), e);
            }
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// The engine's own gemm_i8 (amp_persist.h), operator exponents appended behind the planes.
__global__ __launch_bounds__(256, 1) void ki8e(const signed char* apieces, const int* aexp, const void* wqe,
                                               float* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) signed char sA[8 * 16 * LDA];
    __shared__ int s_ae[16];
    for (int e = threadIdx.x; e < 8 * 16 * KC; e += 256) {
        const int f = e / (16 * KC), rem = e % (16 * KC), row = rem / KC, k = rem % KC;
        sA[(f * 16 + row) * LDA + k] = apieces[e];
    }
    if (threadIdx.x < 16) s_ae[threadIdx.x] = aexp[threadIdx.x];
    __syncthreads();
    constexpr int NT = OC / 16 / 4, G = KC / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 cr[NT], ci[NT];
    float rowf[4];
    for (int r = 0; r < 4; ++r) rowf[r] = ldexpf(1.0f, s_ae[4 * (lane >> 4) + r] - 12);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        amp::gemm_i8<NT, G>(sA, LDA, wqe, OC, wave * NT, rowf, cr, ci);
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

// v (|v| < 2^e) -> four balanced base-256 digits of round(v 2^(30 - e)), top first
static void slice4(double v, int e, signed char d[4]) {
    long long X = llrint(ldexp(v, 30 - e));
    for (int i = 3; i >= 1; --i) {
        long long q = ((X + 128) & 255) - 128;
        d[i] = (signed char)q;
        X = (X - q) >> 8;
    }
    d[0] = (signed char)X;
}
static int exp_of(double m) {   // smallest e with m < 2^e
    int e;
    frexp(m, &e);
    return e;
}

template <int R, bool TR, int TOUT = 0>
static void run(const std::vector<signed char>& ap, const std::vector<int>& ae, const std::vector<signed char>& wp,
                const std::vector<int>& xe, const std::vector<double>& ref, const std::vector<float>& f32c) {
    signed char* dA;
    int *dae, *dxe;
    void* dW;
    float* dO;
    unsigned long long* dc;
    hipMalloc(&dA, ap.size());
    hipMalloc(&dae, ae.size() * 4);
    hipMalloc(&dxe, xe.size() * 4);
    hipMalloc(&dW, wp.size() + OC * 4);
    hipMalloc(&dO, 16 * OC * 2 * 4);
    hipMalloc(&dc, NWG * 8);
    hipMemcpy(dA, ap.data(), ap.size(), hipMemcpyHostToDevice);
    hipMemcpy(dae, ae.data(), ae.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dxe, xe.data(), xe.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW, wp.data(), wp.size(), hipMemcpyHostToDevice);
    hipMemcpy((char*)dW + wp.size(), xe.data(), OC * 4, hipMemcpyHostToDevice);   // the engine's exponent table
    for (int i = 0; i < 3; ++i) {
        if constexpr (TOUT < 0) hipLaunchKernelGGL(ki8e, dim3(NWG), dim3(256), 0, 0, dA, dae, dW, dO, dc);
        else if constexpr (TOUT) hipLaunchKernelGGL((ki8t<TOUT>), dim3(NWG), dim3(256), 0, 0, dA, dae, dW, dxe, dO, dc);
        else hipLaunchKernelGGL((ki8<R, TR>), dim3(NWG), dim3(256), 0, 0, dA, dae, dW, dxe, dO, dc);
    }
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(NWG, 0);
    hipMemcpy(c.data(), dc, NWG * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    std::vector<float> o(16 * OC * 2);
    hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
    double ei = 0, ef = 0, nrm = 0, si = 0, sf = 0;
    for (size_t i = 0; i < o.size(); ++i) {
        ei = std::max(ei, fabs(o[i] - ref[i]));
        ef = std::max(ef, fabs(f32c[i] - ref[i]));
        si += (o[i] - ref[i]) * (o[i] - ref[i]);
        sf += (f32c[i] - ref[i]) * (f32c[i] - ref[i]);
        nrm = std::max(nrm, fabs(ref[i]));
    }
    printf("int8x4 R=%d TR=%d tile-outer D=%d: cycles per GEMM median %.0f max %.0f   max|err| i8x4 %.3e f32-seq %.3e   rms i8x4 %.3e f32-seq %.3e (max|C| %.3f)\n",
           R, (int)TR, TOUT, (double)c[NWG / 2] / REPS, (double)c[NWG - 1] / REPS, ei, ef, sqrt(si / o.size()), sqrt(sf / o.size()), nrm);
    hipFree(dA); hipFree(dae); hipFree(dxe); hipFree(dW); hipFree(dO); hipFree(dc);
}

int main() {
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> A(16 * KC * 2), X(OC * KC * 2);
    for (auto& v : A) v = rnd();
    for (auto& v : X) v = rnd() * 0.0625f;
    for (int k = 0; k < KC; k += 7) A[k * 2] *= 1e-3f;   // a few small entries
    // A slices: planar [Ar s0..s3, Ai s0..s3, -Ai s0..s3][16][KC], one exponent per row
    std::vector<signed char> ap(12 * 16 * KC);
    std::vector<int> ae(16);
    for (int r = 0; r < 16; ++r) {
        double m = 0;
        for (int k = 0; k < 2 * KC; ++k) m = std::max(m, (double)fabsf(A[r * 2 * KC + k]));
        ae[r] = exp_of(m);
        for (int k = 0; k < KC; ++k) {
            signed char p[4], q[4], nq[4];
            slice4(A[(r * KC + k) * 2], ae[r], p);
            slice4(A[(r * KC + k) * 2 + 1], ae[r], q);
            slice4(-(double)A[(r * KC + k) * 2 + 1], ae[r], nq);
            for (int s = 0; s < 4; ++s) {
                ap[(s * 16 + r) * KC + k] = p[s];
                ap[((4 + s) * 16 + r) * KC + k] = q[s];
                ap[((8 + s) * 16 + r) * KC + k] = nq[s];
            }
        }
    }
    // operator slices: [ct][g][f: Xr s0..s3, Xi s0..s3][lane][16], B[k][col] = X[col][k],
    // lane = (col & 15) + 16 ((k & 63) >> 4), byte k & 15; one exponent per column
    const int G = KC / 64;
    std::vector<signed char> wp((size_t)(OC / 16) * G * 8 * 64 * 16);
    std::vector<int> xe(OC);
    for (int o = 0; o < OC; ++o) {
        double m = 0;
        for (int k = 0; k < 2 * KC; ++k) m = std::max(m, (double)fabsf(X[o * 2 * KC + k]));
        xe[o] = exp_of(m);
        for (int k = 0; k < KC; ++k) {
            signed char p[4], q[4];
            slice4(X[(o * KC + k) * 2], xe[o], p);
            slice4(X[(o * KC + k) * 2 + 1], xe[o], q);
            const int ct = o >> 4, g = k >> 6, kk = k & 63, lane = (o & 15) + 16 * (kk >> 4), j = kk & 15;
            for (int s = 0; s < 4; ++s) {
                wp[((((size_t)ct * G + g) * 8 + s) * 64 + lane) * 16 + j] = p[s];
                wp[((((size_t)ct * G + g) * 8 + 4 + s) * 64 + lane) * 16 + j] = q[s];
            }
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
    run<1, false>(ap, ae, wp, xe, ref, f32c);
    run<1, true>(ap, ae, wp, xe, ref, f32c);
    run<2, false>(ap, ae, wp, xe, ref, f32c);
    run<2, true>(ap, ae, wp, xe, ref, f32c);
    // tile-outer: the A planes without -Ai (ap's first eight planes)
    run<1, false, 2>(ap, ae, wp, xe, ref, f32c);
    run<1, false, 3>(ap, ae, wp, xe, ref, f32c);
    run<1, false, 4>(ap, ae, wp, xe, ref, f32c);
    run<1, false, 6>(ap, ae, wp, xe, ref, f32c);
    run<1, false, -1>(ap, ae, wp, xe, ref, f32c);   // the engine's gemm_i8
    return 0;
}
