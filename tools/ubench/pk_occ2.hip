// Reproducer for the two-waves-per-SIMD corruption of the packed denoiser.
//
// Each "VALU" wave runs the packed-f32 instruction mix of denoise_step_gp (amp_denoise.h): per
// step v_pk_mul_f32 + v_pk_fma_f32 for a pair of logits, v_pk_add_f32 / v_pk_mul_f32 for the
// shift, two v_exp_f32, v_pk_add_f32 for the partition sum and two broadcast v_pk_fma_f32 for the
// (re, im) sums — and writes its final registers.  The result of a lane depends only on its own
// inputs, so every run must give the same bits.  Modes (one 512- or 256-thread block per CU):
//   solo   4 VALU waves, one per SIMD                              (the reference bits)
//   mfma   4 VALU waves + 4 MFMA waves (bf16 16x16x32 chains): two waves per SIMD, one of each
//   valu2  8 VALU waves: two packed-VALU waves per SIMD
//   scal   mfma mode with the scalar (unpacked) form of the same arithmetic
// Every mode runs REPS times; the count of lanes whose bits differ from solo is printed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int STEPS = 4096;
constexpr float LOG2E = 1.4426950408889634f;

template <bool PACKED>
__device__ __forceinline__ void valu_work(const float* in, float* out, int gl) {
    float ur = in[4 * gl], ui = in[4 * gl + 1], m = in[4 * gl + 2];
    f32x2 pre = {0.7071f, -0.7071f}, pim = {0.7071f, 0.7071f};
    f32x2 s0 = {0.7071f, 0.7071f}, s1 = {-0.7071f, 0.7071f};
    asm volatile("" : "+v"(pre), "+v"(pim), "+v"(s0), "+v"(s1));
    f32x2 z2 = {0.f, 0.f}, a2 = {0.f, 0.f};
    for (int i = 0; i < STEPS; ++i) {
        if constexpr (PACKED) {
            const f32x2 u2 = {ur, ur}, v2 = {ui, ui};
            f32x2 xk = __builtin_elementwise_fma(u2, pre, v2 * pim);
            const f32x2 d = (xk - f32x2{m, m}) * f32x2{LOG2E, LOG2E};
            const f32x2 e = {__builtin_amdgcn_exp2f(d.x), __builtin_amdgcn_exp2f(d.y)};
            z2 += e;
            a2 = __builtin_elementwise_fma(s0, f32x2{e.x, e.x}, a2);
            a2 = __builtin_elementwise_fma(s1, f32x2{e.y, e.y}, a2);
        } else {
            const float x0 = fmaf(ur, pre.x, ui * pim.x), x1 = fmaf(ur, pre.y, ui * pim.y);
            const float e0 = __builtin_amdgcn_exp2f((x0 - m) * LOG2E), e1 = __builtin_amdgcn_exp2f((x1 - m) * LOG2E);
            z2.x += e0; z2.y += e1;
            a2.x = fmaf(s0.x, e0, a2.x); a2.y = fmaf(s0.y, e0, a2.y);
            a2.x = fmaf(s1.x, e1, a2.x); a2.y = fmaf(s1.y, e1, a2.y);
        }
        // feed back (keeps the chain dependent, values bounded)
        ur = ur * 0.999f + 1e-3f * a2.x / (z2.x + z2.y + 1.f);
        ui = ui * 0.999f + 1e-3f * a2.y / (z2.x + z2.y + 1.f);
    }
    out[4 * gl] = z2.x; out[4 * gl + 1] = z2.y; out[4 * gl + 2] = a2.x; out[4 * gl + 3] = a2.y;
}

__device__ __forceinline__ void mfma_work(float* sink, int gl) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (gl & 7)); b[j] = (__bf16)(0.02f * j); }
    asm volatile("" : "+v"(a), "+v"(b));
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    for (int i = 0; i < STEPS * 2; ++i) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, acc3, 0, 0, 0);
    }
    sink[gl] = acc0[0] + acc1[1] + acc2[2] + acc3[3];
}

// mode 0 solo, 1 mfma, 2 valu2, 3 scal (see the header).  Lane numbering: VALU wave w of block b
// owns gl = base + (b * 4 + w) * 64 + lane for w < 4 and NB * 256 + (b * 4 + w - 4) * 64 + lane for
// the second four (valu2), so two solo launches (base 0 and NB * 256) cover every lane.
template <int MODE>
__global__ __launch_bounds__(512, 1) void pk_occ2(const float* in, float* out, float* sink, int base) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nvw = MODE == 2 ? 8 : 4;            // VALU waves per block
    if (wave < nvw) {
        const int gl = wave < 4 ? base + (blockIdx.x * 4 + wave) * 64 + lane
                                : gridDim.x * 256 + (blockIdx.x * 4 + wave - 4) * 64 + lane;
        if constexpr (MODE == 3) valu_work<false>(in, out, gl);
        else valu_work<true>(in, out, gl);
    } else if (MODE == 1 || MODE == 3) {
        mfma_work(sink, (blockIdx.x * 4 + wave - 4) * 64 + lane);
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = ncu;
    const size_t nl = (size_t)nb * 8 * 64;        // lanes of every VALU wave of valu2
    std::vector<float> hin(4 * nl);
    srand(7);
    for (size_t i = 0; i < nl; ++i) {
        hin[4 * i] = (rand() / (float)RAND_MAX - 0.5f) * 8.f;
        hin[4 * i + 1] = (rand() / (float)RAND_MAX - 0.5f) * 8.f;
        hin[4 * i + 2] = 6.f;
        hin[4 * i + 3] = 0.f;
    }
    float *din, *dout, *dsink;
    hipMalloc(&din, 4 * nl * sizeof(float));
    hipMalloc(&dout, 4 * nl * sizeof(float));
    hipMalloc(&dsink, nl * sizeof(float));
    hipMemcpy(din, hin.data(), 4 * nl * sizeof(float), hipMemcpyHostToDevice);
    hipFuncSetAttribute((const void*)pk_occ2<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)pk_occ2<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)pk_occ2<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipFuncSetAttribute((const void*)pk_occ2<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    auto launch = [&](int mode, int base) {
        // 96 KB of (unused) dynamic LDS: one block per CU in every mode
        const dim3 g(nb), b(mode == 0 ? 256 : 512);
        const size_t lds = 96 * 1024;
        if (mode == 0) hipLaunchKernelGGL(pk_occ2<0>, g, b, lds, 0, din, dout, dsink, base);
        if (mode == 1) hipLaunchKernelGGL(pk_occ2<1>, g, b, lds, 0, din, dout, dsink, base);
        if (mode == 2) hipLaunchKernelGGL(pk_occ2<2>, g, b, lds, 0, din, dout, dsink, base);
        if (mode == 3) hipLaunchKernelGGL(pk_occ2<3>, g, b, lds, 0, din, dout, dsink, base);
    };
    auto fetch = [&](std::vector<float>& h) {
        hipDeviceSynchronize();
        h.resize(4 * nl);
        hipMemcpy(h.data(), dout, 4 * nl * sizeof(float), hipMemcpyDeviceToHost);
    };
    // references: packed and scalar forms, one VALU wave per SIMD
    std::vector<float> ref, got;
    hipMemset(dout, 0xff, 4 * nl * sizeof(float));
    launch(0, 0);
    hipDeviceSynchronize();
    launch(0, nb * 256);
    fetch(ref);
    const char* names[4] = {"solo", "mfma", "valu2", "scal"};
    std::vector<float> ref3;
    for (int mode = 0; mode < 4; ++mode) {
        long bad_total = 0, bad_runs = 0, hi = 0;
        double worst = 0.0;
        const size_t nlm = mode == 2 ? nl : (size_t)nb * 256;   // lanes the mode writes
        for (int r = 0; r < reps; ++r) {
            hipMemset(dout, 0xff, 4 * nl * sizeof(float));
            launch(mode, 0);
            fetch(got);
            if (mode == 3 && r == 0) ref3 = got;     // the scalar form: its own first run
            const std::vector<float>& R = mode == 3 ? ref3 : ref;
            long bad = 0;
            for (size_t g = 0; g < nlm; ++g)
                if (memcmp(&got[4 * g], &R[4 * g], 16) != 0) {
                    ++bad;
                    if ((g & 63) >= 48) ++hi;
                    worst = fmax(worst, fabs((double)got[4 * g]));
                }
            bad_total += bad;
            bad_runs += bad != 0;
        }
        printf("%-6s %3d runs: %ld with differing lanes, %ld lanes in all (%ld of them in lanes 48-63), max |z| among them %.3g\n",
               names[mode], reps, bad_runs, bad_total, hi, worst);
    }
    hipFree(din); hipFree(dout); hipFree(dsink);
    return 0;
}
