// Hazard probe: a packed-f32 VALU write (v_pk_add_f32 v[a:a+1]) read by DPP
// moves of its two halves F instructions later — the pattern the compiler emitted for the
// two-sections-at-a-time group sums of denoise_step_gp in the two-waves-per-SIMD build
// (v_pk_add_f32 v[34:35]; one unrelated VALU; v_mov_b32_dpp v.., v34; v_mov_b32_dpp v.., v35).
// The generic gfx9 rule asks 2 wait states between a VALU write and a DPP read of the same
// VGPR; the compiler counts the unrelated instructions as wait states.  Each case runs the
// exact sequence in inline asm (fixed registers v200-v206, so no compiler padding) and checks
// every lane's two DPP results against the host's model:
//   dpp quad_perm [2,3,0,1]: lane l reads lane (l & ~3) | ((l & 3) ^ 2).
// Partners (same SIMD, the other wave of a 512-thread block): none (256 threads), the same probe,
// an MFMA chain, a packed-FMA chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int STEPS = 2048;

#define FILL1 "v_add_u32 v204, v204, 1\n"
template <int F>
__device__ __forceinline__ void probe(float a0, float a1, float b0, float b1, float& o0, float& o1) {
    asm volatile(
        "v_mov_b32 v200, %2\n"
        "v_mov_b32 v201, %3\n"
        "v_mov_b32 v202, %4\n"
        "v_mov_b32 v203, %5\n"
        "s_nop 7\n"
        "v_pk_add_f32 v[200:201], v[200:201], v[202:203]\n"
#if 1
        ".if %6 >= 1\n" FILL1 ".endif\n"
        ".if %6 >= 2\n" FILL1 ".endif\n"
        ".if %6 >= 3\n" FILL1 ".endif\n"
        ".if %6 >= 4\n" FILL1 ".endif\n"
#endif
        "v_mov_b32_dpp v205, v200 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_mov_b32_dpp v206, v201 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "s_nop 7\n"
        "v_mov_b32 %0, v205\n"
        "v_mov_b32 %1, v206\n"
        : "=v"(o0), "=v"(o1)
        : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "i"(F)
        : "v200", "v201", "v202", "v203", "v204", "v205", "v206");
}

__device__ __forceinline__ void mfma_work(float* sink, int gl) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (gl & 7)); b[j] = (__bf16)(0.02f * j); }
    asm volatile("" : "+v"(a), "+v"(b));
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
    for (int i = 0; i < STEPS * 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c1, 0, 0, 0);
    }
    sink[gl] = c0[0] + c1[1];
}

__device__ __forceinline__ void pk_work(float* sink, int gl) {
    f32x2 x = {1.0f + gl * 1e-6f, 2.0f}, m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    asm volatile("" : "+v"(x), "+v"(m), "+v"(c));
    for (int i = 0; i < STEPS * 16; ++i) x = __builtin_elementwise_fma(x, m, c);
    sink[gl] = x.x + x.y;
}

// PARTNER: 0 none (256-thread block), 1 the same probe, 2 MFMA chain, 3 packed-FMA chain
template <int F, int PARTNER>
__global__ __launch_bounds__(512, 1) void kprobe(const float* in, unsigned* bad, float* sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool prober = wave < 4 || PARTNER == 1;
    const int gl = (blockIdx.x * 8 + wave) * 64 + lane;
    if (prober) {
        unsigned nbad = 0;
        const int src = (lane & ~3) | ((lane & 3) ^ 2);
        for (int i = 0; i < STEPS; ++i) {
            const float a0 = in[(gl * 4 + 0) & 0xffff] + i, a1 = in[(gl * 4 + 1) & 0xffff] - i;
            const float b0 = in[(gl * 4 + 2) & 0xffff], b1 = in[(gl * 4 + 3) & 0xffff];
            float o0, o1;
            probe<F>(a0, a1, b0, b1, o0, o1);
            // expected: the partner lane's sums (same formulas, its own inputs)
            const int gs = (blockIdx.x * 8 + wave) * 64 + src;
            const float e0 = (in[(gs * 4 + 0) & 0xffff] + i) + in[(gs * 4 + 2) & 0xffff];
            const float e1 = (in[(gs * 4 + 1) & 0xffff] - i) + in[(gs * 4 + 3) & 0xffff];
            nbad += (__float_as_uint(o0) != __float_as_uint(e0)) + (__float_as_uint(o1) != __float_as_uint(e1));
        }
        bad[gl] = nbad;
    } else if (PARTNER == 2) {
        mfma_work(sink, gl);
        bad[gl] = 0;
    } else if (PARTNER == 3) {
        pk_work(sink, gl);
        bad[gl] = 0;
    }
}

template <int F, int PARTNER>
static void run(const float* din, unsigned* dbad, float* dsink, int nb, int reps) {
    const size_t nl = (size_t)nb * 512;
    std::vector<unsigned> h(nl);
    long tot = 0, hi = 0, lanes = 0;
    hipFuncSetAttribute((const void*)kprobe<F, PARTNER>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    for (int r = 0; r < reps; ++r) {
        hipMemset(dbad, 0, nl * 4);
        hipLaunchKernelGGL((kprobe<F, PARTNER>), dim3(nb), dim3(PARTNER == 0 ? 256 : 512), 96 * 1024, 0, din, dbad,
                           dsink);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), dbad, nl * 4, hipMemcpyDeviceToHost);
        for (size_t g = 0; g < nl; ++g)
            if (h[g]) { tot += h[g]; ++lanes; if ((g & 63) >= 48) ++hi; }
    }
    const char* pn[4] = {"none", "probe", "mfma", "pk_fma"};
    printf("fillers %d partner %-6s: %ld wrong DPP results, %ld lane-runs (%ld in lanes 48-63)\n", F, pn[PARTNER], tot,
           lanes, hi);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<float> hin(65536);
    srand(3);
    for (auto& v : hin) v = (float)(rand() % 100000) * 0.25f;
    float *din, *dsink;
    unsigned* dbad;
    hipMalloc(&din, 65536 * 4);
    hipMalloc(&dbad, (size_t)ncu * 512 * 4);
    hipMalloc(&dsink, (size_t)ncu * 512 * 4);
    hipMemcpy(din, hin.data(), 65536 * 4, hipMemcpyHostToDevice);
#define RUNF(F)                                      \
    run<F, 0>(din, dbad, dsink, ncu, reps);          \
    run<F, 1>(din, dbad, dsink, ncu, reps);          \
    run<F, 2>(din, dbad, dsink, ncu, reps);          \
    run<F, 3>(din, dbad, dsink, ncu, reps);
    RUNF(0) RUNF(1) RUNF(2) RUNF(3) RUNF(4)
    hipFree(din); hipFree(dbad); hipFree(dsink);
    return 0;
}
