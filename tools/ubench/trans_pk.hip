// Hazard probe (DESIGN.md §3.8, round-5 review item 3): a transcendental result (v_exp_f32 /
// v_rcp_f32) read by a packed-f32 VALU instruction (v_pk_add_f32 / v_pk_mul_f32 of the register
// pair) F instructions later.  The two-waves-per-SIMD build of the per-point packed denoiser
// (denoise_step_gp, -DAMP_OCC2_PK=1) holds this pattern at distance 2 with no s_nop in 10 places
// (tools/ubench/hazard_scan.py on its gfx950 assembly): two v_exp_f32 write v[a], v[a+1], one
// unrelated VALU, then v_pk_add_f32 reads v[a:a+1].  LLVM's gfx950 hazard model asks one wait
// state between a trans def and a non-trans VALU use, which that unrelated instruction provides.
// Each case runs the exact sequence in inline asm (fixed registers v200-v211) and compares every
// lane's packed result with the same operation done after s_nop 7 padding.
// Partners (same SIMD, the other wave of a 512-thread block): none (256 threads), the same probe,
// a v_exp_f32 chain (trans unit busy), a packed-FMA chain, an MFMA chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int STEPS = 2048;

#define FILL1 "v_add_u32 v210, v210, 1\n"
// OP 0: two v_exp_f32 then v_pk_add_f32 of the pair; OP 1: two v_rcp_f32 then v_pk_mul_f32
template <int F, int OP>
__device__ __forceinline__ void probe(float x0, float x1, float y0, float y1, float& o0, float& o1, float& r0,
                                      float& r1) {
    asm volatile(
        "v_mov_b32 v204, %4\n"
        "v_mov_b32 v205, %5\n"
        "v_mov_b32 v206, %6\n"
        "v_mov_b32 v207, %7\n"
        "s_nop 7\n"
        ".if %8 == 0\n"
        "v_exp_f32 v200, v204\n"
        "v_exp_f32 v201, v205\n"
        ".else\n"
        "v_rcp_f32 v200, v204\n"
        "v_rcp_f32 v201, v205\n"
        ".endif\n"
        ".if %9 >= 1\n" FILL1 ".endif\n"
        ".if %9 >= 2\n" FILL1 ".endif\n"
        ".if %9 >= 3\n" FILL1 ".endif\n"
        ".if %8 == 0\n"
        "v_pk_add_f32 v[202:203], v[200:201], v[206:207]\n"
        ".else\n"
        "v_pk_mul_f32 v[202:203], v[200:201], v[206:207]\n"
        ".endif\n"
        "s_nop 7\n"
        // the same operation with the trans results long settled
        ".if %8 == 0\n"
        "v_pk_add_f32 v[208:209], v[200:201], v[206:207]\n"
        ".else\n"
        "v_pk_mul_f32 v[208:209], v[200:201], v[206:207]\n"
        ".endif\n"
        "s_nop 7\n"
        "v_mov_b32 %0, v202\n"
        "v_mov_b32 %1, v203\n"
        "v_mov_b32 %2, v208\n"
        "v_mov_b32 %3, v209\n"
        : "=v"(o0), "=v"(o1), "=v"(r0), "=v"(r1)
        : "v"(x0), "v"(x1), "v"(y0), "v"(y1), "i"(OP), "i"(F)
        : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210");
}

__device__ __forceinline__ void exp_work(float* sink, int gl) {
    float a = 0.001f * (gl & 255), b = -0.002f * (gl & 127);
    for (int i = 0; i < STEPS * 8; ++i) {
        a = __builtin_amdgcn_exp2f(a) * 0.5f - 0.25f;
        b = __builtin_amdgcn_exp2f(b) * 0.5f - 0.25f;
    }
    sink[gl] = a + b;
}

__device__ __forceinline__ void pk_work(float* sink, int gl) {
    f32x2 x = {1.0f + gl * 1e-6f, 2.0f}, m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    asm volatile("" : "+v"(x), "+v"(m), "+v"(c));
    for (int i = 0; i < STEPS * 16; ++i) x = __builtin_elementwise_fma(x, m, c);
    sink[gl] = x.x + x.y;
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

// PARTNER: 0 none (256-thread block), 1 the same probe, 2 exp chain, 3 packed-FMA chain, 4 MFMA chain
template <int F, int OP, int PARTNER>
__global__ __launch_bounds__(512, 1) void kprobe(const float* in, unsigned* bad, float* sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool prober = wave < 4 || PARTNER == 1;
    const int gl = (blockIdx.x * 8 + wave) * 64 + lane;
    if (prober) {
        unsigned nbad = 0;
        for (int i = 0; i < STEPS; ++i) {
            const float x0 = in[(gl * 4 + 0 + i) & 0xffff], x1 = in[(gl * 4 + 1 + i) & 0xffff];
            const float y0 = in[(gl * 4 + 2 + i) & 0xffff], y1 = in[(gl * 4 + 3 + i) & 0xffff];
            float o0, o1, r0, r1;
            probe<F, OP>(x0, x1, y0, y1, o0, o1, r0, r1);
            nbad += (__float_as_uint(o0) != __float_as_uint(r0)) + (__float_as_uint(o1) != __float_as_uint(r1));
        }
        bad[gl] = nbad;
    } else {
        if (PARTNER == 2) exp_work(sink, gl);
        else if (PARTNER == 3) pk_work(sink, gl);
        else if (PARTNER == 4) mfma_work(sink, gl);
        bad[gl] = 0;
    }
}

template <int F, int OP, int PARTNER>
static void run(const float* din, unsigned* dbad, float* dsink, int nb, int reps) {
    const size_t nl = (size_t)nb * 512;
    std::vector<unsigned> h(nl);
    long tot = 0, hi = 0, lanes = 0;
    for (int r = 0; r < reps; ++r) {
        hipMemset(dbad, 0, nl * 4);
        hipLaunchKernelGGL((kprobe<F, OP, PARTNER>), dim3(nb), dim3(PARTNER == 0 ? 256 : 512), 0, 0, din, dbad,
                           dsink);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), dbad, nl * 4, hipMemcpyDeviceToHost);
        for (size_t g = 0; g < nl; ++g)
            if (h[g]) { tot += h[g]; ++lanes; if ((g & 63) >= 48) ++hi; }
    }
    const char* pn[5] = {"none", "probe", "exp", "pk_fma", "mfma"};
    printf("%s fillers %d partner %-6s: %ld wrong packed results, %ld lane-runs (%ld in lanes 48-63)\n",
           OP == 0 ? "exp->pk_add" : "rcp->pk_mul", F, pn[PARTNER], tot, lanes, hi);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<float> hin(65536);
    srand(3);
    for (auto& v : hin) v = (float)(rand() % 100000) * 1e-4f - 5.0f;
    float *din, *dsink;
    unsigned* dbad;
    hipMalloc(&din, 65536 * 4);
    hipMalloc(&dbad, (size_t)ncu * 512 * 4);
    hipMalloc(&dsink, (size_t)ncu * 512 * 4);
    hipMemcpy(din, hin.data(), 65536 * 4, hipMemcpyHostToDevice);
#define RUNP(F, OP)                                    \
    run<F, OP, 0>(din, dbad, dsink, ncu, reps);        \
    run<F, OP, 1>(din, dbad, dsink, ncu, reps);        \
    run<F, OP, 2>(din, dbad, dsink, ncu, reps);        \
    run<F, OP, 3>(din, dbad, dsink, ncu, reps);        \
    run<F, OP, 4>(din, dbad, dsink, ncu, reps);
    RUNP(0, 0) RUNP(1, 0) RUNP(2, 0) RUNP(0, 1) RUNP(1, 1) RUNP(2, 1)
    hipFree(din); hipFree(dbad); hipFree(dsink);
    return 0;
}
