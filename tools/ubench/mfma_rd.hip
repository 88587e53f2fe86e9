// Hazard probe: an MFMA result (v_mfma_f32_16x16x32_bf16, the engines'
// GEMM instruction) read by a VALU or VMEM instruction F unrelated VALU instructions after the
// MFMA issued.  Found with tools/ubench/pair_ubench.hip: a buffer_store whose data was gathered
// by v_mov_b32 / v_mov_b64 / v_pk_mov_b32 from the accumulators right after a GEMM's last MFMAs
// (the wait states LLVM's gfx950 hazard model inserted) stored wrong partial sums in every run;
// 32 wait states after the GEMM removed every error.  Each case runs the exact sequence in inline
// asm (fixed registers v200-v215) and compares every lane's value with the accumulator read after
// s_nop padding.  Consumers: 0 v_mov_b32, 1 v_mov_b64, 2 v_pk_mov_b32, 3 v_add_f32, 4 the
// accumulator stored by global_store_dword; 5 / 6 / 7: a VALU write of the last MFMA's SrcB / SrcA
// / SrcB (64-bit move) F fillers after it (write-after-read), the result against the same chain
// computed beforehand (`mfma_rd REPS 1`).  Partners (the other wave of the SIMD in a 512-thread
// block): none (256 threads), the same probe, an MFMA chain.
// hipcc -O3 --offload-arch=gfx950 -o bin/mfma_rd tools/ubench/mfma_rd.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int STEPS = 1024;

// CH dependent MFMAs into v[208:211], then F fillers, then the consumer OP.  o: the consumer's
// value of accumulator element 3 (the stored word for OP 4), r: element 3 long settled.
template <int F, int OP, int CH>
__device__ __forceinline__ void probe(unsigned a0, unsigned a1, unsigned b0, unsigned b1, float c, float* st,
                                      float& o, float& r) {
    asm volatile(
        "v_mov_b32 v200, %3\n"
        "v_mov_b32 v201, %4\n"
        "v_mov_b32 v202, %3\n"
        "v_mov_b32 v203, %4\n"
        "v_mov_b32 v204, %5\n"
        "v_mov_b32 v205, %6\n"
        "v_mov_b32 v206, %6\n"
        "v_mov_b32 v207, %5\n"
        "v_mov_b32 v208, %7\n"
        "v_mov_b32 v209, %7\n"
        "v_mov_b32 v210, %7\n"
        "v_mov_b32 v211, %7\n"
        ".if %9 >= 5\n"
        // the reference: the same MFMA chain into v[216:219], settled
        "v_mov_b32 v216, %7\n"
        "v_mov_b32 v217, %7\n"
        "v_mov_b32 v218, %7\n"
        "v_mov_b32 v219, %7\n"
        "s_nop 7\n"
        ".rept %10\n"
        "v_mfma_f32_16x16x32_bf16 v[216:219], v[200:203], v[204:207], v[216:219]\n"
        ".endr\n"
        "s_nop 7\n"
        "s_nop 7\n"
        "s_nop 7\n"
        ".endif\n"
        "s_nop 7\n"
        ".rept %10\n"
        "v_mfma_f32_16x16x32_bf16 v[208:211], v[200:203], v[204:207], v[208:211]\n"
        ".endr\n"
        ".rept %8\n"
        "v_add_u32 v212, v212, 1\n"
        ".endr\n"
        ".if %9 == 0\n"
        "v_mov_b32 v214, v211\n"
        ".elseif %9 == 1\n"
        "v_mov_b64 v[214:215], v[210:211]\n"
        "v_mov_b32 v214, v215\n"
        ".elseif %9 == 2\n"
        "v_pk_mov_b32 v[214:215], v[210:211], v[210:211] op_sel:[1,0]\n"
        ".elseif %9 == 3\n"
        "v_add_f32 v214, v211, 0\n"
        ".elseif %9 == 4\n"
        "global_store_dword %2, v211, off\n"
        "v_mov_b32 v214, 0\n"
        ".elseif %9 == 5\n"
        "v_mov_b32 v204, 0\n"          // WAR: overwrite the last MFMA's SrcB
        "v_mov_b32 v205, 0\n"
        ".elseif %9 == 6\n"
        "v_mov_b32 v200, 0\n"          // WAR: overwrite the last MFMA's SrcA
        "v_mov_b32 v201, 0\n"
        ".else\n"
        "v_mov_b64 v[204:205], 0\n"    // WAR: SrcB by a 64-bit move
        ".endif\n"
        "s_nop 7\n"
        "s_nop 7\n"
        "s_nop 7\n"
        "s_nop 7\n"
        ".if %9 >= 5\n"
        "v_mov_b32 %0, v211\n"
        "v_mov_b32 %1, v219\n"
        ".else\n"
        "v_mov_b32 %0, v214\n"
        "v_mov_b32 %1, v211\n"
        ".endif\n"
        "s_waitcnt vmcnt(0)\n"
        : "=v"(o), "=v"(r)
        : "v"(st), "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(c), "i"(F), "i"(OP), "i"(CH)
        : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212",
          "v213", "v214", "v215", "v216", "v217", "v218", "v219", "memory");
}

__device__ __forceinline__ void mfma_work(float* sink, int gl) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (gl & 7)); b[j] = (__bf16)(0.02f * j); }
    asm volatile("" : "+v"(a), "+v"(b));
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
    for (int i = 0; i < STEPS * 8; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c1, 0, 0, 0);
    }
    sink[gl] = c0[0] + c1[1];
}

// PARTNER: 0 none (256-thread block), 1 the same probe, 2 MFMA chain
template <int F, int OP, int CH, int PARTNER>
__global__ __launch_bounds__(512, 1) void kprobe(const unsigned* in, unsigned* bad, float* sink, float* stbuf) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool prober = wave < 4 || PARTNER == 1;
    const int gl = (blockIdx.x * 8 + wave) * 64 + lane;
    if (prober) {
        unsigned nbad = 0;
        for (int i = 0; i < STEPS; ++i) {
            const unsigned a0 = in[(gl * 4 + i) & 0xffff], a1 = in[(gl * 4 + 1 + i) & 0xffff];
            const unsigned b0 = in[(gl * 4 + 2 + i) & 0xffff], b1 = in[(gl * 4 + 3 + i) & 0xffff];
            const float c = __uint_as_float(in[(gl + 7 * i) & 0xffff] & 0x3fffffffu);
            float o, r;
            probe<F, OP, CH>(a0, a1, b0, b1, c, stbuf + gl, o, r);
            if (OP == 4) o = __builtin_nontemporal_load(stbuf + gl);
            nbad += __float_as_uint(o) != __float_as_uint(r);
        }
        bad[gl] = nbad;
    } else {
        if (PARTNER == 2) mfma_work(sink, gl);
        bad[gl] = 0;
    }
}

template <int F, int OP, int CH, int PARTNER>
static void run(const unsigned* din, unsigned* dbad, float* dsink, float* dst, int nb, int reps) {
    const size_t nl = (size_t)nb * 512;
    std::vector<unsigned> h(nl);
    long tot = 0, lanes = 0;
    for (int r = 0; r < reps; ++r) {
        hipMemset(dbad, 0, nl * 4);
        hipLaunchKernelGGL((kprobe<F, OP, CH, PARTNER>), dim3(nb), dim3(PARTNER == 0 ? 256 : 512), 0, 0, din, dbad,
                           dsink, dst);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), dbad, nl * 4, hipMemcpyDeviceToHost);
        for (size_t g = 0; g < nl; ++g)
            if (h[g]) { tot += h[g]; ++lanes; }
    }
    const char* pn[3] = {"none", "probe", "mfma"};
    const char* on[8] = {"v_mov_b32", "v_mov_b64", "v_pk_mov_b32", "v_add_f32", "global_store", "WAR srcB", "WAR srcA", "WAR srcB b64"};
    printf("mfma x%d -> %-12s fillers %2d partner %-5s: %ld wrong of %ld, %ld lane-runs\n", CH, on[OP], F, pn[PARTNER],
           tot, (long)reps * nl / (PARTNER == 1 ? 1 : 2) * STEPS, lanes);
    fflush(stdout);
}

#define RUNF(OP, CH, F)                                     \
    run<F, OP, CH, 0>(din, dbad, dsink, dst, ncu, reps);    \
    run<F, OP, CH, 1>(din, dbad, dsink, dst, ncu, reps);    \
    run<F, OP, CH, 2>(din, dbad, dsink, dst, ncu, reps);
#define RUNW(OP, CH) RUNF(OP, CH, 0) RUNF(OP, CH, 1) RUNF(OP, CH, 2) RUNF(OP, CH, 3) RUNF(OP, CH, 4) RUNF(OP, CH, 6) RUNF(OP, CH, 8)
#define RUNOP(OP, CH) RUNF(OP, CH, 0) RUNF(OP, CH, 2) RUNF(OP, CH, 4) RUNF(OP, CH, 6) RUNF(OP, CH, 8) \
    RUNF(OP, CH, 10) RUNF(OP, CH, 12) RUNF(OP, CH, 16)

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<unsigned> hin(65536);
    srand(5);
    for (auto& v : hin) v = ((unsigned)rand() & 0x3f7f3f7fu) | 0x3c003c00u;   // bf16 pairs in [2^-7, 2)
    unsigned *din, *dbad;
    float *dsink, *dst;
    hipMalloc(&din, 65536 * 4);
    hipMalloc(&dbad, (size_t)ncu * 512 * 4);
    hipMalloc(&dsink, (size_t)ncu * 512 * 4);
    hipMalloc(&dst, (size_t)ncu * 512 * 4);
    hipMemcpy(din, hin.data(), 65536 * 4, hipMemcpyHostToDevice);
    const int which = argc > 2 ? atoi(argv[2]) : 0;
    if (which == 0) { RUNOP(0, 1) RUNOP(1, 1) RUNOP(2, 1) RUNOP(3, 1) RUNOP(4, 1) RUNOP(0, 4) RUNOP(4, 4) }
    else { RUNW(5, 1) RUNW(6, 1) RUNW(7, 1) RUNW(5, 4) }
    hipFree(din); hipFree(dbad); hipFree(dsink); hipFree(dst);
    return 0;
}
