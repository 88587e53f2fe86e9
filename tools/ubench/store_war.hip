// Hazard probe: a VALU write of a vector-memory store's DATA register F
// instructions after the store issued (write-after-read on the store data).  LLVM's gfx950 model
// inserts no wait state for it (tools/ubench/pair_ubench.hip's granule stores:
// `buffer_store_dwordx4 v[12:15] ...` followed at once by `v_pk_mov_b32 v[12:13], ...`).
// Each case stores v[200:203] (global dwordx4 / x3 / x2 / dword, LDS b128 / b64), overwrites all
// four registers F fillers later (VALU, or s_nop 0), and compares the stored words with the values
// the store was issued with.
// Partners (the other wave of the SIMD in a 512-thread block): none, the same probe.
// hipcc -O3 --offload-arch=gfx950 -o bin/store_war tools/ubench/store_war.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int STEPS = 1024;

// W: 0 global_store_dwordx4, 1 global_store_dwordx2, 2 global_store_dword, 3 global_store_dwordx3,
// 4 ds_write_b128, 5 ds_write_b64, 6 buffer_store_dwordx4; SC1: write-through (global stores);
// NOP: the fillers are s_nop 0 instead of v_add_u32
template <int F, int W, int SC1, int NOP = 0>
__device__ __forceinline__ void probe(float* st, unsigned lds_addr, float x0, float x1, float x2, float x3) {
    asm volatile(
        "v_mov_b32 v200, %1\n"
        "v_mov_b32 v201, %2\n"
        "v_mov_b32 v202, %3\n"
        "v_mov_b32 v203, %4\n"
        "s_nop 7\n"
        ".if %6 == 0\n"
        ".if %7\n global_store_dwordx4 %0, v[200:203], off sc1\n .else\n global_store_dwordx4 %0, v[200:203], off\n .endif\n"
        ".elseif %6 == 1\n"
        ".if %7\n global_store_dwordx2 %0, v[200:201], off sc1\n .else\n global_store_dwordx2 %0, v[200:201], off\n .endif\n"
        ".elseif %6 == 2\n"
        ".if %7\n global_store_dword %0, v200, off sc1\n .else\n global_store_dword %0, v200, off\n .endif\n"
        ".elseif %6 == 3\n"
        ".if %7\n global_store_dwordx3 %0, v[200:202], off sc1\n .else\n global_store_dwordx3 %0, v[200:202], off\n .endif\n"
        ".elseif %6 == 4\n"
        "ds_write_b128 %8, v[200:203]\n"
        ".else\n"
        "ds_write_b64 %8, v[200:201]\n"
        ".endif\n"
        ".rept %5\n"
        ".if %9\n s_nop 0\n .else\n v_add_u32 v204, v204, 1\n .endif\n"
        ".endr\n"
        "v_mov_b32 v200, 0\n"
        "v_mov_b32 v201, 0\n"
        "v_mov_b32 v202, 0\n"
        "v_mov_b32 v203, 0\n"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n"
        :
        : "v"(st), "v"(x0), "v"(x1), "v"(x2), "v"(x3), "i"(F), "i"(W), "i"(SC1), "v"(lds_addr), "i"(NOP)
        : "v200", "v201", "v202", "v203", "v204", "memory");
}

template <int F, int W, int SC1, int PARTNER, int NOP>
__global__ __launch_bounds__(512, 1) void kprobe(const float* in, unsigned* bad, float* stbuf) {
    __shared__ float sl[512 * 4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool prober = wave < 4 || PARTNER == 1;
    const int gl = (blockIdx.x * 8 + wave) * 64 + lane;
    if (!prober) { bad[gl] = 0; return; }
    unsigned nbad = 0;
    float* p = stbuf + 4 * gl;
    for (int i = 0; i < STEPS; ++i) {
        const float x0 = in[(gl * 4 + i) & 0xffff] + 1.0f, x1 = in[(gl * 4 + 1 + i) & 0xffff] + 1.0f;
        const float x2 = in[(gl * 4 + 2 + i) & 0xffff] + 1.0f, x3 = in[(gl * 4 + 3 + i) & 0xffff] + 1.0f;
        float* q = sl + 4 * threadIdx.x;
        probe<F, W, SC1, NOP>(p, (unsigned)(size_t)q, x0, x1, x2, x3);
        float v0, v1, v2, v3;
        if (W >= 4) {
            v0 = q[0]; v1 = q[1]; v2 = q[2]; v3 = q[3];
        } else {
            v0 = __builtin_nontemporal_load(p); v1 = __builtin_nontemporal_load(p + 1);
            v2 = __builtin_nontemporal_load(p + 2); v3 = __builtin_nontemporal_load(p + 3);
        }
        const int nw = (W == 0 || W == 4) ? 4 : W == 3 ? 3 : (W == 1 || W == 5) ? 2 : 1;
        nbad += (v0 != x0) + (nw >= 2 && v1 != x1) + (nw >= 3 && v2 != x2) + (nw >= 4 && v3 != x3);
    }
    bad[gl] = nbad;
}

template <int F, int W, int SC1, int PARTNER, int NOP = 0>
static void run(const float* din, unsigned* dbad, float* dst, int nb, int reps) {
    const size_t nl = (size_t)nb * 512;
    std::vector<unsigned> h(nl);
    long tot = 0, lanes = 0;
    for (int r = 0; r < reps; ++r) {
        hipMemset(dbad, 0, nl * 4);
        hipLaunchKernelGGL((kprobe<F, W, SC1, PARTNER, NOP>), dim3(nb), dim3(PARTNER == 0 ? 256 : 512), 0, 0, din, dbad, dst);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), dbad, nl * 4, hipMemcpyDeviceToHost);
        for (size_t g = 0; g < nl; ++g)
            if (h[g]) { tot += h[g]; ++lanes; }
    }
    const char* wn[6] = {"global_store_dwordx4", "global_store_dwordx2", "global_store_dword", "global_store_dwordx3",
                         "ds_write_b128", "ds_write_b64"};
    printf("%s%s -> data overwritten after %d %s, partner %-5s: %ld wrong words, %ld lane-runs\n", wn[W],
           SC1 && W < 4 ? " sc1" : "", F, NOP ? "s_nop 0" : "VALU fillers", PARTNER ? "probe" : "none", tot, lanes);
    fflush(stdout);
}

#define RUNF(W, SC1, F) run<F, W, SC1, 0>(din, dbad, dst, ncu, reps); run<F, W, SC1, 1>(din, dbad, dst, ncu, reps);
#define RUNW(W, SC1) RUNF(W, SC1, 0) RUNF(W, SC1, 1) RUNF(W, SC1, 2) RUNF(W, SC1, 4)
#define RUNN(W, F) run<F, W, 1, 1, 1>(din, dbad, dst, ncu, reps);

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<float> hin(65536);
    srand(7);
    for (auto& v : hin) v = (float)(rand() % 100000) * 1e-4f;
    float *din, *dst;
    unsigned* dbad;
    hipMalloc(&din, 65536 * 4);
    hipMalloc(&dbad, (size_t)ncu * 512 * 4);
    hipMalloc(&dst, (size_t)ncu * 512 * 16);
    hipMemcpy(din, hin.data(), 65536 * 4, hipMemcpyHostToDevice);
    RUNW(0, 1) RUNW(0, 0) RUNW(1, 1) RUNW(2, 1) RUNW(3, 1) RUNW(4, 0) RUNW(5, 0)
    RUNN(0, 1) RUNN(0, 2) RUNN(0, 3) RUNN(3, 1) RUNN(3, 2) RUNN(4, 1) RUNN(4, 2)
    hipFree(din); hipFree(dbad); hipFree(dst);
    return 0;
}
