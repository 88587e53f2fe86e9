// Micro-benchmark of the persistent engine's denoiser phase (diagnostic tool, not shipped):
// 256 workgroups x 16 trials, rows in LDS exactly as vamp_persist holds them, the denoiser
// repeated `reps` times; prints median cycles per call (s_memtime) per workgroup.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -shared -fPIC -o libdenoise_ubench.so denoise_ubench.hip
//   python -c "import ctypes; ctypes.CDLL('tools/ubench/libdenoise_ubench.so').ubench_main()"
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <algorithm>

#include "../../amp-sparc-spatialmodulation_amd/csrc/amp_vamp.h"

using namespace amp;

template <int KK, int U, int NWV, bool PK>
__global__ __launch_bounds__(64 * NWV, 1) void ub(const float* rin, Const c, int N, int M, float inv, int reps,
                                                unsigned long long* out, double* sink) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int ldr = 2 * N + 4, spr = N / M, L = spr;
    float* sR = lds;
    float* sX = sR + 16 * ldr;
    float* v0 = sX + 16 * ldr;
    float* v1 = v0 + 16 * N;
    float* sm = v1 + 16 * N;
    float* sa = sm + 16 * L;
    for (int e = threadIdx.x; e < 16 * 2 * N; e += blockDim.x) {
        const int row = e / (2 * N), col = e % (2 * N);
        sR[row * ldr + col] = rin[((size_t)blockIdx.x * 16 + row) * 2 * N + col];
    }
    for (int e = threadIdx.x; e < 16 * N; e += blockDim.x) v1[e] = 0.1f;
    __syncthreads();
    PartAcc pa;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        PDenoisePolicy pol{sR, sX, (r & 1) ? v1 : v0, (r & 1) ? v0 : v1, sm, sa, ldr, M, 31 - __builtin_clz(spr), N, inv};
        denoise_sections_u<true, KK, U, PK>(pol, 16 * spr, M, c, pa);
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = (t1 - t0) / reps;
    part_wave_reduce(pa);
    if ((threadIdx.x & 63) == 0) sink[blockIdx.x * NWV + (threadIdx.x >> 6)] = pa.sumvar + pa.notclose;
}

template <int KK, int U, int NWV, bool PK>
static void run(const char* tag, const float* dr, const Const& c, int N, int M, float inv, unsigned long long* dout,
                double* dsink) {
    const int nwg = 256, reps = 20;
    const size_t lds = (size_t)(2 * 16 * (2 * N + 4) + 2 * 16 * N + 2 * 16 * (N / M)) * 4;
    hipFuncSetAttribute((const void*)ub<KK, U, NWV, PK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((ub<KK, U, NWV, PK>), dim3(nwg), dim3(64 * NWV), lds, 0, dr, c, N, M, inv, reps, dout, dsink);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((ub<KK, U, NWV, PK>), dim3(nwg), dim3(64 * NWV), lds, 0, dr, c, N, M, inv, reps, dout, dsink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(nwg);
    hipMemcpy(h.data(), dout, nwg * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-28s K=%2d U=%d waves=%d pk=%d  median %7llu cyc/call  p90 %7llu  (kernel %.3f ms / %d reps)\n", tag, KK, U, NWV, (int)PK,
           h[nwg / 2], h[nwg * 9 / 10], ms, reps);
}

extern "C" int ubench_main() {
    const int N = 256, M = 32, B = 4096;
    // 16-QAM of config.py:111 (with its duplicate point), normalised
    const double q[16][2] = {{1, 1}, {1, -1}, {-1, 1}, {-1, -1}, {3, 1}, {3, -1}, {-3, 1}, {-3, -1},
                             {3, 3}, {3, -3}, {-3, 3}, {-3, -3}, {1, 3}, {-1, 3}, {-1, 3}, {-1, -3}};
    double p = 0;
    for (auto& v : q) p += v[0] * v[0] + v[1] * v[1];
    p = sqrt(p / 16);
    Const c;
    c.K = 16;
    for (int k = 0; k < 16; ++k) { c.re[k] = (float)(q[k][0] / p); c.im[k] = (float)(q[k][1] / p); }
    std::vector<float> r((size_t)B * 2 * N);
    srand(1);
    for (auto& v : r) v = (float)((rand() / (double)RAND_MAX - 0.5) * 0.4);
    for (int t = 0; t < B; ++t)        // one active position per section with a symbol
        for (int s = 0; s < N / M; ++s) {
            const int m = (t * 7 + s * 3) % M, k = (t + s) % 16;
            r[((size_t)t * N + s * M + m) * 2] += c.re[k];
            r[((size_t)t * N + s * M + m) * 2 + 1] += c.im[k];
        }
    float* dr;
    unsigned long long* dout;
    double* dsink;
    hipMalloc(&dr, r.size() * 4);
    hipMalloc(&dout, 256 * 8);
    hipMalloc(&dsink, 256 * 8 * 8);
    hipMemcpy(dr, r.data(), r.size() * 4, hipMemcpyHostToDevice);
    const float inv = 1.0f / 0.02f;
    c.grid = 0; c.gfull = 0;
    run<16, 2, 4, true>("cfg4 16QAM direct", dr, c, N, M, inv, dout, dsink);
    run<16, 2, 8, true>("cfg4 16QAM direct", dr, c, N, M, inv, dout, dsink);
    grid_decompose(c);
    printf("grid %d full %d\n", c.grid, c.gfull);
    run<16, 1, 4, true>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 2, 4, true>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 2, 4, false>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 1, 8, false>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 2, 8, true>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 2, 8, false>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    run<16, 1, 16, false>("cfg4 16QAM grid", dr, c, N, M, inv, dout, dsink);
    fflush(stdout);
    return 0;
}
