// VALU issue cost per wave-instruction on gfx950 at 1 and 2 waves per SIMD:
// v_fma_f32, v_pk_fma_f32, v_pk_mul_f32, v_exp_f32, v_add_f64 (16 independent chains each).
// hipcc -O3 --offload-arch=gfx950 -o /tmp/valu_rate tools/ubench/valu_rate.hip && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int IT = 256, CH = 16;

template <int OP>
__global__ void k(float* out, unsigned long long* cyc, float s) {
    f2 a[CH];
    float b[CH];
    double d[CH];
    for (int i = 0; i < CH; ++i) { a[i] = f2{s * i, s + i}; b[i] = s * i; d[i] = s * i; }
    const f2 m = f2{s, 1.0f - s}, c = f2{0.5f, 0.25f};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if constexpr (OP == 0) b[i] = __builtin_fmaf(b[i], s, 0.5f);
            else if constexpr (OP == 1) a[i] = __builtin_elementwise_fma(a[i], m, c);
            else if constexpr (OP == 2) a[i] = a[i] * m;
            else if constexpr (OP == 3) b[i] = __builtin_amdgcn_exp2f(b[i]);
            else if constexpr (OP == 4) d[i] = d[i] + (double)s;
            else if constexpr (OP == 5) b[i] = __builtin_fmaxf(b[i], s);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0.f;
    for (int i = 0; i < CH; ++i) acc += a[i].x + a[i].y + b[i] + (float)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int threads) {
    float* out; unsigned long long* cyc;
    hipMalloc(&out, 256 * threads * 4); hipMalloc(&cyc, 256 * 8);
    hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 0.999f);
    hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 0.999f);
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    unsigned long long mn = h[0];
    for (int i = 0; i < 256; ++i) mn = h[i] < mn ? h[i] : mn;
    printf("%-12s waves/SIMD %d: %.2f cycles per wave-instruction\n", name, threads / 256,
           (double)mn / (IT * CH));
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int th : {256, 512}) {
        run<0>("v_fma_f32", th); run<1>("v_pk_fma_f32", th); run<2>("v_pk_mul_f32", th);
        run<3>("v_exp_f32", th); run<4>("v_add_f64", th); run<5>("v_max_f32", th);
    }
    return 0;
}
