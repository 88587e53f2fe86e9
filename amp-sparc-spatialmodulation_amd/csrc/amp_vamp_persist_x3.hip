// amp_vamp_persist_x3.hip — the persistent VAMP engine with both per-iteration GEMMs on the
// split-precision bf16x3 engine (amp_persist.h gemm_x3); its own translation unit so that the
// f32 and bf16x3 instantiations of vamp_persist compile in parallel.  One wave per SIMD.
#include "amp_vamp_persist_kernel.h"

namespace amp {

// N = 256: eight waves per workgroup (two per SIMD, 256 registers each, half the column tiles per
// wave) by default — the VALU phases (denoiser, plane builds) issue at twice the rate of one wave
// per SIMD, and the GEMMs' operator stream hides better (80.6k -> 70.2k cycles per
// cfg4 iteration).  AMP_VAMP_X3_WAVES=4 keeps the four-wave form (A/B runs).
static bool x3_waves8() {
    static const bool v = [] {
        const char* e = getenv("AMP_VAMP_X3_WAVES");
        return !(e && atoi(e) == 4);
    }();
    return v;
}

int persist_dispatch_x3(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.N) {
    case 64:   // the two-per-CU build for every N = 64 launch, so that one epoch and side-by-side
               // epochs run the same arithmetic (bit-identical results, tests/test_gpu_epochs.py)
        return persist_wg2() ? persist_launch_nt<2, 4, true, 2>(P, dc, st) : persist_launch_nt<2, 4, true>(P, dc, st);
    case 128: return persist_launch_nt<4, 4, true>(P, dc, st);
    case 256:
        return x3_waves8() ? persist_launch_nt<4, 8, true>(P, dc, st) : persist_launch_nt<8, 4, true>(P, dc, st);
    default: break;
    }
    set_error("vamp_persist (bf16x3): N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp

namespace amp {

// y~ = (s Uh) y (vamp.py:22) for the split-precision engines, as its own launch on the bf16x3
// GEMM (24-bit operands, as the engine's own GEMMs): one workgroup per 16 trials, the y rows
// split into six bf16 planes in LDS (n complex per row), the operator s Uh x3-packed (K = n,
// O = k), the result in the accumulator layout straight to ytil.  Replaces the f32-MFMA
// gemm_store launch (47.7 us per cfg4 step at 0.56 of the f32 peak, profiles/r04_cfg4_vamp_x3.txt).
// rows_per_op / wq_stride: side-by-side epochs with a channel each use the operator of their
// epoch, wq + (row / rows_per_op) * wq_stride bytes (rows_per_op a multiple of PBM).
template <int NC, int G, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 1) void ytil_x3_kernel(const float* __restrict__ y, int rows, const void* wq,
                                                               float* __restrict__ ytil, int k, int rows_per_op,
                                                               long long wq_stride) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned short* sP = reinterpret_cast<unsigned short*>(lds);
    constexpr int n = 32 * G;
    const int ldx = pl_ldx(n);
    const int row0 = blockIdx.x * PBM;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int e = tid; e < PBM * (n >> 3); e += 64 * NWV) {   // 8 complex values per item, rows fastest
        const int row = e % PBM, j0 = 8 * (e / PBM);
        float re[8], im[8];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row0 + row < rows) v = *reinterpret_cast<const float4*>(y + (size_t)(row0 + row) * 2 * n + 2 * j0 + 4 * h);
            re[2 * h] = v.x; im[2 * h] = v.y; re[2 * h + 1] = v.z; im[2 * h + 1] = v.w;
        }
        x3_store8(sP, ldx, row, j0, re, im);
    }
    __syncthreads();
    f32x4 cr[NC], ci[NC];
    const void* wop = (const char*)wq + (long long)(row0 / rows_per_op) * wq_stride;
    gemm_x3<NC, G, 1>(sP, ldx, wop, wave * NC, cr, ci);
#pragma unroll
    for (int t = 0; t < NC; ++t) {
        const int o = 16 * (wave * NC + t) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = row0 + 4 * (lane >> 4) + r;
            if (row < rows) *reinterpret_cast<float2*>(ytil + (size_t)row * 2 * k + 2 * o) = make_float2(cr[t][r], ci[t][r]);
        }
    }
}

template <int NC, int G, int NWV = 4>
static int ytil_x3_launch_t(const float* y, int rows, const void* wq, float* ytil, int k, int rows_per_op,
                            long long wq_stride, hipStream_t st) {
    const void* fn = (const void*)ytil_x3_kernel<NC, G, NWV>;
    const size_t lds = (size_t)6 * PBM * pl_ldx(32 * G) * 2;
    static int attr = -1;   // once per instantiation (single-threaded host use, like the rest of the ABI)
    if (attr < 0) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("ytil_x3: hipFuncSetAttribute: %s", hipGetErrorString(e));
            return AMP_E_LAUNCH;
        }
        attr = 1;
    }
    hipLaunchKernelGGL((ytil_x3_kernel<NC, G, NWV>), dim3(cdiv(rows, PBM)), dim3(64 * NWV), lds, st, y, rows, wq, ytil, k,
                       rows_per_op, wq_stride);
    AMP_LAUNCH_CHECK("ytil_x3");
    return AMP_OK;
}

// The shapes of the split-precision engines (k == N, n == 2N): false for any other.
bool ytil_x3_fits(int n, int k) { return n == 2 * k && (k == 64 || k == 128 || k == 256); }

int ytil_x3_launch(const float* y, int n, int rows, const void* wq, float* ytil, int k, hipStream_t st,
                   int rows_per_op, long long wq_stride) {
    if (rows_per_op <= 0) rows_per_op = rows;   // one operator for every row
    AMP_REQUIRE(rows_per_op % PBM == 0 || rows_per_op >= rows, "ytil_x3: rows per operator %d", rows_per_op);
    switch (k) {
    case 64: return ytil_x3_launch_t<1, 4>(y, rows, wq, ytil, k, rows_per_op, wq_stride, st);
    case 128: return ytil_x3_launch_t<2, 8>(y, rows, wq, ytil, k, rows_per_op, wq_stride, st);
    case 256:   // eight waves (two per SIMD) hide the operator stream better, as in the engine
        return ytil_x3_launch_t<2, 16, 8>(y, rows, wq, ytil, k, rows_per_op, wq_stride, st);
    default: break;
    }
    set_error("ytil_x3: n = %d / k = %d not supported", n, k);
    return AMP_E_ARG;
}

}  // namespace amp
