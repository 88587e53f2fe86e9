// Per-phase LDS bank-conflict attribution for the persistent VAMP engine's default cfg4 kernel
// (vamp_persist<8, 16, 4, 2, X3, 1, H2>: N = k = 256, M = 32, 16 trials per workgroup, 4 waves,
// 16-QAM, fp16x2 GEMMs).  Each phase kernel repeats exactly the LDS accesses of one phase of the
// engine's iteration (the same device functions, the same LDS carve), so rocprofv3's per-dispatch
// SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS attribute the engine's total to phases:
//   1 r~ build   (amp_vamp_persist_kernel.h: sX / sR float4 reads, h2_store8, row maxima)
//   2 GEMM A reads (gemm_h2's ds_read_b128 of the four planes; the weights stream from L2)
//   3 w store    (GEMM1 epilogue: row maxima, h2_store_acc)
//   4 GEMM2 epilogue (sX / sR element reads, sR writes)
//   5 denoiser   (denoise_sections_u<true, 16, 2> through PDenoisePolicy)
// Every phase kernel runs at reps = 1 and reps = 11; the counter difference / 10 is one
// phase-iteration of 256 workgroups.  LDXP is the A-plane row pad (16-bit elements): 0 is the
// engine's XOR-permuted layout (amp_persist.h pl_col), 8 the 16-byte row pad of rounds 1-2 (with
// ldx = N + 8, pl_mask is 0: the helpers then address the old unpermuted layout).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I amp-sparc-spatialmodulation_amd/csrc \
//       -o tools/ubench/bin/lds_phase tools/ubench/lds_phase_ubench.hip
//   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d gpurun_out/lds -o lds --output-format csv \
//       -- tools/ubench/bin/lds_phase
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "amp_host.h"
#include "amp_persist.h"
#include "amp_vamp_persist_kernel.h"

using namespace amp;

constexpr int N = 256, KN = 256, L = 8, M = 32, NT = 8, NWV = 4, PWG = 256, NWG = 256;
constexpr int NC = NT / 2, G3 = NT * NWV / 4;

template <int PH, int LDXP>
__global__ __launch_bounds__(256, 1) void kphase(const float* init, const void* wq, Const c, float* out, int reps) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float s_hmax[4][PBM];
    __shared__ int s_hexp[PBM];
    const PLayout Y = playout(N, KN, L, true);
    float* sA = lds + Y.offA;
    float* sR = lds + Y.offR;
    float* sX = lds + Y.offX;
    float* vnew = lds + Y.offV0;
    float* vprev = lds + Y.offV1;
    unsigned short* sP = reinterpret_cast<unsigned short*>(sA);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ldr = Y.ldr, ldx = N + LDXP, twoN = 2 * N;
    const int cc0 = wave * NC;
    const float* src = init + (size_t)blockIdx.x * 2 * PBM * twoN;
    for (int e = tid; e < PBM * twoN; e += PWG) {
        sR[(e / twoN) * ldr + e % twoN] = src[e];
        sX[(e / twoN) * ldr + e % twoN] = src[PBM * twoN + e];
    }
    for (int e = tid; e < PBM * N; e += PWG) { vnew[e] = 1.f; vprev[e] = 1.f; }
    for (int e = tid; e < 4 * 16 * (N + 8) / 2; e += PWG) sA[e] = 0.f;
    if (tid < PBM) s_hexp[tid] = 3;
    __syncthreads();
    float sink = 0.f;
    const float dx = 0.25f, ns = 1.0f;
    for (int rep = 0; rep < reps; ++rep) {
        if constexpr (PH == 1) {
            constexpr int IPT = (NT + 3) / 4;
            const int row = tid % PBM;
            float re[IPT][8], im[IPT][8];
            float m = 0.f;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tid + i * PWG;
                const int j0 = 8 * (e / PBM);
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const float4 x = *reinterpret_cast<const float4*>(sX + row * ldr + 2 * j0 + 4 * h);
                    const float4 q = *reinterpret_cast<const float4*>(sR + row * ldr + 2 * j0 + 4 * h);
                    re[i][2 * h] = (x.x - dx * q.x) * ns;
                    im[i][2 * h] = (x.y - dx * q.y) * ns;
                    re[i][2 * h + 1] = (x.z - dx * q.z) * ns;
                    im[i][2 * h + 1] = (x.w - dx * q.w) * ns;
                }
#pragma unroll
                for (int h = 0; h < 8; ++h) m = fmaxf(m, fmaxf(fabsf(re[i][h]), fabsf(im[i][h])));
            }
            m = fmaxf(m, __shfl_xor(m, 16));
            m = fmaxf(m, __shfl_xor(m, 32));
            if (lane < PBM) s_hmax[wave][lane] = m;
            __syncthreads();
            float mr = s_hmax[0][row];
#pragma unroll
            for (int w = 1; w < 4; ++w) mr = fmaxf(mr, s_hmax[w][row]);
            const int ex = h2_row_exp(mr);
            if (tid < PBM) s_hexp[tid] = ex;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tid + i * PWG;
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    re[i][h] = __builtin_amdgcn_ldexpf(re[i][h], ex);
                    im[i][h] = __builtin_amdgcn_ldexpf(im[i][h], ex);
                }
                h2_store8(sP, ldx, row, 8 * (e / PBM), re[i], im[i]);
            }
        } else if constexpr (PH == 2) {
            f32x4 cr[NC], ci[NC];
            gemm_h2<NC, G3>(sP, ldx, wq, cc0, cr, ci);
#pragma unroll
            for (int t = 0; t < NC; ++t) sink += cr[t][0] + ci[t][3];
        } else if constexpr (PH == 3) {
            f32x4 cr[NC], ci[NC];
#pragma unroll
            for (int t = 0; t < NC; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    cr[t][r] = sR[(4 * (lane >> 4) + r) * ldr + 2 * (16 * (cc0 + t) + (lane & 15))] * (float)(rep + 1);
                    ci[t][r] = cr[t][r] * 0.5f;
                }
            float mrow[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < NC; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) mrow[r] = fmaxf(mrow[r], fmaxf(fabsf(cr[t][r]), fabsf(ci[t][r])));
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int sh = 1; sh < 16; sh <<= 1) mrow[r] = fmaxf(mrow[r], __shfl_xor(mrow[r], sh));
            if ((lane & 15) == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) s_hmax[wave][4 * (lane >> 4) + r] = mrow[r];
            }
            __syncthreads();
            int hew[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float mr = s_hmax[0][4 * (lane >> 4) + r];
#pragma unroll
                for (int w = 1; w < 4; ++w) mr = fmaxf(mr, s_hmax[w][4 * (lane >> 4) + r]);
                hew[r] = h2_row_exp(mr);
            }
#pragma unroll
            for (int t2 = 0; t2 < NC; ++t2) {
                const int o = 16 * (cc0 + t2) + (lane & 15);
                float wr[4], wi[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    wr[r] = __builtin_amdgcn_ldexpf(cr[t2][r], hew[r]);
                    wi[r] = __builtin_amdgcn_ldexpf(ci[t2][r], hew[r]);
                }
                h2_store_acc(sP, ldx, o, wr, wi);
            }
        } else if constexpr (PH == 4) {
#pragma unroll
            for (int t2 = 0; t2 < NC; ++t2) {
                const int o = 16 * (cc0 + t2) + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int b = (4 * (lane >> 4) + r) * ldr + 2 * o;
                    const float rtr = (sX[b] - dx * sR[b]) * ns;
                    const float rti = (sX[b + 1] - dx * sR[b + 1]) * ns;
                    const float xtr = (float)rep + rtr, xti = 0.5f + rti;
                    sR[b] = (xtr - 0.1f * rtr) * 1.1f;
                    sR[b + 1] = (xti - 0.1f * rti) * 1.1f;
                }
            }
        } else if constexpr (PH == 5) {
            PDenoisePolicy pol{sR, sX, vnew, vprev, lds + Y.offSM, lds + Y.offSA, ldr, M, 3, N, 4.0f};
            PartAcc pa;
            denoise_sections_u<true, 16, 2, true>(pol, PBM * (N / M), M, c, pa);
            sink += (float)pa.sumvar;
        }
        __syncthreads();
    }
    out[(size_t)blockIdx.x * PWG + tid] = sink + sR[tid] + sX[tid] + lds[tid];
}

template <int PH, int LDXP>
static void launch(const float* init, const void* wq, const Const& c, float* out, int reps, size_t lbytes) {
    hipFuncSetAttribute((const void*)kphase<PH, LDXP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lbytes);
    hipLaunchKernelGGL((kphase<PH, LDXP>), dim3(NWG), dim3(PWG), lbytes, 0, init, wq, c, out, reps);
}

template <int PH, int LDXP>
static void pair(const float* init, const void* wq, const Const& c, float* out, size_t lbytes) {
    launch<PH, LDXP>(init, wq, c, out, 1, lbytes);
    launch<PH, LDXP>(init, wq, c, out, 11, lbytes);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "phase %d failed\n", PH); exit(1); }
    printf("phase %d ldx pad %d done\n", PH, LDXP);
}

int main() {
    const PLayout Y = playout(N, KN, L, true);
    const size_t lbytes = (size_t)Y.total * 4;
    std::vector<float> h((size_t)NWG * 2 * PBM * 2 * N);
    srand(3);
    for (auto& v : h) v = ((float)rand() / RAND_MAX * 2.f - 1.f) * 1.5f;
    // the reference's 16-QAM table (config.py:112), unit power
    amp_constellation cc{};
    const float pts[16][2] = {{-3, -3}, {-3, -1}, {-3, 1}, {-3, 3}, {-1, -3}, {-1, -1}, {-1, 1}, {-1, 3},
                              {1, -1}, {1, 1}, {1, 3}, {3, -3}, {3, -1}, {3, 1}, {3, 3}, {-1, 3}};
    cc.K = 16;
    for (int k = 0; k < 16; ++k) { cc.re[k] = pts[k][0] / sqrtf(10.f); cc.im[k] = pts[k][1] / sqrtf(10.f); }
    const Const c = to_const(&cc);
    printf("constellation grid %d pattern %d; LDS %zu B\n", c.grid, c.gfull, lbytes);
    float *dI, *dO;
    void* dW;
    hipMalloc(&dI, h.size() * 4);
    hipMalloc(&dO, (size_t)NWG * PWG * 4);
    hipMalloc(&dW, (size_t)(N / 16) * G3 * 4 * 1024 + 4096);
    hipMemset(dW, 0, (size_t)(N / 16) * G3 * 4 * 1024 + 4096);
    hipMemcpy(dI, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    pair<1, 0>(dI, dW, c, dO, lbytes);
    pair<2, 0>(dI, dW, c, dO, lbytes);
    pair<3, 0>(dI, dW, c, dO, lbytes);
    pair<4, 0>(dI, dW, c, dO, lbytes);
    pair<5, 0>(dI, dW, c, dO, lbytes);
    pair<1, 8>(dI, dW, c, dO, lbytes);
    pair<2, 8>(dI, dW, c, dO, lbytes);
    pair<3, 8>(dI, dW, c, dO, lbytes);
    hipFree(dI); hipFree(dO); hipFree(dW);
    return 0;
}
