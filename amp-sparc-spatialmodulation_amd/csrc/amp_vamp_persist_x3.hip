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
        const char* e = diag_env("AMP_VAMP_X3_WAVES");
        return !(e && atoi(e) == 4);
    }();
    return v;
}

int persist_dispatch_x3(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.N) {
    case 64:   // the two-per-CU build for every N = 64 launch, so that one epoch and side-by-side
               // epochs run the same arithmetic (bit-identical results, tests/test_gpu_epochs.py)
        return persist_wg2() ? persist_launch_nt<2, 4, true, 2>(P, dc, st) : AMP_DIAG_ONLY(persist_launch_nt<2, 4, true>(P, dc, st));
    case 128: return persist_launch_nt<4, 4, true>(P, dc, st);
    case 256:
        return x3_waves8() ? persist_launch_nt<4, 8, true>(P, dc, st) : AMP_DIAG_ONLY(persist_launch_nt<8, 4, true>(P, dc, st));
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
            // unconditional load at a clamped row (a lane-divergent branch around it serialises the
            // loads' latencies, amp_gemm.h ALoadPlain); rows past `rows` are never stored
            const float4 v = *reinterpret_cast<const float4*>(y + (size_t)min(row0 + row, rows - 1) * 2 * n + 2 * j0 + 4 * h);
            re[2 * h] = v.x; im[2 * h] = v.y; re[2 * h + 1] = v.z; im[2 * h + 1] = v.w;
        }
        x3_store8(sP, ldx, row, j0, re, im);
    }
    __syncthreads();
    f32x4 cr[NC], ci[NC];
    const void* wop = (const char*)wq + (long long)(row0 / rows_per_op) * wq_stride;
    gemm_x3<NC, G, 1, false, true>(sP, ldx, wop, wave * NC, cr, ci);   // HL: the engines' accumulation
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

// The k = 256 form (cfg4: n = 512): a workgroup takes 32 trials (two 16-row A tiles) and half the
// outputs (eight 16-column tiles, one per wave), so each operator group a wave streams feeds 48
// MFMAs of two row tiles — half the operator bytes per CU of the 16-trial form (1.5 MB, the per-CU
// L2 rate was its wall).  The 32 rows' planes of all n = 512 columns would take 196 KB of LDS, so
// the reduction runs in NH stages of KS columns (96 KB of planes each), in order: every output
// sums the same products in the same order as gemm_x3 (bit-identical y~).
// D: operator groups in flight (the kernel has registers to spare: 94 VGPRs at D = 1).  hook():
// called once after the first group's MFMAs (the next stage's y loads go there, behind this
// stage's first operator loads in the in-order vmcnt).
// lr / li: the cross-piece sums, apart from the leading-piece sums cr / ci (gemm_x3's HL form; the
// caller adds them once after the last stage).
template <int GH, int D, class Hook>
__device__ __forceinline__ void x3_rows2(const unsigned short* sP0, const unsigned short* sP1, int ldx,
                                         __amdgpu_buffer_rsrc_t wr, int gbase, f32x4 (&cr)[2], f32x4 (&ci)[2],
                                         f32x4 (&lr)[2], f32x4 (&li)[2], Hook&& hook) {
    const int lane = threadIdx.x & 63;
    const int vo = lane * 16;
    u32x4 ring[D][6];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int f = 0; f < 6; ++f) ring[d][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((gbase + d) * 6 + f) * 1024, 0);
    const int ln = pl_opaque(lane);
    const int sw = (ln & 15) & pl_mask(ldx);
    const int aoff = (ln & 15) * ldx + 8 * ((ln >> 4) ^ (sw & 3));
    const int s32 = 32 * (sw >> 2);
    const u32x4 sgn = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
    // A fragments one row tile ahead (read from LDS while the previous tile's MFMAs run)
    auto lda = [&](int g, int rt, u32x4 (&a)[6]) {
        const unsigned short* ap = (rt ? sP1 : sP0) + aoff + ((32 * g) ^ s32);
#pragma unroll
        for (int f = 0; f < 6; ++f) a[f] = *reinterpret_cast<const u32x4*>(ap + f * 16 * ldx);
    };
    u32x4 acur[6];
    lda(0, 0, acur);
#pragma unroll
    for (int g = 0; g < GH; ++g) {
        const u32x4* w = ring[g % D];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            u32x4 a[6], anx[6], na[3];
#pragma unroll
            for (int f = 0; f < 6; ++f) a[f] = acur[f];
            if (rt == 0) lda(g, 1, anx);
            else if (g + 1 < GH) lda(g + 1, 0, anx);
#pragma unroll
            for (int f = 0; f < 3; ++f) na[f] = a[3 + f] ^ sgn;
            f32x4 gr = cr[rt], gi = ci[rt], sr = lr[rt], si = li[rt];
#define AMP_MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(x), as_bf16x8(y), acc, 0, 0, 0)
            // gemm_x3's product order (smallest terms first), HL form
            AMP_MF(sr, a[0], w[2]);  AMP_MF(si, a[0], w[5]);
            AMP_MF(sr, a[1], w[1]);  AMP_MF(si, a[1], w[4]);
            AMP_MF(sr, a[2], w[0]);  AMP_MF(si, a[2], w[3]);
            AMP_MF(sr, na[0], w[5]); AMP_MF(si, a[3], w[2]);
            AMP_MF(sr, na[1], w[4]); AMP_MF(si, a[4], w[1]);
            AMP_MF(sr, na[2], w[3]); AMP_MF(si, a[5], w[0]);
            AMP_MF(sr, a[0], w[1]);  AMP_MF(si, a[0], w[4]);
            AMP_MF(sr, a[1], w[0]);  AMP_MF(si, a[1], w[3]);
            AMP_MF(sr, na[0], w[4]); AMP_MF(si, a[3], w[1]);
            AMP_MF(sr, na[1], w[3]); AMP_MF(si, a[4], w[0]);
            AMP_MF(gr, a[0], w[0]);  AMP_MF(gi, a[0], w[3]);
            AMP_MF(gr, na[0], w[3]); AMP_MF(gi, a[3], w[0]);
#undef AMP_MF
            cr[rt] = gr; ci[rt] = gi; lr[rt] = sr; li[rt] = si;
            if (rt == 0 || g + 1 < GH) {
#pragma unroll
                for (int f = 0; f < 6; ++f) acur[f] = anx[f];
            }
        }
        if (g + D < GH) {
#pragma unroll
            for (int f = 0; f < 6; ++f)
                ring[g % D][f] = __builtin_amdgcn_raw_buffer_load_b128(wr, vo, ((gbase + g + D) * 6 + f) * 1024, 0);
        }
        if (g == 0) hook();
        __builtin_amdgcn_sched_barrier(0);
    }
}

#ifndef AMP_YTIL_RING
#define AMP_YTIL_RING 3
#endif
template <int GH, int NH>
__global__ __launch_bounds__(512, 1) void ytil_x3_r2_kernel(const float* __restrict__ y, int rows, const void* wq,
                                                             float* __restrict__ ytil, int k, int rows_per_op,
                                                             long long wq_stride) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned short* sP0 = reinterpret_cast<unsigned short*>(lds);
    constexpr int KS = 32 * GH, n = KS * NH, G = GH * NH;
    const int ldx = pl_ldx(KS);
    unsigned short* sP1 = sP0 + 6 * 16 * ldx;
    const int row0 = blockIdx.x * 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ct = blockIdx.y * 8 + wave;   // this wave's 16-column output tile
    const int ctu = __builtin_amdgcn_readfirstlane(ct);
    const char* wop = (const char*)wq + (long long)(row0 / rows_per_op) * wq_stride;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(wop) + (size_t)ctu * G * 6 * 1024, (short)0, 0x7ffffff0, 0x00020000);
    f32x4 cr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 ci[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 lr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 li[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    // stage h's KS columns of the 32 rows: 8 complex values per item, rows fastest; the next
    // stage's loads are in flight while this stage's GEMM runs
    constexpr int ITEMS = 32 * (KS >> 3), PER = ITEMS / 512;
    float4 v[PER][4];
    auto load_stage = [&](int h) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = tid + i * 512, row = e % 32, j0 = 8 * (e / 32);
#pragma unroll
            for (int q = 0; q < 4; ++q)   // clamped row, no branch (see ytil_x3_kernel); rows past `rows` are never stored
                v[i][q] = *reinterpret_cast<const float4*>(y + (size_t)min(row0 + row, rows - 1) * 2 * n + 2 * (h * KS + j0) + 4 * q);
        }
    };
    load_stage(0);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        if (h > 0) __syncthreads();   // every wave is done with the previous stage's planes
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = tid + i * 512, row = e % 32, j0 = 8 * (e / 32);
            float re[8], im[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                re[2 * q] = v[i][q].x; im[2 * q] = v[i][q].y; re[2 * q + 1] = v[i][q].z; im[2 * q + 1] = v[i][q].w;
            }
            x3_store8(row < 16 ? sP0 : sP1, ldx, row & 15, j0, re, im);
        }
        __syncthreads();
        x3_rows2<GH, AMP_YTIL_RING>(sP0, sP1, ldx, wr, h * GH, cr, ci, lr, li, [&] {
            if (h + 1 < NH) load_stage(h + 1);
        });
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) { cr[rt] += lr[rt]; ci[rt] += li[rt]; }
    const int o = 16 * ct + (lane & 15);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = row0 + 16 * rt + 4 * (lane >> 4) + r;
            if (row < rows) *reinterpret_cast<float2*>(ytil + (size_t)row * 2 * k + 2 * o) = make_float2(cr[rt][r], ci[rt][r]);
        }
}

static int ytil_x3_r2_launch(const float* y, int rows, const void* wq, float* ytil, int k, int rows_per_op,
                             long long wq_stride, hipStream_t st) {
    const void* fn = (const void*)ytil_x3_r2_kernel<8, 2>;
    const size_t lds = (size_t)2 * 6 * 16 * pl_ldx(256) * 2;
    static int attr = -1;
    if (attr < 0) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("ytil_x3_r2: hipFuncSetAttribute: %s", hipGetErrorString(e));
            return AMP_E_LAUNCH;
        }
        attr = 1;
    }
    hipLaunchKernelGGL((ytil_x3_r2_kernel<8, 2>), dim3(cdiv(rows, 32), 2), dim3(512), lds, st, y, rows, wq, ytil, k,
                       rows_per_op, wq_stride);
    AMP_LAUNCH_CHECK("ytil_x3_r2");
    return AMP_OK;
}

// AMP_YTIL_R2=0 keeps the 16-trial form at k = 256 (A/B runs; read per launch, so a test can
// compare both forms in one process)
static bool ytil_r2_env() {
    const char* e = getenv("AMP_YTIL_R2");
    return !(e && e[0] == '0');
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
    case 256:   // 32 trials x half the outputs per workgroup (every operator group feeds two row
                // tiles); else eight waves of 16 trials, as in the engine
        if (ytil_r2_env() && (rows_per_op % 32 == 0 || rows_per_op >= rows))
            return ytil_x3_r2_launch(y, rows, wq, ytil, k, rows_per_op, wq_stride, st);
        return ytil_x3_launch_t<2, 16, 8>(y, rows, wq, ytil, k, rows_per_op, wq_stride, st);
    default: break;
    }
    set_error("ytil_x3: n = %d / k = %d not supported", n, k);
    return AMP_E_ARG;
}

}  // namespace amp
