// amp_vamp_persist_kernel.h — the persistent VAMP engine kernel (vamp_persist) and its launch
// templates, shared by the f32-MFMA instantiations (amp_vamp_persist.hip) and the split-precision
// bf16x3 ones (amp_vamp_persist_x3.hip), which compile as separate translation units.
// Design notes: amp_vamp_persist.hip.
#pragma once

#include <stdlib.h>

#include <type_traits>

#include "amp_decide_fused.h"
#include "amp_persist.h"
#include "amp_vamp.h"

namespace amp {

constexpr int AMP_TRACE_STRIDE = 10;   // diagnostic stamps per (workgroup, iteration)
#ifndef AMP_OCC2_PK
#define AMP_OCC2_PK 0                   // 1: the packed denoiser also at two waves per SIMD (diagnostic builds)
#endif
#ifndef AMP_KK4_DU
#define AMP_KK4_DU 4                    // QPSK sections in flight per lane group (diagnostic builds vary it)
#endif
#ifndef AMP_X3_W8_PIN
#define AMP_X3_W8_PIN 0
#endif
#ifndef AMP_X3_W8_RING
#define AMP_X3_W8_RING 1                // eight-wave bf16x3 GEMM ring depth (A/B builds try 2 with AMP_X3_W8_PIN)
#endif
#ifndef AMP_X3_W8_PKGRID
#define AMP_X3_W8_PKGRID 1              // the eight-wave bf16x3 form keeps 16-QAM's packed grid denoiser
#endif
#ifndef AMP_X3_DU
#define AMP_X3_DU 2                     // 16-QAM sections in flight per lane group (bf16x3 engine; 4 measured: no gain)
#endif

// LDS carve (floats).  Row strides 2N+4 / max(2N,2k)+4 keep the f32 engine's 16-row ds_read_b128
// and accumulator stores conflict-free (row r and r+4 land 16 banks apart); the split-precision
// engines read r / x~ as complex pairs (ds_read_b64 of rows 4 apart) and take 2N+8 (rows r and r+4
// 32 banks apart: the two 16-lane halves of a 32-lane group on disjoint banks).
struct PLayout {
    int lda, ldr;
    int offA, offR, offX, offV0, offV1, offSM, offSA, offScr, total;
};

// split-precision A planes (X3 engine): six (bf16x3) or four (fp16x2) planes of 16 rows x N 16-bit
// pieces in the XOR-permuted layout of amp_persist.h (pl_col)
__host__ __device__ inline int x3_ldx(int N) { return pl_ldx(N); }
__host__ __device__ inline int x3_plane_floats(int N) { return 6 * 16 * x3_ldx(N) / 2; }

__host__ __device__ inline PLayout playout(int N, int k, int L, bool x3 = false) {
    PLayout y;
    y.lda = (2 * N > 2 * k ? 2 * N : 2 * k) + 4;
    y.ldr = 2 * N + (x3 ? 8 : 4);
    int o = 0;
    y.offA = o; o += (x3 && x3_plane_floats(N) > PBM * y.lda) ? x3_plane_floats(N) : PBM * y.lda;
    y.offR = o; o += PBM * y.ldr;
    y.offX = o; o += PBM * y.ldr;
    y.offV0 = o; o += PBM * N;
    y.offV1 = o; o += PBM * N;
    y.offSM = o; o += PBM * L;
    y.offSA = o; o += PBM * L;
    o = (o + 3) & ~3;
    y.offScr = o; o += 1024;
    y.total = o;
    return y;
}

// dc: the decision table; its Const64 base is also the exact rare path's float64 constellation.
// X3: both per-iteration GEMMs on the split-precision bf16x3 engine (gemm_x3): the A operand
// (r~, then w) lives in LDS as six bf16 planes, each wave owns NT/2 complex column tiles (the
// same 16 NT real columns as the f32 form), the operators are the X3-packed Vh / V (Wx1 / Wx2).
// OCC: workgroups per CU the register allocation is bounded for (__launch_bounds__' minimum
// waves per SIMD = OCC * NWV / 4); 2 only for the side-by-side cfg2 epochs (N = 64).
// H2 (with X3): the split-precision GEMMs in the fp16x2 form (gemm_h2: four A planes, the operators
// h2-packed); every A row (r~, then w) is scaled by its own power of two (h2_row_exp) before the
// split and the accumulators are scaled back by 2^-(e_row + H2_EX).
// I8 (with X3): the split-precision GEMMs in the int8x4 form (gemm_i8: eight int8 digit planes of
// the A operand, each row with its own exponent; the operators i8-packed with per-column
// exponents); the results come out of the GEMM fully scaled.
// The kernel arguments (VampK at kernarg offset 0, DecConst behind it: 2.6 KB) are read through the
// kernarg segment pointer, laundered at the top of every iteration and before the denoiser, GEMM2
// and the exchange (amp_persist.h karg_launder): the compiler then reloads a field (s_load, scalar
// cache) where a phase uses it instead of hoisting every field the loop reads into an SGPR for the
// whole launch, which spilled ~390 SGPRs into VGPR lanes (v_readlane in every phase) and ~75 VGPRs
// to scratch in the eight-wave cfg4 build.
constexpr int KARG_DC_OFF = karg_second_offset<VampK, DecConst>();

template <int NT, int KK, int NWV, int DU, bool X3, int OCC = 1, bool H2 = false, bool I8 = false>
__global__ __launch_bounds__(64 * NWV, OCC * NWV / 4) void vamp_persist(VampK P_arg, DecConst dc_arg) {
    (void)P_arg;
    (void)dc_arg;
    unsigned long long kbase = karg_base();
    const VampK* Pp = karg_at<VampK>(kbase, 0);
    const DecConst* Dp = karg_at<DecConst>(kbase, KARG_DC_OFF);
#define P (*Pp)
#define dc (*Dp)
    static_assert(!X3 || ((NWV == 4 || (NWV == 8 && !H2 && OCC == 1)) && NT % 2 == 0),
                  "X3: four waves (eight for the bf16x3 two-waves-per-SIMD form), whole complex tiles");
    static_assert(!(H2 && I8) && (!I8 || X3), "I8: a split-precision form of its own");
    // packed denoiser at one wave per SIMD; with two (OCC = 2, or the eight-wave bf16x3 form) at most
    // the packed product-grid form, for 16-QAM (AMP_X3_W8_PKGRID; 16PSK, not a grid, runs the scalar
    // per-point form: the packed per-point form lost results there)
    constexpr int PKDEN = ((OCC * NWV / 4 == 1) || AMP_OCC2_PK) ? PK_ALL
                          : (NWV == 8 && KK == 16 && AMP_X3_W8_PKGRID) ? PK_GRID : PK_NONE;
    constexpr int PWG = 64 * NWV;
    constexpr int NC = X3 ? NT / 2 : 1;        // complex column tiles per wave (X3)
    constexpr int G3 = NT * NWV / 4;           // 32-wide complex reduction groups: N / 32
    constexpr int X3R = (NWV == 8) ? AMP_X3_W8_RING : 1;   // weight groups in flight (gemm_x3)
    // eight waves: no A-fragment prefetch in gemm_x3 (the partner wave covers the LDS reads;
    // 24 registers fewer) when AMP_X3_W8_PIN (A/B builds)
    constexpr bool X3PIN = NWV == 8 && AMP_X3_W8_PIN;
#define c64 (static_cast<const Const64&>(*Dp))
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_flag;
    __shared__ double s_d[PWG / 64][4];
    __shared__ float s_hmax[PWG / 64][PBM];   // H2: per-wave row maxima of the A operand
    __shared__ int s_hexp[PBM];               // H2: r~ row exponents (for GEMM1's epilogue)
    const PLayout Y = playout(P.N, P.k, P.L, X3);
    float* sA = lds + Y.offA;
    float* sR = lds + Y.offR;
    float* sX = lds + Y.offX;
    float* sM = lds + Y.offSM;
    float* sS = lds + Y.offSA;
    float* scr = lds + Y.offScr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wg = blockIdx.x, nwg = gridDim.x;
    // the exchange: workgroup wgx of nwx (a trial-sharded batch, amp_vamp_detect_count_shard: every
    // rank's grid publishes into one shared granule array at its global workgroup index, so the
    // batch scalars are reduced in the whole batch's order; else wgx = wg, nwx = nwg)
    const int wgx = wg + P.wg_off, nwx = P.nwg_x;
    // side-by-side epochs: workgroups [ep * wpe, (ep + 1) * wpe) hold epoch ep's B trials and
    // exchange its batch scalars among themselves only
    const int ep = wgx / P.wpe, wl = wgx - ep * P.wpe, wg0 = ep * P.wpe;
    const int lrow0 = wl * PBM;                       // first trial within the epoch (the batch's index)
    // its row in this launch's arrays (a shard holds rows [row_off, row_off + its B) of the batch)
    const int row0 = ep * P.B + lrow0 - P.row_off, nrows = min(PBM, P.B - lrow0);
#define ebar (P.pbar + (P.E > 1 ? PBAR_EPOCH + ep : 0))   // this epoch's arrival counter
    const int N = P.N, twoN = 2 * N, twok = 2 * P.k, M = P.M, spr = N / M;
    // this epoch's channel (one per epoch, or one shared: wch = sch = 0)
    const float* const sv_ep = P.s + (size_t)ep * P.sch;
    // (formed where used, from the laundered arguments: not live across the loop)
#define Wx1 ((const void*)((const char*)P.Wx1 + ep * P.wch))
#define Wx2 ((const void*)((const char*)P.Wx2 + ep * P.wch))
    const int ldr = Y.ldr, lda = Y.lda;
    const int ct0 = wave * NT;                 // this wave's 16-column tiles (both GEMMs: 2k == 2N)
    const int cc0 = wave * NC;                 // X3: this wave's complex 16-column tiles
    unsigned short* sP = reinterpret_cast<unsigned short*>(sA);
    const int ldx = x3_ldx(N);
    signed char* sB = reinterpret_cast<signed char*>(sA);   // I8: the digit planes
    const int ldb = i8_ldb(N);

    // y~ rows and s^2 of this wave's GEMM1 columns, in the accumulator layout
    // (X3: yt[2t] / yt[2t+1] = Re / Im of complex tile t, s2c[t] its s^2)
    float yt[NT][4], s2c[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = X3 ? 2 * (16 * (cc0 + (t < NC ? t : 0)) + (lane & 15)) : 16 * (ct0 + t) + (lane & 15);
        const float sv = sv_ep[col >> 1];
        s2c[t] = sv * sv;                                   // vamp.py:17
    }
    if (H2 && P.ytil_in_kernel) {
      if constexpr (H2) {
        // y~ = (s Uh) y (vamp.py:22) for this workgroup's rows on the fp16x2 GEMM (n == 2N): the y
        // rows scaled per row and split into four planes over the A / R / X region (free until
        // the Tracker's state is formed below), the operator s Uh h2-packed with exponent YH2_EX
        constexpr int IPY = NT / 2;                   // items per thread: PBM n / 8 / PWG, n = 64 NT
        const int n = P.n, ldy = pl_ldx(n);
        const int row = tid % PBM;
        float re[IPY][8], im[IPY][8];
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < IPY; ++i) {
            const int e = tid + i * PWG;
            const int j0 = 8 * (e / PBM);
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                // unconditional load at a clamped row, zeroed after it (a lane-divergent branch around
                // the load serialises the loads' latencies: amp_gemm.h ALoadPlain)
                float4 v = *reinterpret_cast<const float4*>(P.y + (size_t)(row0 + max(min(row, nrows - 1), 0)) * 2 * n + 2 * j0 + 4 * h);
                if (!(row < nrows)) v = make_float4(0.f, 0.f, 0.f, 0.f);
                re[i][2 * h] = v.x; im[i][2 * h] = v.y; re[i][2 * h + 1] = v.z; im[i][2 * h + 1] = v.w;
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
        for (int w = 1; w < PWG / 64; ++w) mr = fmaxf(mr, s_hmax[w][row]);
        const int ex = h2_row_exp(mr);
        if (tid < PBM) s_hexp[tid] = ex;
#pragma unroll
        for (int i = 0; i < IPY; ++i) {
            const int e = tid + i * PWG;
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                re[i][h] = __builtin_amdgcn_ldexpf(re[i][h], ex);
                im[i][h] = __builtin_amdgcn_ldexpf(im[i][h], ex);
            }
            h2_store8(sP, ldy, row, 8 * (e / PBM), re[i], im[i]);
        }
        __syncthreads();
        f32x4 yr[NC], yi[NC];
        gemm_h2<NC, 2 * G3>(sP, ldy, P.Wq0, cc0, yr, yi);   // K = n = 2N: 2 G3 groups of 32
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float sc = __builtin_amdgcn_ldexpf(1.0f, -(s_hexp[4 * (lane >> 4) + r] + YH2_EX));
#pragma unroll
            for (int t = 0; t < NC; ++t) {
                yt[2 * t][r] = yr[t][r] * sc;
                yt[2 * t + 1][r] = yi[t][r] * sc;
            }
        }
        __syncthreads();   // the planes region becomes the Tracker's state
      }
    } else if (X3) {
      if constexpr (!I8) {   // (I8 reads y~ back every iteration)
#pragma unroll
        for (int t = 0; t < NC; ++t) {
            const int o = 16 * (cc0 + t) + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r;
                const bool in = row < nrows;
                // unconditional loads at a clamped row, zeroed after them (see the y load above)
                const size_t yo = (size_t)(row0 + max(min(row, nrows - 1), 0)) * twok + 2 * o;
                const float a = P.ytil[yo], b = P.ytil[yo + 1];
                yt[2 * t][r] = in ? a : 0.f;
                yt[2 * t + 1][r] = in ? b : 0.f;
            }
        }
      }
    } else if (P.ytil_in_kernel) {
        // y~ = (s Uh) y (vamp.py:22) for this workgroup's rows: y staged in LDS over the A/R/X
        // region (row stride 2n + 4 = 4N + 4), GEMM on the packed s Uh operand (K = 2n = 4N)
        const int ldy = 4 * N + 4;
        for (int e = tid; e < PBM * N; e += PWG) {          // float4 units: 4N floats per row
            const int row = e / N, c4 = 4 * (e - row * N);
            float4 v = *reinterpret_cast<const float4*>(P.y + (size_t)(row0 + max(min(row, nrows - 1), 0)) * 4 * N + c4);
            if (!(row < nrows)) v = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(lds + row * ldy + c4) = v;
        }
        __syncthreads();
        f32x4 acc[NT];
        gemm16<NT, 2 * NT * NWV>(lds, ldy, P.Wq0, ct0, acc);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) yt[t][r] = acc[t][r];
        __syncthreads();
    } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int col = 16 * (ct0 + t) + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r;
                const float yv = P.ytil[(size_t)(row0 + max(min(row, nrows - 1), 0)) * twok + col];
                yt[t][r] = (row < nrows) ? yv : 0.f;
            }
        }
    }
    VampIter cur;
    {
        const S2Lane s2l = s2_lane(P, sv_ep);     // s^2 for the first LMMSE sum (re-read per exchange below)
        cur = vamp_first_iter(P, scr, &s2l);      // vamp.py:26, 66-82 at t = 0
    }
    // Tracker (vamp.py:22-26): xmmse = p, r = 0 (so r~ = p at t = 0), var(prev) = 1
    {
        const float p = (float)P.sparsity;
        for (int e = tid; e < PBM * twoN; e += PWG) {
            const int row = e / twoN, col = e - row * twoN;
            sR[row * ldr + col] = 0.f;
            sX[row * ldr + col] = (row < nrows && (col & 1) == 0) ? p : 0.f;
        }
        for (int e = tid; e < PBM * N; e += PWG) lds[Y.offV1 + e] = 1.0f;
    }

    unsigned long long* trc = P.trace;
    auto stamp = [&](int t, int ph) {
        if (trc && tid == 0 && t < P.max_iter) trc[((size_t)wg * P.max_iter + t) * AMP_TRACE_STRIDE + ph] = __builtin_amdgcn_s_memtime();
    };
    if (trc && tid == 0) {
        trc[(size_t)nwg * P.max_iter * AMP_TRACE_STRIDE + 2 * wg] = __builtin_amdgcn_s_memtime();
        trc[(size_t)nwg * P.max_iter * AMP_TRACE_STRIDE + 2 * wg + 1] = __builtin_amdgcn_s_memrealtime();
    }
    unsigned nbar = 0;
#define grs (gran_rsrc(P.pparts, (unsigned)(P.max_iter * nwx) * 32u))
    int fixed = 0, last_t = 0, aborted = 0;
    VampIter nx = cur;
    // 5. batch scalars of iteration te (its partials published): every workgroup gathers and reduces
    // every partial, settles the rare exact-float64 sections, and forms the scalars of te + 1 (nx).
    // vnew / vprev: te's var buffers.  False: a grid exchange timed out (the grid is released).
    auto exchange = [&](int te, float* vnew, const float* vprev) -> bool {
            PartAcc g;
            // this lane's s^2 for the LMMSE sum of vamp_advance, loaded here so that the loads
            // complete during the gather's wait: through the per-phase kernel-argument pointer
            // they are not hoisted out of the loop (held across it, the values were spilled, and
            // vamp_advance waited on their scratch reload)
            const S2Lane s2x = s2_lane(P, P.s + (size_t)ep * P.sch);
            const unsigned tag = P.gen * (unsigned)(P.max_iter + 1) + (unsigned)te + 1u;
            if (!part_gather(grs, ((unsigned)te * nwx + wg0) * 32u, P.wpe, tag, P.pbar + 1, g, scr, &s_flag)) return false;
            stamp(te, 6);
            fixed = 0;
            if (part_allnan(g)) {
                // the reference's G is NaN / inf: every section of this iteration is NaN
                if (!cur.fixed_all) {
                    const float qn = __int_as_float(0x7fc00000);
                    for (int e = tid; e < nrows * twoN; e += PWG) sX[(e / twoN) * ldr + e % twoN] = qn;
                    for (int e = tid; e < nrows * N; e += PWG) vnew[e] = qn;
                }
                g.sumvar = __longlong_as_double(0x7ff8000000000000LL);
                g.notclose = 1;
                fixed = -1;
            } else if (part_danger(g)) {
                // (a) exact float64 G over the candidate sections of every workgroup
                const double G32 = g.maxabs, slack = logit_slack(G32);
                const float inv = cur.inv_sigma2;
                auto ldf = [=](int s) {
                    const int row = s / spr, sj = s - row * spr;
                    const float* rp = sR + row * ldr + 2 * sj * M;
                    return [=](int m, float& rr, float& ri, float& it) {
                        rr = rp[2 * m]; ri = rp[2 * m + 1]; it = inv;
                    };
                };
                double gm = 0.0;
                for (int s = tid; s < nrows * spr; s += PWG)
                    if ((double)sS[s] >= G32 - slack) gm = fmax(gm, section_absmax_f64(ldf(s), M, c64));
                gm = group_max(gm, 64);
                if (lane == 0) s_d[wave][0] = gm;
                __syncthreads();
                if (tid == 0) {
                    double m4 = 0.0;
                    for (int w = 0; w < PWG / 64; ++w) m4 = fmax(m4, s_d[w][0]);
                    P.pxch[((size_t)te * nwx + wgx) * 4 + 0] = m4;
                }
                if (!grid_sync_on(ebar, P.pbar + 1, ++nbar * (unsigned)P.wpe, &s_flag)) return false;
                double G = 0.0;
                for (int w = wg0; w < wg0 + P.wpe; ++w) G = fmax(G, P.pxch[((size_t)te * nwx + w) * 4 + 0]);
                // (b) exact recompute of this workgroup's sections below the danger line
                double dsum = 0.0;
                int dnc = 0, cnt = 0;
                for (int s = tid; s < nrows * spr; s += PWG) {
                    if (!((double)sM[s] - G < AMP_DANGER + slack)) continue;
                    ++cnt;
                    const int row = s / spr, sj = s - row * spr;
                    float* xp = sX + row * ldr + 2 * sj * M;
                    const int v0 = row * N + sj * M;
                    auto st = [&](int m, float xr, float xi, float var) {
                        const float old = vnew[v0 + m];
                        dsum += (double)var - (double)old;
                        dnc += (torch_close(var, vprev[v0 + m]) ? 0 : 1) - (torch_close(old, vprev[v0 + m]) ? 0 : 1);
                        xp[2 * m] = xr; xp[2 * m + 1] = xi;
                        vnew[v0 + m] = var;
                    };
                    exact_section_f64<true>(ldf(s), st, M, c64, G);
                }
                dsum = group_sum(dsum, 64);
                dnc = group_sum(dnc, 64);
                cnt = group_sum(cnt, 64);
                __syncthreads();
                if (lane == 0) { s_d[wave][1] = dsum; s_d[wave][2] = (double)dnc; s_d[wave][3] = (double)cnt; }
                __syncthreads();
                if (tid == 0) {
                    double a = 0.0, b = 0.0, c = 0.0;
                    for (int w = 0; w < PWG / 64; ++w) { a += s_d[w][1]; b += s_d[w][2]; c += s_d[w][3]; }
                    P.pxch[((size_t)te * nwx + wgx) * 4 + 1] = a;
                    P.pxch[((size_t)te * nwx + wgx) * 4 + 2] = b;
                    P.pxch[((size_t)te * nwx + wgx) * 4 + 3] = c;
                }
                if (!grid_sync_on(ebar, P.pbar + 1, ++nbar * (unsigned)P.wpe, &s_flag)) return false;
                double a = 0.0, b = 0.0, c = 0.0;
                for (int w = wg0; w < wg0 + P.wpe; ++w) {
                    const double* q = P.pxch + ((size_t)te * nwx + w) * 4;
                    a += q[1]; b += q[2]; c += q[3];
                }
                g.sumvar += a;   // (sum - old) + new, in float64
                g.notclose = (uint32_t)((long long)g.notclose + (long long)b);
                g.maxabs = G;
                fixed = (int)c;
            }
        stamp(te, 9);   // (slot 9: vamp_advance starts)
        nx = vamp_advance(P, cur, g, fixed, te, scr, &s2x);
        stamp(te, 7);
        return true;
    };

    for (int t = 0; t < P.max_iter; ++t) {
        kbase = karg_launder(kbase);
        Pp = karg_at<VampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, KARG_DC_OFF);
        last_t = t;
        stamp(t, 0);
        const float* vprev = lds + ((t & 1) ? Y.offV0 : Y.offV1);
        float* vnew = lds + ((t & 1) ? Y.offV1 : Y.offV0);
        // 1. A <- r~ (vamp.py:91; t = 0: dxdr 0, normScalar 1)
        if constexpr (H2 || I8) {
            // r~ rows in registers (item e: row e % PBM == tid % PBM, 8 complex values), the
            // row's max |value| over the workgroup, then the scaled split
            constexpr int IPT = (NT + 3) / 4;             // items per thread: PBM N / 8 / PWG
            const int tdp = I8 ? pl_opaque(tid) : tid;     // I8: addresses formed here, not hoisted
            const int row = tdp % PBM;
            float re[IPT][8], im[IPT][8];
            float m = 0.f;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tdp + i * PWG;
                const int j0 = 8 * (e / PBM);
                const bool ok = e < PBM * (N >> 3);
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    float4 x = make_float4(0.f, 0.f, 0.f, 0.f), q = x;
                    if (ok) {
                        x = *reinterpret_cast<const float4*>(sX + row * ldr + 2 * j0 + 4 * h);
                        q = *reinterpret_cast<const float4*>(sR + row * ldr + 2 * j0 + 4 * h);
                    }
                    re[i][2 * h] = (x.x - cur.dxdr_prev * q.x) * cur.ns_prev;
                    im[i][2 * h] = (x.y - cur.dxdr_prev * q.y) * cur.ns_prev;
                    re[i][2 * h + 1] = (x.z - cur.dxdr_prev * q.z) * cur.ns_prev;
                    im[i][2 * h + 1] = (x.w - cur.dxdr_prev * q.w) * cur.ns_prev;
                }
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    if constexpr (I8) m = i8_absmax(i8_absmax(m, re[i][h]), im[i][h]);
                    else m = fmaxf(m, fmaxf(fabsf(re[i][h]), fabsf(im[i][h])));
                }
            }
            m = fmaxf(m, __shfl_xor(m, 16));
            m = fmaxf(m, __shfl_xor(m, 32));
            if (lane < PBM) s_hmax[wave][lane] = m;
            __syncthreads();
            float mr = s_hmax[0][row];
#pragma unroll
            for (int w = 1; w < PWG / 64; ++w) mr = fmaxf(mr, s_hmax[w][row]);
            const int ex = I8 ? i8_row_exp(mr) : h2_row_exp(mr);
            if (tid < PBM) s_hexp[tid] = ex;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tdp + i * PWG;
                if (e < PBM * (N >> 3)) {
                    if constexpr (I8) {
                        i8_store8(sB, ldb, row, 8 * (e / PBM), re[i], im[i], ex);
                    } else {
#pragma unroll
                        for (int h = 0; h < 8; ++h) {
                            re[i][h] = __builtin_amdgcn_ldexpf(re[i][h], ex);
                            im[i][h] = __builtin_amdgcn_ldexpf(im[i][h], ex);
                        }
                        h2_store8(sP, ldx, row, 8 * (e / PBM), re[i], im[i]);
                    }
                }
            }
        } else if constexpr (X3) {
            const int tdx = NWV == 8 ? pl_opaque(tid) : tid;   // eight waves: addresses formed here
            for (int e = tdx; e < PBM * (N >> 3); e += PWG) {   // 8 complex values per item
                // consecutive items walk the 16 rows (row stride 2N + 4 floats): each group of 16
                // lanes reads 16 different bank quads (item-major rows put 4 lanes on each)
                const int row = e % PBM, j0 = 8 * (e / PBM);
                float re[8], im[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const float4 x = *reinterpret_cast<const float4*>(sX + row * ldr + 2 * j0 + 4 * h);
                    const float4 q = *reinterpret_cast<const float4*>(sR + row * ldr + 2 * j0 + 4 * h);
                    re[2 * h] = (x.x - cur.dxdr_prev * q.x) * cur.ns_prev;
                    im[2 * h] = (x.y - cur.dxdr_prev * q.y) * cur.ns_prev;
                    re[2 * h + 1] = (x.z - cur.dxdr_prev * q.z) * cur.ns_prev;
                    im[2 * h + 1] = (x.w - cur.dxdr_prev * q.w) * cur.ns_prev;
                }
                x3_store8(sP, ldx, row, j0, re, im);
            }
        } else
        for (int e = tid; e < PBM * (twoN >> 2); e += PWG) {
            const int row = e / (twoN >> 2), c4 = 4 * (e - row * (twoN >> 2));
            const float4 x = *reinterpret_cast<const float4*>(sX + row * ldr + c4);
            const float4 q = *reinterpret_cast<const float4*>(sR + row * ldr + c4);
            *reinterpret_cast<float4*>(sA + row * lda + c4) =
                make_float4((x.x - cur.dxdr_prev * q.x) * cur.ns_prev, (x.y - cur.dxdr_prev * q.y) * cur.ns_prev,
                            (x.z - cur.dxdr_prev * q.z) * cur.ns_prev, (x.w - cur.dxdr_prev * q.w) * cur.ns_prev);
        }
        __syncthreads();
        stamp(t, 1);
        // 2. q = Vh r~ ; w = scale (y~ + vr q) - q  -> A   (vamp.py:67-72)
        f32x4 acc[NT];
        f32x4 cr[NC], ci[NC];
        if constexpr (I8) {
            float rowf[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) rowf[r] = i8_row_factor(s_hexp[4 * (lane >> 4) + r]);
            gemm_i8<NC, G3 / 2>(sB, ldb, Wx1, N, cc0, rowf, cr, ci);   // 64-deep groups: N / 64
        } else if constexpr (H2)
            gemm_h2<NC, G3>(sP, ldx, Wx1, cc0, cr, ci);
        else if constexpr (X3)
            gemm_x3<NC, G3, X3R, X3PIN, true>(sP, ldx, Wx1, cc0, cr, ci);
        else
            gemm16<NT, NT * NWV>(sA, lda, P.Wq1, ct0, acc);   // G = 2N / 16 = NT * NWV
        float hsc[4];                                 // H2: 2^-(e_row + H2_EX) of this lane's rows
        int hew[4];                                   // H2 / I8: the w rows' exponents
        if constexpr (H2 || I8) {
            // w = scale (y~ + vr q) - q for every tile of this wave, its rows' max |w| to LDS; the
            // barrier below also ends every wave's reads of the r~ planes
#pragma unroll
            for (int r = 0; r < 4; ++r) hsc[r] = I8 ? 1.0f : __builtin_amdgcn_ldexpf(1.0f, -(s_hexp[4 * (lane >> 4) + r] + H2_EX));
            float mrow[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t2 = 0; t2 < NC; ++t2) {
                const float sc = 1.0f / (s2c[t2] + cur.vr);
                float ytr[4], yti[4];
                if constexpr (I8) {
                    // y~ read back each iteration (16 rows x 2N floats per workgroup, L2-resident)
                    // rather than held in 32 registers across the loop: the int8x4 GEMMs' ring and
                    // level sums need them.  The lane index is pinned so the addresses are formed here
                    const int ln = pl_opaque(lane);
                    const int oo = 16 * (cc0 + t2) + (ln & 15);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 4 * (ln >> 4) + r;
                        const float2 u = *reinterpret_cast<const float2*>(P.ytil + (size_t)(row0 + max(min(row, nrows - 1), 0)) * twok + 2 * oo);
                        const float2 v = row < nrows ? u : make_float2(0.f, 0.f);
                        ytr[r] = v.x; yti[r] = v.y;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) { ytr[r] = yt[2 * t2][r]; yti[r] = yt[2 * t2 + 1][r]; }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float qr = I8 ? cr[t2][r] : cr[t2][r] * hsc[r], qi = I8 ? ci[t2][r] : ci[t2][r] * hsc[r];
                    cr[t2][r] = sc * (ytr[r] + cur.vr * qr) - qr;
                    ci[t2][r] = sc * (yti[r] + cur.vr * qi) - qi;
                    if constexpr (I8) mrow[r] = i8_absmax(i8_absmax(mrow[r], cr[t2][r]), ci[t2][r]);
                    else mrow[r] = fmaxf(mrow[r], fmaxf(fabsf(cr[t2][r]), fabsf(ci[t2][r])));
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int sh = 1; sh < 16; sh <<= 1) mrow[r] = fmaxf(mrow[r], __shfl_xor(mrow[r], sh));
            }
            if ((lane & 15) == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) s_hmax[wave][4 * (lane >> 4) + r] = mrow[r];
            }
        }
        __syncthreads();
        stamp(t, 2);
        if constexpr (H2 || I8) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float mr = s_hmax[0][4 * (lane >> 4) + r];
#pragma unroll
                for (int w = 1; w < PWG / 64; ++w) mr = fmaxf(mr, s_hmax[w][4 * (lane >> 4) + r]);
                hew[r] = I8 ? i8_row_exp(mr) : h2_row_exp(mr);
            }
            const int lnw = I8 ? pl_opaque(lane) : lane;   // I8: addresses formed here, not hoisted
#pragma unroll
            for (int t2 = 0; t2 < NC; ++t2) {
                const int o = 16 * (cc0 + t2) + (lnw & 15);
                if constexpr (I8) {
                    int wr[4], wi[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) { wr[r] = i8_fix(cr[t2][r], hew[r]); wi[r] = i8_fix(ci[t2][r], hew[r]); }
                    i8_store_acc(sB, ldb, o, wr, wi);
                } else {
                    float wr[4], wi[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        wr[r] = __builtin_amdgcn_ldexpf(cr[t2][r], hew[r]);
                        wi[r] = __builtin_amdgcn_ldexpf(ci[t2][r], hew[r]);
                    }
                    h2_store_acc(sP, ldx, o, wr, wi);
                }
                if (P.dump) {
                    float* dp = P.dump + (((size_t)t * nwg + wg) * 5 + 0) * PBM * twoN;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o] = cr[t2][r];
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o + 1] = ci[t2][r];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) hsc[r] = I8 ? i8_row_factor(hew[r]) : __builtin_amdgcn_ldexpf(1.0f, -(hew[r] + H2_EX));
        } else if constexpr (X3) {
            const int lnx = NWV == 8 ? pl_opaque(lane) : lane;   // eight waves: addresses formed here
#pragma unroll
            for (int t2 = 0; t2 < NC; ++t2) {
                const int o = 16 * (cc0 + t2) + (lnx & 15);
                const float sc = 1.0f / (s2c[t2] + cur.vr);
                float wr[4], wi[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float qr = cr[t2][r], qi = ci[t2][r];
                    wr[r] = sc * (yt[2 * t2][r] + cur.vr * qr) - qr;
                    wi[r] = sc * (yt[2 * t2 + 1][r] + cur.vr * qi) - qi;
                }
                x3_store_acc(sP, ldx, o, wr, wi);
                if (P.dump) {
                    float* dp = P.dump + (((size_t)t * nwg + wg) * 5 + 0) * PBM * twoN;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o] = wr[r];
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o + 1] = wi[r];
                    }
                }
            }
        } else
#pragma unroll
        for (int t2 = 0; t2 < NT; ++t2) {
            const int col = 16 * (ct0 + t2) + (lane & 15);
            const float sc = 1.0f / (s2c[t2] + cur.vr);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float q = acc[t2][r];
                sA[(4 * (lane >> 4) + r) * lda + col] = sc * (yt[t2][r] + cur.vr * q) - q;
            }
        }
        __syncthreads();
        stamp(t, 3);
        kbase = karg_launder(kbase);
        Pp = karg_at<VampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, KARG_DC_OFF);
        // 3. x~ = V w + r~ ; r = (x~ - alpha r~) / (1 - alpha)   (vamp.py:72, 79)
        // r = (x~ - alpha r~) / (1 - alpha) for the complex column tiles ccs ... of this wave.  The
        // lane index pinned here: the 4 NC LDS addresses below are then formed in this epilogue
        // instead of being hoisted out of the iteration loop (and kept live across it)
        auto r_epi = [&](int ccs, auto& er, auto& ei) __attribute__((always_inline)) {
            constexpr int NCX = std::extent<std::remove_reference_t<decltype(er)>>::value;
            const int lnr = (I8 || NWV == 8) ? pl_opaque(lane) : lane;
#pragma unroll
            for (int t2 = 0; t2 < NCX; ++t2) {
                const int o = 16 * (ccs + t2) + (lnr & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int b = (4 * (lnr >> 4) + r) * ldr + 2 * o;
                    const float rtr = (sX[b] - cur.dxdr_prev * sR[b]) * cur.ns_prev;
                    const float rti = (sX[b + 1] - cur.dxdr_prev * sR[b + 1]) * cur.ns_prev;
                    const float xtr = er[t2][r] + rtr, xti = ei[t2][r] + rti;
                    sR[b] = (xtr - cur.alpha * rtr) * cur.inv1ma;
                    sR[b + 1] = (xti - cur.alpha * rti) * cur.inv1ma;
                    if (P.dump) {
                        float* dp = P.dump + (((size_t)t * nwg + wg) * 5 + 1) * PBM * twoN;
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o] = sR[b];
                        dp[(4 * (lane >> 4) + r) * twoN + 2 * o + 1] = sR[b + 1];
                    }
                }
            }
        };
        if constexpr (X3) {
            if constexpr (I8) {
                gemm_i8<NC, G3 / 2>(sB, ldb, Wx2, N, cc0, hsc, cr, ci);   // hsc: the w rows' factors
            } else if constexpr (H2) {
                gemm_h2<NC, G3>(sP, ldx, Wx2, cc0, cr, ci);
#pragma unroll
                for (int t2 = 0; t2 < NC; ++t2)
#pragma unroll
                    for (int r = 0; r < 4; ++r) { cr[t2][r] *= hsc[r]; ci[t2][r] *= hsc[r]; }
            }
            if constexpr (!I8 && !H2) gemm_x3<NC, G3, X3R, X3PIN, true>(sP, ldx, Wx2, cc0, cr, ci);
            r_epi(cc0, cr, ci);
        } else {
        gemm16<NT, NT * NWV>(sA, lda, P.Wq2, ct0, acc);
#pragma unroll
        for (int t2 = 0; t2 < NT; ++t2) {
            const int col = 16 * (ct0 + t2) + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = (4 * (lane >> 4) + r) * ldr + col;
                const float rt = (sX[o] - cur.dxdr_prev * sR[o]) * cur.ns_prev;
                const float xt = acc[t2][r] + rt;
                sR[o] = (xt - cur.alpha * rt) * cur.inv1ma;
            }
        }
        }
        __syncthreads();
        // 4. denoiser (vamp.py:84)
        PDenoisePolicy pol{sR, sX, vnew, vprev, sM, sS, ldr, M, 31 - __builtin_clz(spr), N, cur.inv_sigma2};
        if (P.dump) pol.dbg = P.dump + (((size_t)t * nwg + wg) * 5 + 4) * PBM * twoN;
        PartAcc pa;
        kbase = karg_launder(kbase);
        Pp = karg_at<VampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, KARG_DC_OFF);
        stamp(t, 4);
        if constexpr (KK > 16)
            denoise_sections_wide_m<true, KK>(pol, nrows * spr, M, P.c, pa);
        else
            denoise_sections_u<true, KK, DU, PKDEN>(pol, nrows * spr, M, P.c, pa);   // two waves per SIMD: scalar f32 (amp_denoise.h)
        stamp(t, 8);
        const unsigned tag = P.gen * (unsigned)(P.max_iter + 1) + (unsigned)t + 1u;   // never 0 mod 2^32 in practice
        part_publish(pa, grs, ((unsigned)t * nwx + wgx) * 32u, tag, scr);
        if (P.dump) {   // xmmse and var after the denoiser (part_publish's barrier ordered the LDS writes)
            float* dp = P.dump + (((size_t)t * nwg + wg) * 5 + 2) * PBM * twoN;
            for (int e = tid; e < PBM * twoN; e += PWG) dp[e] = sX[(e / twoN) * ldr + e % twoN];
            for (int e = tid; e < PBM * N; e += PWG) dp[PBM * twoN + (e / N) * twoN + e % N] = vnew[e];
            if (tid == 0) {
                const Partial* sp = reinterpret_cast<const Partial*>(scr);
                for (int w = 0; w < PWG / 64; ++w) {
                    double v = sp[w].sumvar;
                    __builtin_memcpy(dp + PBM * twoN + N + 2 * w, &v, 8);
                }
                dp[PBM * twoN + twoN + N] = cur.inv_sigma2;   // row 1, column N: the denoiser's 1 / sigma2
            }
        }
        stamp(t, 5);
        kbase = karg_launder(kbase);
        Pp = karg_at<VampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, KARG_DC_OFF);
        if (!exchange(t, vnew, vprev)) { aborted = 1; break; }
        if (nx.stopped || t + 1 == P.max_iter) break;
        cur = nx;
    }
    __syncthreads();
    if (trc && tid == 0) {   // end stamps: per-workgroup clock rate against the global 100 MHz clock
        trc[(size_t)nwg * P.max_iter * AMP_TRACE_STRIDE + 2 * nwg + 2 * wg] = __builtin_amdgcn_s_memtime();
        trc[(size_t)nwg * P.max_iter * AMP_TRACE_STRIDE + 2 * nwg + 2 * wg + 1] = __builtin_amdgcn_s_memrealtime();
    }
    // outputs: r (decision input, vamp.py:187), xmmse, var of the last executed iteration
    const float* vlast = lds + ((last_t & 1) ? Y.offV1 : Y.offV0);
    for (int e = tid; e < nrows * twoN; e += PWG) {
        const int row = e / twoN, col = e - row * twoN;
        P.r[(size_t)(row0 + row) * twoN + col] = sR[row * ldr + col];
        P.xm[(size_t)(row0 + row) * twoN + col] = sX[row * ldr + col];
    }
    for (int e = tid; e < nrows * N; e += PWG) P.var0[(size_t)row0 * N + e] = vlast[e];
    amp_status st_rec = vamp_make_status(P, cur, nx, fixed);
    if (aborted) st_rec.nan_state = -1;
    if (wl == P.wg_off && tid == 0) P.status[ep] = st_rec;   // this launch's first workgroup of the epoch
    if (P.dec_on) {
        __syncthreads();   // the V0/V1 region (vlast) becomes the label / mismatch scratch
        // the records are folded here, by the epoch's first workgroup of this launch, from the
        // tagged granules every workgroup publishes (no fold launch; tag unique per launch)
        const unsigned dtag = P.fold_in ? P.gen * (unsigned)(P.max_iter + 1) + (unsigned)P.max_iter + 1u : 0u;
        decide_epilogue<PWG, KK, true>(P, dc, sR, sX, ldr, row0, lrow0, nrows, sA, lds + Y.offV0,
                                       4 * (Y.offScr - Y.offV0), scr, dtag);
        const int nloc = nwg / P.E;                    // this launch's workgroups of one epoch
        if (P.fold_in && wg % nloc == 0) {             // wl == P.wg_off: the status writer above
            __syncthreads();
            const bool ok = dec_fold_gather(P, wg, nloc, dtag, P.counts + ep, scr, &s_flag);
            if (tid == 0) {
                if (!ok) {                             // a workgroup never published: results invalid
                    st_rec.nan_state = -1;
                    P.status[ep] = st_rec;
                }
                if (P.host_rec && P.E == 1) host_record_write(P.host_rec, st_rec, P.counts[ep]);
            }
        }
    }
#undef P
#undef dc
#undef c64
#undef ebar
#undef Wx1
#undef Wx2
#undef grs
}

int device_cu_count();

// Launch path: persist_grid_launch (amp_host.h): a plain launch after an explicit co-residency
// check (default), or hipLaunchCooperativeKernel (AMP_PERSIST_LAUNCH=coop).
template <int NT, int KK, int NWV, int DU, bool X3, int OCC = 1, bool H2 = false, bool I8 = false>
static int persist_launch_t(const VampK& P, const DecConst& dc, hipStream_t st) {
    const void* fn = (const void*)vamp_persist<NT, KK, NWV, DU, X3, OCC, H2, I8>;
    const size_t lds = (size_t)playout(P.N, P.k, P.L, X3).total * 4;
    // the dynamic-LDS attribute and the occupancy query cost tens of us per call: once per
    // instantiation and LDS size (single-threaded host use, like the rest of the ABI)
    static size_t attr_lds = 0;
    static int per_cu = 0;
    hipError_t e = hipSuccess;
    if (attr_lds != lds) {
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("vamp_persist: hipFuncSetAttribute: %s", hipGetErrorString(e));
            return AMP_E_LAUNCH;
        }
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * NWV, lds);
        if (e != hipSuccess) per_cu = 0;
        attr_lds = lds;
    }
    // the bounded barrier spins stay as the backstop of either launch path
    VampK Pc = P;
    DecConst dd = dc;
    void* args[] = {(void*)&Pc, (void*)&dd};
    return persist_grid_launch("vamp_persist", fn, P.nwg, 64 * NWV, lds, per_cu, args, st);
}

template <int NT, int NWV, bool X3, int OCC = 1, bool H2 = false, bool I8 = false>
static int persist_launch_nt(const VampK& P, const DecConst& dc, hipStream_t st) {
    switch (P.c.K) {
    case 1: return persist_launch_t<NT, 1, NWV, 4, X3, OCC, H2, I8>(P, dc, st);
    case 2: return persist_launch_t<NT, 2, NWV, 4, X3, OCC, H2, I8>(P, dc, st);
    case 4: return persist_launch_t<NT, 4, NWV, AMP_KK4_DU, X3, OCC, H2, I8>(P, dc, st);
    case 8: return persist_launch_t<NT, 8, NWV, 2, X3, OCC, H2, I8>(P, dc, st);
    case 16:
        // two sections in flight per lane group (4 and 8 measured no faster, and spill)
        return persist_launch_t<NT, 16, NWV, X3 ? AMP_X3_DU : 2, X3, OCC, H2, I8>(P, dc, st);
    default: return persist_launch_t<NT, 64, NWV, 1, X3, OCC, H2, I8>(P, dc, st);
    }
}

}  // namespace amp
