// amp_scamp_persist_kernel.h — the persistent SCAMP engine kernel (scamp_persist) and its launch
// templates, shared by the f32-MFMA instantiations (amp_scamp_persist.hip) and the
// split-precision bf16x3 ones (amp_scamp_persist_x3.hip).  Design notes: amp_scamp_persist.hip.
#pragma once

#include <stdlib.h>

#include "amp_decide_fused.h"
#include "amp_persist.h"
#include "amp_scamp.h"

namespace amp {

constexpr int SPB = 16;   // trials per workgroup (the MFMA tile height)

// LDS carve (floats).  Row strides 2N + 4 and 2n + 4 keep the 16-row ds_read_b128 of gemm16 and
// the accumulator stores conflict-free.
struct SLayout {
    int ldx, ldz;
    int offX, offR, offZ, offS, offP0, offP1, offPhi, offB, offIph, offTau, offITau, offSM, offSA, offScr, total;
};

// X3: the GEMM A operands (x for GEMM1, s = z / phi for GEMM2) as six bf16 planes of 16 rows x
// K (amp_persist.h's XOR-permuted layout) in the region of the f32 s rows (one operand at a time)
__host__ __device__ inline int sx3_plane_floats(int K) { return 6 * 16 * pl_ldx(K) / 2; }

__host__ __device__ inline SLayout slayout(int N, int n, int L, int Lin, int Lout, bool x3 = false) {
    SLayout y;
    y.ldx = 2 * N + 4;
    y.ldz = 2 * n + 4;
    int o = 0;
    y.offX = o; o += SPB * y.ldx;
    y.offR = o; o += SPB * y.ldx;
    y.offZ = o; o += SPB * y.ldz;
    const int kmax = N > n ? N : n;
    y.offS = o; o += (x3 && sx3_plane_floats(kmax) > SPB * y.ldz) ? sx3_plane_floats(kmax) : SPB * y.ldz;
    y.offP0 = o; o += SPB * Lin;
    y.offP1 = o; o += SPB * Lin;
    y.offPhi = o; o += SPB * Lout;
    y.offB = o; o += SPB * Lout;
    y.offIph = o; o += SPB * Lout;
    y.offTau = o; o += SPB * Lin;
    y.offITau = o; o += SPB * Lin;
    y.offSM = o; o += SPB * L;
    y.offSA = o; o += SPB * L;
    o = (o + 3) & ~3;
    y.offScr = o; o += 1024;
    y.total = o;
    return y;
}

// Denoiser policy over the LDS-resident xmap rows (scamp.py:61-68): mean only, tau_use / 2 per
// coupling block.
struct SPDenoisePolicy {
    const float* r;       // xmap rows
    float* x;             // xmmse rows (out)
    const float* itau;    // [SPB][Lin] 1 / (tau * 0.5)
    float* sm;
    float* sa;
    int ldx, M, lspr, Nt, Lin;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const int row = sec >> lspr, sj = sec & ((1 << lspr) - 1);
        const int cc = sj * M + m;
        const float2 v = *reinterpret_cast<const float2*>(r + row * ldx + 2 * cc);
        rr = v.x; ri = v.y;
        it = itau[row * Lin + cc / Nt];
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float, PartAcc&) const {
        const int row = sec >> lspr, sj = sec & ((1 << lspr) - 1);
        *reinterpret_cast<float2*>(x + row * ldx + 2 * (sj * M + m)) = make_float2(xr, xi);
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        sm[sec] = smax;
        sa[sec] = sabs;
    }
};

// psi of one (row, coupling block) by one wavefront: 1 - sum |x|^2 / Na, |x| as torch.abs
// (float32 hypot via float64), the sum in float64 (scamp.py:59).
__device__ __forceinline__ float block_psi(const float* xrow, int lc, int Nt, int Na) {
    const int lane = threadIdx.x & 63;
    double ssum = 0.0;
    for (int m = lane; m < Nt; m += 64) {
        const float2 v = *reinterpret_cast<const float2*>(xrow + 2 * (lc * Nt + m));
        const float a = (float)sqrt((double)v.x * v.x + (double)v.y * v.y);
        ssum += (double)(a * a);
    }
    ssum = group_sum(ssum, 64);
    return 1.0f - (float)ssum / (float)Na;
}

// X3: both GEMMs on the split-precision bf16x3 engine (amp_persist.h gemm_x3); the wave's complex
// column tiles are NT1/2 (GEMM1) and NT2/2 (GEMM2), the same real columns as the f32 form.
// H2 (with X3): the fp16x2 form (gemm_h2): every A row (x, then s = z / phi) scaled by its own
// power of two before the split, the accumulators scaled back by 2^-(e_row + SH2_EX).
// NWV: waves per workgroup — 4 (one per SIMD) or, for bf16x3, 8 (two per SIMD, 256 registers
// each, half the column tiles per wave; the per-point packed denoiser is then replaced by the
// scalar one, the 16-point alphabets keep the packed product grid: DESIGN.md §3.1, §3.8).
// The arguments are read through the laundered kernarg pointer (amp_persist.h karg_launder), as in
// vamp_persist: the eight-wave cfg3 build held them in SGPRs for the whole launch (387 spilled).
constexpr int SKARG_DC_OFF = karg_second_offset<ScampK, DecConst>();
template <int NT1, int G1, int NT2, int G2, int KK, bool X3, bool H2 = false, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, NWV / 4) void scamp_persist(ScampK P_arg, DecConst dc_arg) {
    (void)P_arg;
    (void)dc_arg;
    unsigned long long kbase = karg_base();
    const ScampK* Pp = karg_at<ScampK>(kbase, 0);
    const DecConst* Dp = karg_at<DecConst>(kbase, SKARG_DC_OFF);
#define P (*Pp)
#define dc (*Dp)
#define c64 (static_cast<const Const64&>(*Dp))   // the rare path's float64 table; dc also the fused decision's (dec_on)
    constexpr int PWG = 64 * NWV, NW = NWV;
    static_assert(NWV == 4 || (NWV == 8 && X3 && !H2), "eight waves: the bf16x3 form only");
    constexpr int NC1 = X3 ? NT1 / 2 : 1, NC2 = X3 ? NT2 / 2 : 1;
    static_assert(!X3 || (NT1 % 2 == 0 && NT2 % 2 == 0), "X3: whole complex tiles");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_flag;
    __shared__ double s_d[NW][4];
    __shared__ float s_hmax[NW][SPB];   // H2: per-wave row maxima of the A operand
    __shared__ int s_hexp[SPB];         // H2: x row exponents (for GEMM1's epilogue)
    const int N = P.N, n = P.n, L = P.L, M = P.M, Lin = P.Lin, Lout = P.Lout, Nt = P.Nt, Nr = P.Nr;
    const SLayout Y = slayout(N, n, L, Lin, Lout, X3);
    const int ldx = Y.ldx, ldz = Y.ldz;
    float* sX = lds + Y.offX;
    float* sR = lds + Y.offR;
    float* sZ = lds + Y.offZ;
    float* sS = lds + Y.offS;
    float* sPhi = lds + Y.offPhi;
    float* sB = lds + Y.offB;
    float* sIph = lds + Y.offIph;
    float* sTau = lds + Y.offTau;
    float* sITau = lds + Y.offITau;
    float* sM = lds + Y.offSM;
    float* sA = lds + Y.offSA;
    float* scr = lds + Y.offScr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wg = blockIdx.x, nwg = gridDim.x;
    const int row0 = wg * SPB, nrows = min(SPB, P.B - row0);
    const int twoN = 2 * N, twon = 2 * n, spr = N / M;

    // y rows of this wave's GEMM1 columns, in the accumulator layout (read once; X3: yt[2t] / yt[2t+1]
    // = Re / Im of complex tile t)
    const int ct1 = wave * NT1, ct2 = wave * NT2;
    const int cc1 = wave * NC1, cc2 = wave * NC2;
    unsigned short* sP = reinterpret_cast<unsigned short*>(sS);
    const int ldp1 = pl_ldx(N), ldp2 = pl_ldx(n);      // X3 plane row strides (bf16) of the GEMM1 / GEMM2 operands
    float yt[NT1][4];
#pragma unroll
    for (int t2 = 0; t2 < NT1; ++t2) {
        const int col = X3 ? 2 * (16 * (cc1 + t2 / 2) + (lane & 15)) + (t2 & 1) : 16 * (ct1 + t2) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * (lane >> 4) + r;
            // unconditional load at a clamped row, zeroed after it (a lane-divergent branch around
            // the load serialises the loads' latencies: amp_gemm.h ALoadPlain)
            const float yv = P.y[(size_t)(row0 + max(min(row, nrows - 1), 0)) * twon + col];
            yt[t2][r] = (row < nrows) ? yv : 0.f;
        }
    }
    // Tracker (scamp.py:9-25): x = 0, z = y, psi = 1, phi = +inf
    for (int e = tid; e < SPB * twoN; e += PWG) {
        const int row = e / twoN, col = e - row * twoN;
        sX[row * ldx + col] = 0.f;
    }
    for (int e = tid; e < SPB * twon; e += PWG) {
        const int row = e / twon, col = e - row * twon;
        const float yv = P.y[(size_t)(row0 + max(min(row, nrows - 1), 0)) * twon + col];
        sZ[row * ldz + col] = (row < nrows) ? yv : 0.f;
    }
    for (int e = tid; e < SPB * Lin; e += PWG) lds[Y.offP0 + e] = lds[Y.offP1 + e] = 1.0f;
    for (int e = tid; e < SPB * Lout; e += PWG) sPhi[e] = INFINITY;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t grs = gran_rsrc(P.pparts, (unsigned)(P.max_iter * nwg) * 32u);
    unsigned nbar = 0;
    int fixed = 0, fixed_all = 0, aborted = 0, stopped = 0, T = P.max_iter, last_t = 0;
    // diagnostic phase stamps (amp_scamp_persist_trace): 0 start, 1 scalars + x planes, 2 GEMM1,
    // 3 s stored, 4 GEMM2 + xmap, 5 denoiser, 6 psi + publish, 7 gather, 8 iteration end
    unsigned long long* trc = P.trace;
    auto stamp = [&](int t, int ph) {
        if (trc && tid == 0) trc[((size_t)wg * P.max_iter + t) * 10 + ph] = __builtin_amdgcn_s_memtime();
    };

    for (int t = 0; t < P.max_iter; ++t) {
        kbase = karg_launder(kbase);
        Pp = karg_at<ScampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, SKARG_DC_OFF);
        last_t = t;
        stamp(t, 0);
        float* psi_prev = lds + ((t & 1) ? Y.offP0 : Y.offP1);
        float* psi_new = lds + ((t & 1) ? Y.offP1 : Y.offP0);
        // 1. coupling scalars per trial (scamp.py:45-53), float32 as amp_scamp.hip forms them
        for (int e = tid; e < SPB * Lout; e += PWG) {
            const int row = e / Lout, lo = e - row * Lout;
            float g = 0.f;
            for (int lc = 0; lc < Lin; ++lc) g += P.W[lo * Lin + lc] * psi_prev[row * Lin + lc];
            const float gma = g / (float)Lin;                  // gamma = W psi / Lc
            sB[e] = gma / sPhi[e];                            // b = gamma / phi_old (0 at t = 0)
            const float ph = P.sigma2 + gma;                  // phi = sigma2 + gamma
            sIph[e] = 1.0f / ph;
            sPhi[e] = ph;
        }
        __syncthreads();
        for (int e = tid; e < SPB * Lin; e += PWG) {
            const int row = e / Lin, lc = e - row * Lin;
            float acc = 0.f;                                  // (W^T (1/phi))[lc]
            for (int lo = 0; lo < Lout; ++lo) acc += P.W[lo * Lin + lc] * (1.0f / sPhi[row * Lout + lo]);
            const float tv = ((1.0f / acc) * (float)L) / (float)Nr;   // L / x = recip(x) * L ; / Mr
            sTau[e] = tv;
            sITau[e] = 1.0f / (tv * 0.5f);                    // tau_use / 2 (scamp.py:63)
        }
        // 2. GEMM1 A x (A operand: the x rows as they lie) ; z = y - A x + b z ; s = z / phi
        f32x4 acc1[NT1];
        f32x4 cr1[NC1], ci1[NC1];
        if constexpr (H2) {
            // x rows in registers (item e: row e % SPB == tid % SPB), each row's max |x| over the
            // workgroup, then the scaled split into the four fp16 planes
            constexpr int IPT = (SPB * G1 + PWG - 1) / PWG;  // items per thread: SPB N / 8 / PWG, N = G1 * 8
            const int row = tid % SPB;
            float re[IPT][8], im[IPT][8];
            float m = 0.f;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tid + i * PWG;
                const bool ok = e < SPB * (N >> 3);
                const int j0 = 8 * (e / SPB);
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (ok) v = *reinterpret_cast<const float4*>(sX + row * ldx + 2 * j0 + 4 * h);
                    re[i][2 * h] = v.x; im[i][2 * h] = v.y; re[i][2 * h + 1] = v.z; im[i][2 * h + 1] = v.w;
                }
#pragma unroll
                for (int h = 0; h < 8; ++h) m = fmaxf(m, fmaxf(fabsf(re[i][h]), fabsf(im[i][h])));
            }
            m = fmaxf(m, __shfl_xor(m, 16));
            m = fmaxf(m, __shfl_xor(m, 32));
            if (lane < SPB) s_hmax[wave][lane] = m;
            __syncthreads();
            float mr = s_hmax[0][row];
#pragma unroll
            for (int w = 1; w < NW; ++w) mr = fmaxf(mr, s_hmax[w][row]);
            const int ex = h2_row_exp(mr);
            if (tid < SPB) s_hexp[tid] = ex;
#pragma unroll
            for (int i = 0; i < IPT; ++i) {
                const int e = tid + i * PWG;
                if (e < SPB * (N >> 3)) {
#pragma unroll
                    for (int h = 0; h < 8; ++h) {
                        re[i][h] = __builtin_amdgcn_ldexpf(re[i][h], ex);
                        im[i][h] = __builtin_amdgcn_ldexpf(im[i][h], ex);
                    }
                    h2_store8(sP, ldp1, row, 8 * (e / SPB), re[i], im[i]);
                }
            }
            __syncthreads();
            stamp(t, 1);
            gemm_h2<NC1, G1 / 4>(sP, ldp1, P.Wx1, cc1, cr1, ci1);
        } else if constexpr (X3) {
            for (int e = tid; e < SPB * (N >> 3); e += PWG) {   // x rows -> bf16 planes, 8 per item
                // consecutive items walk the 16 rows (stride 2N + 4 floats): conflict-free reads
                const int row = e % SPB, j0 = 8 * (e / SPB);
                float re[8], im[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const float4 v = *reinterpret_cast<const float4*>(sX + row * ldx + 2 * j0 + 4 * h);
                    re[2 * h] = v.x; im[2 * h] = v.y; re[2 * h + 1] = v.z; im[2 * h + 1] = v.w;
                }
                x3_store8(sP, ldp1, row, j0, re, im);
            }
            __syncthreads();
            stamp(t, 1);
            gemm_x3<NC1, G1 / 4>(sP, ldp1, P.Wx1, cc1, cr1, ci1);
        } else {
            stamp(t, 1);
            gemm16<NT1, G1>(sX, ldx, P.Wq1, ct1, acc1);
        }
        float hsc[4];   // H2: 2^-(e_row + SH2_EX) of this lane's rows (x rows, then s rows)
        if constexpr (H2) {
            // z and s = z / phi of every tile of this wave (s kept in cr1 / ci1), the rows' max |s|
            // to LDS; the barrier below also ends every wave's reads of the x planes
#pragma unroll
            for (int r = 0; r < 4; ++r) hsc[r] = __builtin_amdgcn_ldexpf(1.0f, -(s_hexp[4 * (lane >> 4) + r] + SH2_EX));
        }
        __syncthreads();   // tau / b / phi published; every wave done reading x
        stamp(t, 2);
        if constexpr (H2) {
            float mrow[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t2 = 0; t2 < NC1; ++t2) {
                const int o = 16 * (cc1 + t2) + (lane & 15);
                const int lo = o / Nr;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * (lane >> 4) + r;
                    const int b = row * ldz + 2 * o;
                    const float bz = sB[row * Lout + lo], ip = sIph[row * Lout + lo];
                    const float zr = (yt[2 * t2][r] - cr1[t2][r] * hsc[r]) + bz * sZ[b];
                    const float zi = (yt[2 * t2 + 1][r] - ci1[t2][r] * hsc[r]) + bz * sZ[b + 1];
                    sZ[b] = zr; sZ[b + 1] = zi;
                    cr1[t2][r] = zr * ip; ci1[t2][r] = zi * ip;
                    mrow[r] = fmaxf(mrow[r], fmaxf(fabsf(cr1[t2][r]), fabsf(ci1[t2][r])));
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
            __syncthreads();
            int hes[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float mr = s_hmax[0][4 * (lane >> 4) + r];
#pragma unroll
                for (int w = 1; w < NW; ++w) mr = fmaxf(mr, s_hmax[w][4 * (lane >> 4) + r]);
                hes[r] = h2_row_exp(mr);
                hsc[r] = __builtin_amdgcn_ldexpf(1.0f, -(hes[r] + SH2_EX));
            }
#pragma unroll
            for (int t2 = 0; t2 < NC1; ++t2) {
                const int o = 16 * (cc1 + t2) + (lane & 15);
                float sr[4], si[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sr[r] = __builtin_amdgcn_ldexpf(cr1[t2][r], hes[r]);
                    si[r] = __builtin_amdgcn_ldexpf(ci1[t2][r], hes[r]);
                }
                h2_store_acc(sP, ldp2, o, sr, si);
            }
        } else if constexpr (X3) {
#pragma unroll
            for (int t2 = 0; t2 < NC1; ++t2) {
                const int o = 16 * (cc1 + t2) + (lane & 15);
                const int lo = o / Nr;
                float sr[4], si[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * (lane >> 4) + r;
                    const int b = row * ldz + 2 * o;
                    const float bz = sB[row * Lout + lo], ip = sIph[row * Lout + lo];
                    const float zr = (yt[2 * t2][r] - cr1[t2][r]) + bz * sZ[b];
                    const float zi = (yt[2 * t2 + 1][r] - ci1[t2][r]) + bz * sZ[b + 1];
                    sZ[b] = zr; sZ[b + 1] = zi;
                    sr[r] = zr * ip; si[r] = zi * ip;
                }
                x3_store_acc(sP, ldp2, o, sr, si);
            }
        } else
#pragma unroll
        for (int t2 = 0; t2 < NT1; ++t2) {
            const int col = 16 * (ct1 + t2) + (lane & 15);
            const int lo = (col >> 1) / Nr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r;
                const int o = row * ldz + col;
                const float zz = (yt[t2][r] - acc1[t2][r]) + sB[row * Lout + lo] * sZ[o];
                sZ[o] = zz;
                sS[o] = zz * sIph[row * Lout + lo];
            }
        }
        __syncthreads();
        stamp(t, 3);
        // 3. GEMM2 A^H s ; xmap = x + tau (A^H s)
        f32x4 acc2[NT2];
        if constexpr (X3) {
            f32x4 cr2[NC2], ci2[NC2];
            if constexpr (H2) {
                gemm_h2<NC2, G2 / 4>(sP, ldp2, P.Wx2, cc2, cr2, ci2);
#pragma unroll
                for (int t2 = 0; t2 < NC2; ++t2)
#pragma unroll
                    for (int r = 0; r < 4; ++r) { cr2[t2][r] *= hsc[r]; ci2[t2][r] *= hsc[r]; }
            } else {
                gemm_x3<NC2, G2 / 4>(sP, ldp2, P.Wx2, cc2, cr2, ci2);
            }
#pragma unroll
            for (int t2 = 0; t2 < NC2; ++t2) {
                const int o = 16 * (cc2 + t2) + (lane & 15);
                const int lc = o / Nt;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * (lane >> 4) + r;
                    const int b = row * ldx + 2 * o;
                    const float tv = sTau[row * Lin + lc];
                    sR[b] = sX[b] + tv * cr2[t2][r];
                    sR[b + 1] = sX[b + 1] + tv * ci2[t2][r];
                }
            }
        } else {
        gemm16<NT2, G2>(sS, ldz, P.Wq2, ct2, acc2);
#pragma unroll
        for (int t2 = 0; t2 < NT2; ++t2) {
            const int col = 16 * (ct2 + t2) + (lane & 15);
            const int lc = (col >> 1) / Nt;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r;
                const int o = row * ldx + col;
                sR[o] = sX[o] + sTau[row * Lin + lc] * acc2[t2][r];
            }
        }
        }
        __syncthreads();
        stamp(t, 4);
        kbase = karg_launder(kbase);
        Pp = karg_at<ScampK>(kbase, 0);
        Dp = karg_at<DecConst>(kbase, SKARG_DC_OFF);
        // 4. denoiser -> x, then psi and its allclose count
        SPDenoisePolicy pol{sR, sX, sITau, sM, sA, ldx, M, 31 - __builtin_clz(spr), Nt, Lin};
        PartAcc pa;
        if constexpr (KK > 16)
            denoise_sections_wide_m<false, KK>(pol, nrows * spr, M, P.c, pa);
        else
            denoise_sections_u<false, KK, (KK >= 8 ? 2 : 4), (NWV == 4 ? PK_ALL : KK == 16 ? PK_GRID : PK_NONE)>(pol, nrows * spr, M, P.c, pa);
        __syncthreads();
        stamp(t, 5);
        unsigned nc = 0;
        {
            // psi of every (row, block): groups of GS = min(16, Nt) lanes, 64 / GS blocks per wave
            // pass, each lane summing every GS-th |x|^2 of its block in float64, then a GS-lane
            // butterfly (the terms as block_psi forms them; one short reduction per pass instead
            // of a 64-lane one per block)
            const int GS = Nt < 16 ? Nt : 16, bpw = 64 / GS, gi = lane / GS, gl = lane - gi * GS;
            for (int b0 = wave * bpw; b0 < nrows * Lin; b0 += NW * bpw) {   // wave-uniform
                const int b = b0 + gi;
                const bool in = b < nrows * Lin;
                double ssum = 0.0;
                if (in) {
                    const int row = b / Lin, lc = b - row * Lin;
                    const float* xr = sX + row * ldx + 2 * lc * Nt;
                    for (int m = gl; m < Nt; m += GS) {
                        const float2 v = *reinterpret_cast<const float2*>(xr + 2 * m);
                        const float a = (float)sqrt((double)v.x * v.x + (double)v.y * v.y);
                        ssum += (double)(a * a);
                    }
                }
                for (int off = GS >> 1; off > 0; off >>= 1) ssum += __shfl_xor(ssum, off);
                if (in && gl == 0) {
                    const float ps = 1.0f - (float)ssum / (float)P.Na;
                    nc += torch_close(ps, psi_prev[b]) ? 0u : 1u;             // scamp.py:105
                    psi_new[b] = ps;
                }
            }
        }
        pa.notclose += nc;
        const unsigned tag = P.gen * (unsigned)(P.max_iter + 1) + (unsigned)t + 1u;
        part_publish(pa, grs, ((unsigned)t * nwg + wg) * 32u, tag, scr);
        stamp(t, 6);
        // 5. batch-global max|xi| / danger test / allclose count
        PartAcc g;
        if (!part_gather(grs, (unsigned)t * nwg * 32u, nwg, tag, P.pbar + 1, g, scr, &s_flag)) {
            aborted = 1;
            break;
        }
        stamp(t, 7);
        fixed = 0;
        uint32_t notclose = g.notclose;
        if (part_allnan(g)) {
            // torch's max|xi| is NaN / inf: every section of this iteration is NaN, psi too
            if (!fixed_all) {
                const float qn = __int_as_float(0x7fc00000);
                for (int e = tid; e < nrows * twoN; e += PWG) sX[(e / twoN) * ldx + e % twoN] = qn;
                for (int e = tid; e < nrows * Lin; e += PWG) psi_new[e] = qn;
            }
            notclose = 1;
            fixed = -1;
            fixed_all = 1;
        } else if (part_danger(g)) {
            // (a) exact float64 G over the candidate sections of every workgroup
            const double G32 = g.maxabs, slack = logit_slack(G32);
            auto ldf = [=](int s) {
                const int row = s / spr, sj = s - row * spr;
                const float* rp = sR + row * ldx + 2 * sj * M;
                const float it = sITau[row * Lin + (sj * M) / Nt];
                return [=](int m, float& rr, float& ri, float& itv) {
                    rr = rp[2 * m]; ri = rp[2 * m + 1]; itv = it;
                };
            };
            double gm = 0.0;
            for (int s = tid; s < nrows * spr; s += PWG)
                if ((double)sA[s] >= G32 - slack) gm = fmax(gm, section_absmax_f64(ldf(s), M, c64));
            gm = group_max(gm, 64);
            if (lane == 0) s_d[wave][0] = gm;
            __syncthreads();
            if (tid == 0) {
                double m4 = 0.0;
                for (int w = 0; w < NW; ++w) m4 = fmax(m4, s_d[w][0]);
                P.pxch[((size_t)t * nwg + wg) * 4 + 0] = m4;
            }
            if (!grid_sync(P.pbar, ++nbar * (unsigned)nwg, &s_flag)) { aborted = 1; break; }
            double G = 0.0;
            for (int w = 0; w < nwg; ++w) G = fmax(G, P.pxch[((size_t)t * nwg + w) * 4 + 0]);
            // (b) exact recompute of this workgroup's sections below the danger line, then the
            //     psi of their coupling blocks (scamp_fix_sec / scamp_fix_psi of the launch engine)
            int cnt = 0;
            for (int s = tid; s < nrows * spr; s += PWG) {
                if (!((double)sM[s] - G < AMP_DANGER + slack)) continue;
                ++cnt;
                const int row = s / spr, sj = s - row * spr;
                float* xp = sX + row * ldx + 2 * sj * M;
                auto st = [=](int m, float xr, float xi, float) { xp[2 * m] = xr; xp[2 * m + 1] = xi; };
                exact_section_f64<false>(ldf(s), st, M, c64, G);
            }
            __syncthreads();
            int dnc = 0;
            const int spb = Nt / M;   // sections per coupling block
            for (int b = wave; b < nrows * Lin; b += NW) {
                bool hit = false;
                for (int j = 0; j < spb && !hit; ++j) hit = (double)sM[b * spb + j] - G < AMP_DANGER + slack;
                if (!hit) continue;                            // wave-uniform
                const int row = b / Lin, lc = b - row * Lin;
                const float ps = block_psi(sX + row * ldx, lc, Nt, P.Na);
                if (lane == 0) {
                    dnc += (torch_close(ps, psi_prev[b]) ? 0 : 1) - (torch_close(psi_new[b], psi_prev[b]) ? 0 : 1);
                    psi_new[b] = ps;
                }
            }
            cnt = group_sum(cnt, 64);
            dnc = group_sum(dnc, 64);
            __syncthreads();
            if (lane == 0) { s_d[wave][1] = (double)cnt; s_d[wave][2] = (double)dnc; }
            __syncthreads();
            if (tid == 0) {
                double a = 0.0, b = 0.0;
                for (int w = 0; w < NW; ++w) { a += s_d[w][1]; b += s_d[w][2]; }
                P.pxch[((size_t)t * nwg + wg) * 4 + 1] = a;
                P.pxch[((size_t)t * nwg + wg) * 4 + 2] = b;
            }
            if (!grid_sync(P.pbar, ++nbar * (unsigned)nwg, &s_flag)) { aborted = 1; break; }
            double a = 0.0, b = 0.0;
            for (int w = 0; w < nwg; ++w) {
                a += P.pxch[((size_t)t * nwg + w) * 4 + 1];
                b += P.pxch[((size_t)t * nwg + w) * 4 + 2];
            }
            fixed = (int)a;
            notclose = (uint32_t)((long long)notclose + (long long)b);
        }
        __syncthreads();
        stamp(t, 8);
        if (notclose == 0) {                                   // scamp.py:105-106
            stopped = 1;
            T = t + 1;
            break;
        }
    }
    __syncthreads();
    // outputs: xmap (the decision input, scamp.py:107), xmmse, psi of the last executed iteration
    const float* psi_last = lds + ((last_t & 1) ? Y.offP1 : Y.offP0);
    for (int e = tid; e < nrows * twoN; e += PWG) {
        const int row = e / twoN, col = e - row * twoN;
        P.xmap[(size_t)(row0 + row) * twoN + col] = sR[row * ldx + col];
        P.xm[(size_t)(row0 + row) * twoN + col] = sX[row * ldx + col];
    }
    for (int e = tid; e < nrows * Lin; e += PWG) P.psi0[(size_t)row0 * Lin + e] = psi_last[e];
    amp_status s;
    s.T = stopped ? T : P.max_iter;
    s.nan_state = aborted ? -1 : (fixed != 0 ? 1 : 0);
    s.stopped = stopped;
    s.gemm = P.x3 + 1;   // x3: 0 f32, 1 bf16x3, 2 fp16x2
    s.last_scalar[0] = s.last_scalar[1] = s.last_scalar[2] = s.last_scalar[3] = 0.f;
    if (wg == 0 && tid == 0) *P.status = s;
    if (P.dec_on) {
        // fused MAP decision + counters on xmap (scamp.py:107 -> loss.py:67-179): the s / plane region
        // holds the truth rows (n >= N: rows of ldx floats fit), the z region the labels; workgroup 0
        // folds every workgroup's record from its tagged granules (no fold launch)
        __syncthreads();
        const unsigned dtag = P.fold_in ? P.gen * (unsigned)(P.max_iter + 1) + (unsigned)P.max_iter + 1u : 0u;
        decide_epilogue<PWG, KK, true>(P, dc, sR, sX, ldx, row0, row0, nrows, sS, sZ, 4 * SPB * Y.ldz, scr, dtag);
        if (P.fold_in && wg == 0) {
            __syncthreads();
            const bool ok = dec_fold_gather(P, 0, nwg, dtag, P.counts, scr, &s_flag);
            if (tid == 0) {
                if (!ok) {   // a workgroup never published: results invalid
                    s.nan_state = -1;
                    *P.status = s;
                }
                if (P.host_rec) host_record_write(P.host_rec, s, *P.counts);
            }
        }
    }
#undef P
#undef dc
#undef c64
}

int device_cu_count();

template <int NT1, int G1, int NT2, int G2, int KK, bool X3, bool H2 = false, int NWV = 4>
static int spersist_launch_t(const ScampK& P, const DecConst& dc, hipStream_t st) {
    const void* fn = (const void*)scamp_persist<NT1, G1, NT2, G2, KK, X3, H2, NWV>;
    const size_t lds = (size_t)slayout(P.N, P.n, P.L, P.Lin, P.Lout, X3).total * 4;
    // the dynamic-LDS attribute and the occupancy query: once per instantiation and LDS size
    static size_t attr_lds = 0;
    static int per_cu = 0;
    if (attr_lds != lds) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("scamp_persist: hipFuncSetAttribute: %s", hipGetErrorString(e));
            return AMP_E_LAUNCH;
        }
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * NWV, lds) != hipSuccess) per_cu = 0;
        attr_lds = lds;
    }
    // persist_grid_launch (amp_host.h): plain launch after the co-residency check, or the
    // cooperative one; every barrier spin is bounded (2 s) as the backstop
    ScampK Pc = P;
    DecConst cc = dc;
    void* args[] = {(void*)&Pc, (void*)&cc};
    return persist_grid_launch("scamp_persist", fn, P.nwg, 64 * NWV, lds, per_cu, args, st);
}

template <int NT1, int G1, int NT2, int G2, bool X3, bool H2 = false, int NWV = 4>
static int spersist_launch_s(const ScampK& P, const DecConst& c64, hipStream_t st) {
    switch (P.c.K) {
    case 1: return spersist_launch_t<NT1, G1, NT2, G2, 1, X3, H2, NWV>(P, c64, st);
    case 2: return spersist_launch_t<NT1, G1, NT2, G2, 2, X3, H2, NWV>(P, c64, st);
    case 4: return spersist_launch_t<NT1, G1, NT2, G2, 4, X3, H2, NWV>(P, c64, st);
    case 8: return spersist_launch_t<NT1, G1, NT2, G2, 8, X3, H2, NWV>(P, c64, st);
    case 16: return spersist_launch_t<NT1, G1, NT2, G2, 16, X3, H2, NWV>(P, c64, st);
    default: return spersist_launch_t<NT1, G1, NT2, G2, 64, X3, H2, NWV>(P, c64, st);
    }
}

}  // namespace amp
