// amp_scamp_persist.hip — persistent SCAMP engine: the whole iteration loop of SCAMP.forward
// (scamp.py:77-107) in ONE launch.
//
// Each workgroup (256 threads, one wave per SIMD, one workgroup per CU) owns PB = 16 trials for
// the whole forward; their state lives in LDS across iterations: xmmse (x), xmap, z, the GEMM2
// operand s = z / phi, psi (this and the previous iteration), phi, and the per-row coupling
// scalars.  Per iteration t (same arithmetic, element by element, as amp_scamp.hip):
//   1. per (trial, row block lo): gamma = W psi / Lc, b = gamma / phi_old, phi = sigma2 + gamma
//      (scamp.py:45-51); per (trial, column block lc): tau = L / (W^T (1/phi)) / Mr (scamp.py:53)
//   2. GEMM1 A x on v_mfma_f32_16x16x4_f32 (A 16x16x4-packed, streamed from L2) with the
//      epilogue z = y - A x + b z, s = z / phi  (scamp.py:47-49, 57)
//   3. GEMM2 A^H s, epilogue xmap = x + tau (A^H s)  (scamp.py:55-57)
//   4. the mean-only section denoiser on xmap (tau/2, scamp.py:61-68) -> x, and
//      psi = 1 - sum_block |x|^2 / Na with its allclose count (scamp.py:59, 105)
//   5. the batch-global exchange (amp_persist.h granules): max|xi|, the danger test of the
//      float64 softmax, and the allclose count; the rare exact float64 path (amp_denoise.h) takes
//      two bounded grid barriers, uniformly in every workgroup.
// Launch-engine parity: the same f32 operations in the same order per element, so the only
// differences are the GEMM summation order (16x16x4 vs 32x32x2 MFMA) and psi's float64 sum
// order — the summation-order noise the curve tests accept.
#include <stdlib.h>

#include <atomic>
#include <mutex>

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

__host__ __device__ inline SLayout slayout(int N, int n, int L, int Lin, int Lout) {
    SLayout y;
    y.ldx = 2 * N + 4;
    y.ldz = 2 * n + 4;
    int o = 0;
    y.offX = o; o += SPB * y.ldx;
    y.offR = o; o += SPB * y.ldx;
    y.offZ = o; o += SPB * y.ldz;
    y.offS = o; o += SPB * y.ldz;
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

template <int NT1, int G1, int NT2, int G2, int KK>
__global__ __launch_bounds__(256, 1) void scamp_persist(ScampK P, Const64 c64) {
    constexpr int PWG = 256, NW = 4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_flag;
    __shared__ double s_d[NW][4];
    const int N = P.N, n = P.n, L = P.L, M = P.M, Lin = P.Lin, Lout = P.Lout, Nt = P.Nt, Nr = P.Nr;
    const SLayout Y = slayout(N, n, L, Lin, Lout);
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

    // y rows of this wave's GEMM1 columns, in the accumulator layout (read once)
    const int ct1 = wave * NT1, ct2 = wave * NT2;
    float yt[NT1][4];
#pragma unroll
    for (int t2 = 0; t2 < NT1; ++t2) {
        const int col = 16 * (ct1 + t2) + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * (lane >> 4) + r;
            yt[t2][r] = (row < nrows) ? P.y[(size_t)(row0 + row) * twon + col] : 0.f;
        }
    }
    // Tracker (scamp.py:9-25): x = 0, z = y, psi = 1, phi = +inf
    for (int e = tid; e < SPB * twoN; e += PWG) {
        const int row = e / twoN, col = e - row * twoN;
        sX[row * ldx + col] = 0.f;
    }
    for (int e = tid; e < SPB * twon; e += PWG) {
        const int row = e / twon, col = e - row * twon;
        sZ[row * ldz + col] = (row < nrows) ? P.y[(size_t)(row0 + row) * twon + col] : 0.f;
    }
    for (int e = tid; e < SPB * Lin; e += PWG) lds[Y.offP0 + e] = lds[Y.offP1 + e] = 1.0f;
    for (int e = tid; e < SPB * Lout; e += PWG) sPhi[e] = INFINITY;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t grs = gran_rsrc(P.pparts, (unsigned)(P.max_iter * nwg) * 32u);
    unsigned nbar = 0;
    int fixed = 0, fixed_all = 0, aborted = 0, stopped = 0, T = P.max_iter, last_t = 0;

    for (int t = 0; t < P.max_iter; ++t) {
        last_t = t;
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
        gemm16<NT1, G1>(sX, ldx, P.Wq1, ct1, acc1);
        __syncthreads();   // tau / b / phi published; every wave done reading x
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
        // 3. GEMM2 A^H s ; xmap = x + tau (A^H s)
        f32x4 acc2[NT2];
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
        __syncthreads();
        // 4. denoiser -> x, then psi and its allclose count
        SPDenoisePolicy pol{sR, sX, sITau, sM, sA, ldx, M, 31 - __builtin_clz(spr), Nt, Lin};
        PartAcc pa;
        if constexpr (KK > 16)
            denoise_sections_wide_m<false, KK>(pol, nrows * spr, M, P.c, pa);
        else
            denoise_sections_u<false, KK, (KK >= 8 ? 2 : 4)>(pol, nrows * spr, M, P.c, pa);
        __syncthreads();
        unsigned nc = 0;
        for (int b = wave; b < nrows * Lin; b += NW) {        // one wavefront per (row, block)
            const int row = b / Lin, lc = b - row * Lin;
            const float ps = block_psi(sX + row * ldx, lc, Nt, P.Na);
            if (lane == 0) {
                nc += torch_close(ps, psi_prev[b]) ? 0u : 1u;                 // scamp.py:105
                psi_new[b] = ps;
            }
        }
        pa.notclose += nc;
        const unsigned tag = P.gen * (unsigned)(P.max_iter + 1) + (unsigned)t + 1u;
        part_publish(pa, grs, ((unsigned)t * nwg + wg) * 32u, tag, scr);
        // 5. batch-global max|xi| / danger test / allclose count
        PartAcc g;
        if (!part_gather(grs, (unsigned)t * nwg * 32u, nwg, tag, P.pbar + 1, g, scr, &s_flag)) {
            aborted = 1;
            break;
        }
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
    if (wg == 0 && tid == 0) {
        amp_status s;
        s.T = stopped ? T : P.max_iter;
        s.nan_state = aborted ? -1 : (fixed != 0 ? 1 : 0);
        s.stopped = stopped;
        s.pad = 0;
        s.last_scalar[0] = s.last_scalar[1] = s.last_scalar[2] = s.last_scalar[3] = 0.f;
        *P.status = s;
    }
}

bool scamp_persist_eligible(const amp_dims* d, int ncu) {
    const int twoN = 2 * d->N, twon = 2 * d->n;
    const bool shape = (twoN == 128 && twon == 256) || (twoN == 256 && twon == 512) || (twoN == 256 && twon == 256);
    if (!shape || d->M > 64 || d->Lin > SMAXLIN || d->Lout > SMAXLIN || !is_pow2(d->N / d->M)) return false;
    if (ncu <= 0 || cdiv(d->B, SPB) > ncu) return false;
    return (size_t)slayout(d->N, d->n, d->L, d->Lin, d->Lout).total * 4 + 1024 <= 160 * 1024;
}

template <int NT1, int G1, int NT2, int G2, int KK>
static int spersist_launch_t(const ScampK& P, const Const64& c64, hipStream_t st) {
    const void* fn = (const void*)scamp_persist<NT1, G1, NT2, G2, KK>;
    const size_t lds = (size_t)slayout(P.N, P.n, P.L, P.Lin, P.Lout).total * 4;
    // the dynamic-LDS attribute and the occupancy query: once per instantiation and LDS size
    static size_t attr_lds = 0;
    static int per_cu = 0;
    if (attr_lds != lds) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("scamp_persist: hipFuncSetAttribute: %s", hipGetErrorString(e));
            return AMP_E_LAUNCH;
        }
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess) per_cu = 0;
        attr_lds = lds;
    }
    // plain launch after the co-residency check a cooperative launch would make; every barrier
    // spin is bounded (2 s) as the backstop
    if (per_cu < 1 || (long)per_cu * device_cu_count() < P.nwg) {
        set_error("scamp_persist: grid of %d workgroups cannot be co-resident (%d per CU x %d CUs)", P.nwg, per_cu,
                  device_cu_count());
        return AMP_E_LAUNCH;
    }
    hipLaunchKernelGGL((scamp_persist<NT1, G1, NT2, G2, KK>), dim3(P.nwg), dim3(256), lds, st, P, c64);
    AMP_LAUNCH_CHECK("scamp_persist");
    return AMP_OK;
}

template <int NT1, int G1, int NT2, int G2>
static int spersist_launch_s(const ScampK& P, const Const64& c64, hipStream_t st) {
    switch (P.c.K) {
    case 1: return spersist_launch_t<NT1, G1, NT2, G2, 1>(P, c64, st);
    case 2: return spersist_launch_t<NT1, G1, NT2, G2, 2>(P, c64, st);
    case 4: return spersist_launch_t<NT1, G1, NT2, G2, 4>(P, c64, st);
    case 8: return spersist_launch_t<NT1, G1, NT2, G2, 8>(P, c64, st);
    case 16: return spersist_launch_t<NT1, G1, NT2, G2, 16>(P, c64, st);
    default: return spersist_launch_t<NT1, G1, NT2, G2, 64>(P, c64, st);
    }
}

// NT1 = 2n / 64 column tiles per wave (GEMM1, K = 2N = 16 G1); NT2 = 2N / 64 (GEMM2, K = 2n)
int scamp_persist_launch(const ScampK& P, const Const64& c64, hipStream_t st) {
    const int twoN = 2 * P.N, twon = 2 * P.n;
    if (twoN == 128 && twon == 256) return spersist_launch_s<4, 8, 2, 16>(P, c64, st);
    if (twoN == 256 && twon == 512) return spersist_launch_s<8, 16, 4, 32>(P, c64, st);
    if (twoN == 256 && twon == 256) return spersist_launch_s<4, 16, 4, 16>(P, c64, st);
    set_error("scamp_persist: (2N, 2n) = (%d, %d) not supported", twoN, twon);
    return AMP_E_ARG;
}

}  // namespace amp
