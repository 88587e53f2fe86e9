// Split-K workgroup-pair microbenchmark (cfg4 GEMM shape).
// 256 workgroups x 8 waves, REPS iterations of the engine's two per-iteration GEMMs
// (C = A . X^T, complex, K = O = 256), A resident in LDS as bf16x3 planes:
//   MODE 0: the round-5 engine form — 16 trials per workgroup, every wave two complex column tiles
//           over the whole K (gemm_x3<2, 8>): the whole operator streams through every CU;
//   MODE 1: split-K pairs (amp_pair.h) — 32 trials per workgroup pair, each workgroup its K half,
//           each wave its partner's tile then its own (two row tiles per operator fragment), the
//           partner partials handed over as tagged granules;
//   MODE 2: MODE 1 without the hand-off (the pure GEMM time of the pair form);
//   MODE 3: MODE 1 with plain (L2-resident) granule stores — same-XCD pairs only;
//   MODE 4 / 5: the granule stores (write-through / plain) without the partner's read (store cost);
//   MODE 6 / 7: MODE 1 / 3 with the hand-off inside the own tile's GEMM (two operator groups in
//               flight; stores after the first groups' loads, the poll loads issued two groups early);
//   MODE 8: MODE 2 with two operator groups in flight; MODE 9 / 10: MODE 6 with the poll loads
//   issued after group 2 / 1 (MODE 6: after the last group's MFMAs); MODE 11: MODE 1 with 32 wait
//   states after each GEMM (an MFMA-result hazard probe); MODE 12 / 13: MODE 9's stores only / its
//   poll loads only (reading zeroed slots with tag 0: the load cost without the partner);
//   MODE 14 / 15: raw f32 partials (64 B per lane, write-through) and a per-wave flag behind a
//   vmcnt(0) drain after group 2 / 1 of the own tile's GEMM.
// Reports median cycles per iteration over the workgroups and the max error against float64.
// hipcc -O3 --offload-arch=gfx950 -o bin/pair tools/ubench/pair_ubench.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "pair_gemm.h"

using namespace amp;

constexpr int KC = 256, OC = 256, REPS = 20, NWG = 256, G = KC / 32;

template <int MODE>
__global__ __launch_bounds__(512, 1) void kpair(const float* __restrict__ A, const void* w1, const void* w2,
                                                void* xbuf, float* out, unsigned long long* cyc, unsigned* abortw,
                                                unsigned gen) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    unsigned short* sP = reinterpret_cast<unsigned short*>(lds);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wg = blockIdx.x;
    const int h = (wg >> 3) & 1, pr = ((wg >> 4) << 3) | (wg & 7);
    constexpr int ROWS = MODE == 0 ? 16 : 32, KL = MODE == 0 ? KC : KC / 2;
    const int ldx = KL;
    unsigned short* sP1 = sP + 6 * 16 * ldx;
    for (int e = tid; e < ROWS * (KL >> 3); e += 512) {
        const int row = e % ROWS, j0 = 8 * (e / ROWS);
        float re[8], im[8];
        for (int q = 0; q < 8; ++q) {
            const int k = (MODE == 0 ? 0 : 128 * h) + j0 + q;
            re[q] = A[(row * KC + k) * 2];
            im[q] = A[(row * KC + k) * 2 + 1];
        }
        x3_store8(row < 16 ? sP : sP1, ldx, row & 15, j0, re, im);
    }
    __syncthreads();
    f32x4 cr[2], ci[2];
    float sink = 0.f;
    const __amdgpu_buffer_rsrc_t xr = gran_rsrc(xbuf, 128u * 2 * 2 * 8 * PAIR_WAVE_BYTES);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; ++rep) {
        for (int gi = 0; gi < 2; ++gi) {
            const void* wq = gi ? w2 : w1;
            if constexpr (MODE == 0) {
                gemm_x3<2, G, 1, false>(sP, ldx, wq, wave * 2, cr, ci);
            } else {
                const unsigned tag = gen * 1000u + 2u * rep + gi + 1u;
                const int cp = 8 * (1 - h) + wave, co = 8 * h + wave;
                auto rsrc = [&](int ct) {
                    const int ctu = __builtin_amdgcn_readfirstlane(ct);
                    return __builtin_amdgcn_make_buffer_rsrc((char*)const_cast<void*>(wq) + (size_t)ctu * G * 6 * 1024,
                                                             (short)0, 0x7ffffff0, 0x00020000);
                };
                // slot of (pair, gemm, receiver half, wave)
                const int slot_to = (((pr * 2 + gi) * 2 + (1 - h)) * 8 + wave) * PAIR_WAVE_BYTES;
                const int slot_me = (((pr * 2 + gi) * 2 + h) * 8 + wave) * PAIR_WAVE_BYTES;
                f32x4 pr_[2], pi_[2];
                if constexpr (MODE >= 6) {
                    if constexpr (MODE >= 14) asm volatile("s_nop 15\n s_nop 15" ::: "memory");
                    constexpr int PG = (MODE == 9 || MODE == 13) ? 2 : MODE == 10 ? 1 : 3;   // poll-issue group
                    gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(cp), 4 * h, pr_, pi_);
                    u32x4 gg[PAIR_GRAN];
                    if constexpr (MODE == 14 || MODE == 15) {
                        // raw partials (64 B per lane, write-through) + a per-wave flag behind a drain
                        const int base_to = slot_to, base_me = slot_me;
                        auto put_raw = [&] {
                            const int o = __builtin_amdgcn_readfirstlane(base_to);
                            const int vo = lane * 16;
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pr_[0]), xr, vo, o, 16);
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pi_[0]), xr, vo, o + 1024, 16);
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pr_[1]), xr, vo, o + 2048, 16);
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pi_[1]), xr, vo, o + 3072, 16);
                        };
                        auto flag = [&] {
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            const int o = __builtin_amdgcn_readfirstlane(base_to);
                            if (lane == 0) __builtin_amdgcn_raw_buffer_store_b32(tag, xr, 0, o + 4096, 16);
                        };
                        gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci, put_raw,
                                         [&](int g) { if (g == (MODE == 14 ? 2 : 1)) flag(); });
                        asm volatile("s_nop 15\n s_nop 15" ::: "memory");
                        const int o = __builtin_amdgcn_readfirstlane(base_me);
                        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                        for (;;) {
                            const unsigned f = __builtin_amdgcn_raw_buffer_load_b32(xr, 0, o + 4096, 16);
                            if (__builtin_amdgcn_readfirstlane(f) == tag) break;
                            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { *abortw = 1u; break; }
                            __builtin_amdgcn_s_sleep(1);
                        }
                        const int vo = lane * 16;
                        const u32x4 d0 = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, o, 16);
                        const u32x4 d1 = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, o + 1024, 16);
                        const u32x4 d2 = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, o + 2048, 16);
                        const u32x4 d3 = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, o + 3072, 16);
                        cr[0] += __builtin_bit_cast(f32x4, d0); ci[0] += __builtin_bit_cast(f32x4, d1);
                        cr[1] += __builtin_bit_cast(f32x4, d2); ci[1] += __builtin_bit_cast(f32x4, d3);
                    } else if constexpr (MODE == 12) {   // the puts only
                        gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci,
                                         [&] { pair_put<16>(xr, slot_to, tag, pr_, pi_); });
                    } else if constexpr (MODE == 13) {   // the poll loads only (tag 0: the zeroed slots of pair 127)
                        gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci, NoHook(),
                                         [&](int g) { if (g == PG) pair_issue(xr, (((127 * 2 + gi) * 2 + h) * 8 + wave) * PAIR_WAVE_BYTES, gg); });
                        pair_take_add(xr, slot_me, 0u, abortw, gg, cr, ci);
                        sink += pr_[0][0] + pi_[1][3];
                    } else if constexpr (MODE == 8) {
                        sink += pr_[0][0] + pi_[1][3];
                        gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci);
                    } else {
                        gemm_x3_r2<4, 2>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci,
                                         [&] { pair_put<MODE == 7 ? 0 : 16>(xr, slot_to, tag, pr_, pi_); },
                                         [&](int g) { if (g == PG) pair_issue(xr, slot_me, gg); });
                        pair_take_add(xr, slot_me, tag, abortw, gg, cr, ci);
                    }
                } else {
                gemm_x3_r2<4, 1>(sP, sP1, ldx, rsrc(cp), 4 * h, pr_, pi_);
                if constexpr (MODE == 11 || MODE >= 14) asm volatile("s_nop 15\n s_nop 15" ::: "memory");
                if constexpr (MODE == 1 || MODE == 4 || MODE == 11) pair_put<16>(xr, slot_to, tag, pr_, pi_);
                else if constexpr (MODE == 3 || MODE == 5) pair_put<0>(xr, slot_to, tag, pr_, pi_);
                else sink += pr_[0][0] + pi_[1][3];
                gemm_x3_r2<4, 1>(sP, sP1, ldx, rsrc(co), 4 * h, cr, ci);
                if constexpr (MODE == 11) asm volatile("s_nop 15\n s_nop 15" ::: "memory");
                if constexpr (MODE == 1 || MODE == 3 || MODE == 11) pair_get_add(xr, slot_me, tag, abortw, cr, ci);
                }
            }
            __syncthreads();
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (wg == 0 || wg == 8) {   // pair 0's outputs of the last GEMM (w2)
        const int co = MODE == 0 ? 2 * wave : 8 * h + wave;
        for (int t = 0; t < (MODE == 0 ? 2 : 1); ++t)
            for (int rt = 0; rt < (MODE == 0 ? 1 : 2); ++rt)
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * rt + 4 * (lane >> 4) + r, o = 16 * (co + t) + (lane & 15);
                    const float vr = MODE == 0 ? cr[t][r] : cr[rt][r], vi = MODE == 0 ? ci[t][r] : ci[rt][r];
                    if (MODE == 0 && wg != 0) continue;
                    out[(row * OC + o) * 2] = vr;
                    out[(row * OC + o) * 2 + 1] = vi;
                }
    }
    if (sink == 12345.f) out[0] = sink;
    if (tid == 0) cyc[wg] = t1 - t0;
}

static unsigned short bf16_rn(float x) {
    unsigned u;
    memcpy(&u, &x, 4);
    const unsigned r = 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)((u + r) >> 16);
}
static float bf2f(unsigned short h) {
    unsigned u = (unsigned)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static void split3(float x, unsigned short p[3]) {
    p[0] = bf16_rn(x);
    const float r1 = x - bf2f(p[0]);
    p[1] = bf16_rn(r1);
    const float r2 = r1 - bf2f(p[1]);
    p[2] = bf16_rn(r2);
}

template <int MODE>
static void run(const float* dA, void* dW1, void* dW2, void* dX, unsigned* dAb, const std::vector<double>& ref) {
    float* dO;
    unsigned long long* dc;
    hipMalloc(&dO, 32 * OC * 2 * 4);
    hipMalloc(&dc, NWG * 8);
    hipMemset(dO, 0, 32 * OC * 2 * 4);
    const size_t lds = 6 * 32 * 128 * 2;
    hipFuncSetAttribute((const void*)kpair<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (unsigned i = 0; i < 4; ++i)
        hipLaunchKernelGGL((kpair<MODE>), dim3(NWG), dim3(512), lds, 0, dA, dW1, dW2, dX, dO, dc, dAb, i + 1);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(NWG, 0);
    hipMemcpy(c.data(), dc, NWG * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const int rows = MODE == 0 ? 16 : 32;
    std::vector<float> o(32 * OC * 2);
    hipMemcpy(o.data(), dO, o.size() * 4, hipMemcpyDeviceToHost);
    unsigned ab = 0;
    hipMemcpy(&ab, dAb, 4, hipMemcpyDeviceToHost);
    double e = 0, rms = 0, nrm = 0;
    for (int i = 0; i < rows * OC * 2; ++i) {
        e = std::max(e, fabs(o[i] - ref[i]));
        rms += (o[i] - ref[i]) * (o[i] - ref[i]);
        nrm = std::max(nrm, fabs(ref[i]));
    }
    rms = sqrt(rms / (rows * OC * 2));
    printf("MODE %d: cycles per iteration (2 GEMMs) median %.0f  p90 %.0f  max %.0f   max|err| %.3e rms %.3e (max|C| %.3f) abort %u\n",
           MODE, (double)c[NWG / 2] / REPS, (double)c[NWG * 9 / 10] / REPS, (double)c[NWG - 1] / REPS, e, rms, nrm, ab);
    hipFree(dO);
    hipFree(dc);
}

int main() {
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> A(32 * KC * 2), X(OC * KC * 2);
    for (auto& v : A) v = rnd();
    for (auto& v : X) v = rnd() * 0.0625f;
    std::vector<unsigned short> wp((size_t)(OC / 16) * G * 6 * 64 * 8);
    for (int o = 0; o < OC; ++o)
        for (int k = 0; k < KC; ++k) {
            unsigned short p[3], q[3];
            split3(X[(o * KC + k) * 2], p);
            split3(X[(o * KC + k) * 2 + 1], q);
            const int ct = o >> 4, g = k >> 5, kk = k & 31, lane = (o & 15) + 16 * (kk >> 3), j = kk & 7;
            for (int s = 0; s < 3; ++s) {
                wp[((((size_t)ct * G + g) * 6 + s) * 64 + lane) * 8 + j] = p[s];
                wp[((((size_t)ct * G + g) * 6 + 3 + s) * 64 + lane) * 8 + j] = q[s];
            }
        }
    std::vector<double> ref(32 * OC * 2);
    for (int r = 0; r < 32; ++r)
        for (int o = 0; o < OC; ++o) {
            double sr = 0, si = 0;
            for (int k = 0; k < KC; ++k) {
                const double ar = A[(r * KC + k) * 2], ai = A[(r * KC + k) * 2 + 1];
                const double xr = X[(o * KC + k) * 2], xi = X[(o * KC + k) * 2 + 1];
                sr += ar * xr - ai * xi;
                si += ar * xi + ai * xr;
            }
            ref[(r * OC + o) * 2] = sr;
            ref[(r * OC + o) * 2 + 1] = si;
        }
    float* dA;
    void *dW1, *dW2, *dX;
    unsigned* dAb;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dW1, wp.size() * 2);
    hipMalloc(&dW2, wp.size() * 2);
    const size_t xb = 128u * 2 * 2 * 8 * PAIR_WAVE_BYTES;
    hipMalloc(&dX, xb);
    hipMalloc(&dAb, 4);
    hipMemset(dX, 0, xb);
    hipMemset(dAb, 0, 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW1, wp.data(), wp.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW2, wp.data(), wp.size() * 2, hipMemcpyHostToDevice);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    if (ncu < NWG) {
        printf("needs %d CUs (one workgroup each), device has %d\n", NWG, ncu);
        return 1;
    }
    for (int it = 0; it < 2; ++it) {
        run<0>(dA, dW1, dW2, dX, dAb, ref);
        run<8>(dA, dW1, dW2, dX, dAb, ref);
        run<9>(dA, dW1, dW2, dX, dAb, ref);
        run<14>(dA, dW1, dW2, dX, dAb, ref);
        run<15>(dA, dW1, dW2, dX, dAb, ref);
    }
    return 0;
}
