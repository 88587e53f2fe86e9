// amp_scamp.h — SCAMP state shared by the launch engine (amp_scamp.hip) and the persistent
// engine (amp_scamp_persist.hip): parameter block, workspace carve, per-iteration record.
#pragma once

#include <algorithm>

#include "amp_decide.h"
#include "amp_denoise.h"
#include "amp_gemm.h"
#include "amp_host.h"

namespace amp {

// fp16x2 persistent GEMMs (amp_scamp_persist_kernel.h, H2): the operator A is packed as A 2^SH2_EX,
// so its entries must stay below 64 in magnitude (the channel's are ~CN(0, 1/Nr)).
constexpr int SH2_EX = 10;


constexpr int SRWG = 1024;
constexpr int SMAXLIN = 64;     // coupling blocks per trial handled in registers / LDS

struct alignas(16) ScampIter {
    int32_t stopped, T, fixed, fixed_all;
    // exact float64 fix-up of iteration T-1 pending (set by scamp_r, done by scamp_fix_sec and
    // scamp_fix_psi_fin, settled by the latter; scamp_fix_* and scamp_sxr* in the trial-sharded
    // stages): the exact batch max |xi| G, the float32 estimate's slack, and the
    // allclose count before the fix-up
    double G, slack;
    uint32_t notclose;
    int32_t active, pad[2];
};

struct ScampK {
    int B, N, n, L, M, Nt, Nr, Na, Lin, Lout, bn;
    int kapA, ncpA, kapB, ncpB;
    int nblk, max_iter;
    float sigma2;          // f32(noise_var) (scamp.py:51)
    const float* W;        // [Lout][Lin]
    const float* WA;       // [ncpA][kapA]  A xmmse
    const float* WAH;      // [ncpB][kapB]  A^H (z/phi)
    const float* y;        // [B][2n]
    float* z;              // [B][2n]
    float* s;              // [B][2n] z / phi_use
    float* phi;            // [2][B][Lout] ping-pong
    float* tau;            // [B][Lin] (per iteration)
    float* xmap;           // caller [B][2N]
    float* xm;             // caller [B][2N]
    float* psi0;           // caller's psi [B][Lin] (even iterations)
    float* psi1;           // workspace     (odd iterations)
    float* secmax;         // [B*L] per-section max logit (fast path)
    float* secabs;         // [B*L] per-section max |logit|
    Partial* parts;
    ScampIter* iters;
    unsigned* psi_nc;      // [max_iter][psi_nblk] allclose counts of scamp_psi (split tiles only)
    int psi_nblk, psi_split;
    amp_status* status;
    // persistent engine (amp_scamp_persist.hip)
    int nwg;               // ceil(B / 16) workgroups
    unsigned gen;          // launch generation: granule tags are gen * (max_iter + 1) + t + 1
    const float* Wq1;      // A    16x16x4-packed [2n][2N]
    const float* Wq2;      // A^H  16x16x4-packed [2N][2n]
    Partial* pparts;       // [max_iter][nwg] 32-B granule pairs
    double* pxch;          // [max_iter][nwg][4] rare-path exchange
    unsigned* pbar;        // [0] arrivals, [1] abort flag (zeroed by the prepare launch)
    int x3;                // persistent GEMMs on the bf16x3 engine (Wx1 / Wx2)
    const void* Wx1;       // A    X3-packed (x3_index, O = n, J = N)
    const void* Wx2;       // A^H  X3-packed (O = N, J = n)
    // launch engine, block-banded A (Lin > 1 or Lout > 1: the ISI / coupled channel): per column
    // tile of WA (128 wide) / WAH (bn wide) the reduction range holding its nonzero blocks
    const int* bandA;
    const int* bandB;
    // launch engine, bf16x3 tiles (amp_gemm_x3.h, lx3 = 1): WA / WAH hold the x3-packed operators
    // (x3_index), each GEMM's A rows split first into `lap` (six bf16 planes)
    int lx3, rows_pad;
    unsigned short* lap;
    XState* xs;            // trial-sharded exchange words (amp_scamp_run_sharded)
    // fused decision (amp_scamp_detect_count: decide_epilogue at the end of scamp_persist)
    int dec_on, ibits;
    const float2* xtrue;   // [B][N] transmitted x
    const long long* sym;  // [B*L] gray labels
    const long long* idx;  // [B*L] flat nonzero indices
    DecWG* dwg;            // per-workgroup records: [nwg] x 256 B of tagged granules (folded in the
                           // persistent kernel, amp_decide_fused.h dec_fold_gather)
    amp_counts* counts;    // out
    unsigned char* host_rec;   // optional page-locked host record (amp_vamp_decide_args.host_record)
    int fold_in;               // the persistent kernel folds the records itself (else vamp_decide_fold)
    unsigned long long* trace;   // diagnostic phase stamps (amp_scamp_persist_trace), else null
    // launch engine: rcnt[1] is scamp_fix_psi_fin's arrival counter (zeroed by scamp_init_kernel)
    unsigned* rcnt;
    Const c;
};

struct ScampWs {
    float *WA, *WAH, *z, *s, *phi, *tau, *psi1;
    float *secmax, *secabs;
    Partial* parts;
    ScampIter* iters;
    unsigned* psi_nc;
    float *Wq1, *Wq2, *Wx1, *Wx2;
    unsigned* pbar;
    Partial* pparts;
    double* pxch;
    int *bandA, *bandB;
    unsigned short* lap;
    XState* xs;
    DecWG* dwg;
    size_t bytes;
};

// the launch engine's bf16x3 tiles need whole 64-wide reduction groups and output tiles
inline bool scamp_lx3_shape(const amp_dims* d) { return d->N % 64 == 0 && d->n % 64 == 0; }

// 128 columns whenever a section fits (2M <= 128): twice the workgroups of a whole-coupling-
// block tile (cfg3: 256 instead of 128).  A tile that does not hold whole coupling blocks
// (2 Nt > BN) leaves psi to scamp_psi.
inline int scamp_bn(const amp_dims* d) { return section_bn(d); }
inline int scamp_psi_nblk(const amp_dims* d) { return std::max(1, std::min(cdiv(d->B * d->Lin, AMP_WG / 64), 2048)); }

inline void scamp_geometry(const amp_dims* d, ScampK& P) {
    P.B = d->B; P.N = d->N; P.n = d->n; P.L = d->L; P.M = d->M;
    P.Nt = d->Nt; P.Nr = d->Nr; P.Na = d->Na; P.Lin = d->Lin; P.Lout = d->Lout;
    P.bn = scamp_bn(d);
    P.kapA = round_up(2 * d->N, GBK); P.ncpA = round_up(2 * d->n, 128);
    P.kapB = round_up(2 * d->n, GBK); P.ncpB = round_up(2 * d->N, P.bn);
    P.nblk = cdiv(d->B, GBM) * (P.ncpB / P.bn);
}

inline ScampWs scamp_carve(const amp_dims* d, int max_iter, void* base) {
    ScampK P;
    scamp_geometry(d, P);
    Carve cv(base);
    ScampWs w;
    w.WA = cv.take<float>((size_t)P.ncpA * P.kapA);
    w.WAH = cv.take<float>((size_t)P.ncpB * P.kapB);
    w.z = cv.take<float>((size_t)d->B * 2 * d->n);
    w.s = cv.take<float>((size_t)d->B * 2 * d->n);
    w.phi = cv.take<float>((size_t)2 * d->B * d->Lout);
    w.tau = cv.take<float>((size_t)d->B * d->Lin);
    w.psi1 = cv.take<float>((size_t)d->B * d->Lin);
    w.secmax = cv.take<float>((size_t)d->B * d->L);
    w.secabs = cv.take<float>((size_t)d->B * d->L);
    w.parts = cv.take<Partial>((size_t)max_iter * P.nblk);
    w.iters = cv.take<ScampIter>((size_t)max_iter + 1);
    w.psi_nc = cv.take<unsigned>((size_t)max_iter * scamp_psi_nblk(d));
    const int nwg = cdiv(d->B, 16);
    w.Wq1 = cv.take<float>((size_t)2 * d->n * 2 * d->N);
    w.Wq2 = cv.take<float>((size_t)2 * d->N * 2 * d->n);
    w.Wx1 = cv.take<float>((size_t)3 * d->n * d->N);    // 6 bf16 per complex entry
    w.Wx2 = cv.take<float>((size_t)3 * d->N * d->n);
    w.pxch = cv.take<double>((size_t)max_iter * nwg * 4);
    w.pbar = cv.take<unsigned>(64);
    w.pparts = cv.take<Partial>((size_t)max_iter * nwg);
    w.bandA = cv.take<int>((size_t)2 * (P.ncpA / 128));
    w.bandB = cv.take<int>((size_t)2 * (P.ncpB / P.bn));
    w.xs = cv.take<XState>(1);
    w.dwg = cv.take<DecWG>((size_t)2 * nwg);   // 256 B of granules per workgroup
    w.lap = scamp_lx3_shape(d) ? cv.take<unsigned short>((size_t)6 * round_up(d->B, GBM) * std::max(d->N, d->n))
                               : nullptr;
    w.bytes = cv.off;
    return w;
}

__device__ __forceinline__ float* spsi(const ScampK& P, int t) { return (t & 1) ? P.psi1 : P.psi0; }
__device__ __forceinline__ float* sphi(const ScampK& P, int t) { return P.phi + (size_t)(t & 1) * P.B * P.Lout; }

// gamma[lo] = (W psi)[lo] / Lc (scamp.py:45), float32 as torch's [Lout x Lin] @ [Lin] product
__device__ __forceinline__ float scamp_gamma(const ScampK& P, const float* psi_row, int lo) {
    float g = 0.f;
    for (int lc = 0; lc < P.Lin; ++lc) g += P.W[lo * P.Lin + lc] * psi_row[lc];
    return g / (float)P.Lin;
}

bool scamp_persist_eligible(const amp_dims* d, int ncu);
bool scamp_persist_x3_fits(const amp_dims* d);
int scamp_persist_launch(const ScampK& P, const DecConst& dc, hipStream_t st);

}  // namespace amp
