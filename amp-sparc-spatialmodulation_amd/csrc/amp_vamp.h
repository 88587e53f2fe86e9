// amp_vamp.h — VAMP state shared by the launch-per-kernel engine (amp_vamp.hip) and the
// persistent engine (amp_vamp_persist.hip): parameter block, workspace carve, and the batch
// scalars of one iteration (vamp.py:66-82).
#pragma once

#include "amp_decide.h"
#include "amp_denoise.h"
#include "amp_gemm.h"
#include "amp_host.h"

namespace amp {

constexpr int RWG = 1024;   // threads of the reduction / fix-up workgroup
constexpr int PBAR_EPOCH = 64;                 // first per-epoch barrier counter in pbar
constexpr int PBAR_WORDS = PBAR_EPOCH + 256;   // one counter per epoch (E <= 256 workgroups)

struct VampK {
    int B, N, n, k, L, M;
    int Bmean;          // the batch var.mean() runs over (vamp.py:85): B, or the whole batch when sharded
    int kap0, ncp0, kap1, ncp1, kap2, ncp2, bn2;
    int nblk2, max_iter;
    double noise_var, sparsity;
    const float* Wt0;
    const float* Wt1;
    const float* Wt2;
    const float* s;     // singular values (f32 [k])
    float* s2;          // s**2 (vamp.py:17)
    float* ytil;        // [B][2k]
    float* w;           // [B][2k]
    float* r;           // [B][2N]  (caller's r)
    float* xm;          // [B][2N]  (caller's xmmse)
    float* var0;        // [B][N] caller's var: var of even iterations
    float* var1;        // [B][N] workspace:    var of odd iterations
    float* secmax;      // [B*L] per-section max logit (fast path, natural units)
    float* secabs;      // [B*L] per-section max |logit|
    Partial* parts;     // [max_iter][nblk2]
    VampIter* iters;    // [max_iter + 1]: iters[t] drives iteration t
    amp_status* status;
    // persistent engine
    int nwg;            // workgroups: E * wpe
    int E, wpe;         // side-by-side epochs (independent batches of B trials, one channel) and
                        // workgroups per epoch (ceil(B / PBM)); E = 1 outside amp_vamp_detect_count_epochs
    const float* Wq1;   // Vh   16x16x4-packed [2k][2N]
    const float* Wq2;   // V    16x16x4-packed [2N][2k]
    Partial* pparts;    // [max_iter][nwg] 32-B granule pairs (amp_vamp_persist.hip), right after pbar
    double* pxch;       // [max_iter][nwg][4] rare-path exchange
    unsigned* pbar;     // [0] arrivals, [1] abort flag, [PBAR_EPOCH + e] epoch e's arrivals
                        // (PBAR_WORDS words zeroed by the prepare launch)
    unsigned gen;       // launch generation: granule tags are gen * (max_iter + 1) + t + 1
    int ytil_in_kernel; // y~ = (s Uh) y computed by the persistent kernel itself (n == 2N)
    const float* Wq0;   // s Uh 16x16x4-packed [2k][2n] (ytil_in_kernel)
    const float* y;     // [B][2n] received signal (ytil_in_kernel)
    // fused decision + counters (amp_vamp_detect_count), persistent engine only
    int dec_on, ibits, Na, Lin;
    const float2* xtrue;        // [B][N] transmitted x
    const long long* sym;       // [B*L] gray labels
    const long long* idx;       // [B*L] flat nonzero indices
    DecWG* dwg;                 // per-workgroup records: [nwg] x 256 B of tagged granules (the
                                // persistent engine folds them itself, amp_decide_fused.h)
    unsigned char* host_rec;    // optional page-locked host record (amp_vamp_decide_args.host_record)
    int fold_in;                // the persistent kernel folds the records itself (else vamp_decide_fold)
    amp_counts* counts;         // out
    unsigned long long* trace;   // diagnostic phase stamps (amp_vamp_persist_trace), else null
    int x3;                      // persistent engine GEMMs: 0 f32 MFMA, 1 bf16x3, 2 fp16x2 (Wx1 / Wx2)
    const void* Wx1;             // Vh X3- / H2-packed (x3_index / h2_index, O = k, J = N)
    const void* Wx2;             // V  X3- / H2-packed (O = N, J = k)
    XState* xs;                  // trial-sharded exchange words (amp_vamp_run_sharded)
    float* dump;                 // diagnostic per-iteration state dump (amp_vamp_debug_dump), else null
    // side-by-side epochs with one channel per epoch (amp_vamp_detect_count_epochs_ch): epoch e's
    // split-precision operators at Wx1 / Wx2 + e * wch bytes and its singular values at s + e * sch
    // (0, 0: one channel shared by every epoch)
    long long wch;
    int sch;
    // trial sharding of one batch over several persistent grids (amp_vamp_detect_count_shard):
    // this grid's first workgroup in the shared exchange, the exchange's workgroups, and its first
    // trial (0, nwg, 0 for a whole batch or side-by-side epochs)
    int wg_off, nwg_x, row_off;
    Const c;
};

struct VampWs {
    float *Wt0, *Wt1, *Wt2, *s2, *ytil, *w, *var1;
    float *secmax, *secabs;
    Partial* parts;
    VampIter* iters;
    float *Wq0, *Wq1, *Wq2;
    float *Wx1, *Wx2;
    Partial* pparts;
    double* pxch;
    unsigned* pbar;
    DecWG* dwg;
    XState* xs;
    size_t bytes;
};

static void vamp_geometry(const amp_dims* d, int k, VampK& P) {
    P.Na = d->Na; P.Lin = d->Lin;
    P.B = d->B; P.N = d->N; P.n = d->n; P.k = k; P.L = d->L; P.M = d->M;
    P.kap0 = round_up(2 * d->n, GBK); P.ncp0 = round_up(2 * k, 128);
    P.kap1 = round_up(2 * d->N, GBK); P.ncp1 = round_up(2 * k, 128);
    P.bn2 = section_bn(d);
    P.kap2 = round_up(2 * k, GBK); P.ncp2 = round_up(2 * d->N, P.bn2);
    P.nblk2 = cdiv(d->B, GBM) * (P.ncp2 / P.bn2);
}

// chans: channel-dependent operator sets (Wq0 / Wx1 / Wx2) to hold — one per epoch for side-by-side
// epochs with a channel each (amp_vamp_epochs_workspace_bytes carves `epochs` of them).
static VampWs vamp_carve(const amp_dims* d, int k, int max_iter, void* base, int chans = 1) {
    VampK P;
    vamp_geometry(d, k, P);
    Carve cv(base);
    VampWs w;
    w.Wt0 = cv.take<float>((size_t)P.ncp0 * P.kap0);
    w.Wt1 = cv.take<float>((size_t)P.ncp1 * P.kap1);
    w.Wt2 = cv.take<float>((size_t)P.ncp2 * P.kap2);
    w.s2 = cv.take<float>((size_t)k);
    w.ytil = cv.take<float>((size_t)d->B * 2 * k);
    w.w = cv.take<float>((size_t)d->B * 2 * k);
    w.var1 = cv.take<float>((size_t)d->B * d->N);
    w.secmax = cv.take<float>((size_t)d->B * d->L);
    w.secabs = cv.take<float>((size_t)d->B * d->L);
    w.parts = cv.take<Partial>((size_t)max_iter * P.nblk2);
    w.iters = cv.take<VampIter>((size_t)max_iter + 1);
    const int nwg = cdiv(d->B, 16);
    w.Wq0 = cv.take<float>((size_t)2 * k * 2 * d->n * chans);
    w.Wq1 = cv.take<float>((size_t)2 * k * 2 * d->N);
    w.Wq2 = cv.take<float>((size_t)2 * d->N * 2 * k);
    w.Wx1 = cv.take<float>((size_t)3 * k * d->N * chans);      // 6 bf16 per complex entry
    w.Wx2 = cv.take<float>((size_t)3 * k * d->N * chans);
    w.pxch = cv.take<double>((size_t)max_iter * nwg * 4);
    w.pbar = cv.take<unsigned>(PBAR_WORDS);                  // barrier words (zeroed per launch); the
    w.pparts = cv.take<Partial>((size_t)max_iter * nwg);     // granules carry generation tags
    w.dwg = cv.take<DecWG>((size_t)2 * nwg);              // 256 B of granules per workgroup
    w.xs = cv.take<XState>(1);
    w.bytes = cv.off;
    return w;
}

__device__ __forceinline__ float* var_buf(const VampK& P, int t) { return (t & 1) ? P.var1 : P.var0; }

// ---------------------------------------------------------------------------
// Batch scalars of iteration t (vamp.py:66-82) from sigma2_tilde; t == 0 uses the
// Tracker's Python-float sigma2_tilde (vamp.py:26).  Called by one workgroup.
// ---------------------------------------------------------------------------
// This lane's s^2 (vamp.py:17) at i = lane + 64 j, held in registers by the persistent engine for
// the whole forward (k <= 256), so the per-iteration LMMSE sum reads no memory.
struct S2Lane {
    float v[4];
};
__device__ inline S2Lane s2_lane(const VampK& P, const float* s) {
    S2Lane a;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = lane + 64 * j;
        const float x = s[min(i, P.k - 1)];   // unconditional load (no branch: amp_gemm.h ALoadPlain)
        a.v[j] = i < P.k ? x * x : 0.f;
    }
    return a;
}

__device__ inline void vamp_lmmse_scalars(const VampK& P, bool first, double s2t64, float s2t, float* lds, VampIter& it,
                                          const S2Lane* sl = nullptr) {
    const float vr = first ? (float)(P.noise_var / s2t64) : (1.0f / s2t) * (float)P.noise_var;   // vamp.py:66
    // every wave sums all k terms in the same order (no LDS round trip, no barrier): the
    // workgroup's waves hold bit-identical scalars
    (void)lds;
    double ss = 0.0;
    if (sl) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (lane + 64 * j < P.k) ss += (double)(1.0f / (sl->v[j] + vr));                        // vamp.py:17, 68
    } else {
        for (int i = threadIdx.x & 63; i < P.k; i += 64) ss += (double)(1.0f / (P.s[i] * P.s[i] + vr));  // vamp.py:17, 68
    }
    ss = group_sum(ss, 64);
    const float varL = (float)(ss / (double)P.k) * (float)P.noise_var;                         // vamp.py:71
    const double eta = (double)P.k / (double)P.N;                                              // vamp.py:28
    float xtv, s2t32;
    if (first) {
        xtv = (float)eta * varL + (float)((1.0 - eta) * s2t64);                                // vamp.py:73
        s2t32 = (float)s2t64;
    } else {
        xtv = (float)eta * varL + (float)(1.0 - eta) * s2t;
        s2t32 = s2t;
    }
    const float alpha = clampf_t(xtv / s2t32, AMP_VAR_RATIO_MIN, 1.0f - AMP_VAR_RATIO_MIN);    // vamp.py:75-77
    const float sigma2 = clampf_t((alpha / (1.0f - alpha)) * s2t32, AMP_VAR_MIN, AMP_VAR_MAX);  // vamp.py:80-82
    it.vr = vr;
    it.alpha = alpha;
    it.inv1ma = 1.0f / (1.0f - alpha);
    it.sigma2 = sigma2;
    it.inv_sigma2 = 1.0f / sigma2;
    it.s2t = s2t32;
}

// The record that drives iteration 0 (vamp.py:22-26, 66-82 with the Tracker's Python-float
// sigma2_tilde).  Called uniformly by every thread of one workgroup.
__device__ inline VampIter vamp_first_iter(const VampK& P, float* lds, const S2Lane* sl = nullptr) {
    VampIter it;
    it.stopped = 0; it.T = 0; it.fixed = 0; it.fixed_all = 0; it.G = 0.0;
    it.pad1[0] = it.pad1[1] = it.pad1[2] = 0.f;
    it.dxdr_prev = 0.f;   // r~ = (xmmse - 0 * r) * 1 = sparsity at t = 0 (vamp.py:25)
    it.ns_prev = 1.f;
    const double p = P.sparsity;
    vamp_lmmse_scalars(P, true, p * p * (1 - p) + (1 - p) * (1 - p) * p, 0.f, lds, it, sl);   // vamp.py:26
    return it;
}

// The record that drives iteration t+1, from the reduced partials of iteration t: the stop
// record when allclose held (vamp.py:185-186), else the scalars of vamp.py:85-94 and 66-82.
// Called uniformly by every thread of one workgroup (vamp_lmmse_scalars reduces over k).
__device__ inline VampIter vamp_advance(const VampK& P, const VampIter& cur, const PartAcc& pa, int fixed, int t,
                                        float* lds, const S2Lane* sl = nullptr) {
    VampIter nx;
    nx.stopped = 0; nx.T = 0; nx.fixed = fixed; nx.fixed_all = (fixed < 0) ? 1 : 0; nx.G = pa.maxabs;
    nx.pad1[0] = nx.pad1[1] = nx.pad1[2] = 0.f;
    if (pa.notclose == 0) {                                              // vamp.py:185-186
        nx = cur;
        nx.stopped = 1;
        nx.T = t + 1;
        nx.fixed = fixed;
    } else {
        // var.mean() (vamp.py:85): float64 sum of the float32 values, NaN / inf propagate
        const float mean = (float)(pa.sumvar / ((double)P.Bmean * (double)P.N));
        const float dxdr = clampf_t(mean / cur.sigma2, AMP_VAR_RATIO_MIN, 1.0f - AMP_VAR_RATIO_MIN);  // vamp.py:85-87
        const float ns = 1.0f / (1.0f - dxdr);                                                        // vamp.py:89
        const float s2t = clampf_t((cur.sigma2 * dxdr) * ns, AMP_VAR_MIN, AMP_VAR_MAX);              // vamp.py:92-94
        nx.dxdr_prev = dxdr;
        nx.ns_prev = ns;
        vamp_lmmse_scalars(P, false, 0.0, s2t, lds, nx, sl);
    }
    return nx;
}

__device__ inline amp_status vamp_make_status(const VampK& P, const VampIter& cur, const VampIter& nx, int fixed) {
    amp_status s;
    s.T = nx.stopped ? nx.T : P.max_iter;
    s.nan_state = fixed != 0 ? 1 : 0;
    s.stopped = nx.stopped;
    s.gemm = P.x3 + 1;   // x3: 0 f32, 1 bf16x3, 2 fp16x2, 3 int8x4 (the launch engine: 0)
    s.last_scalar[0] = cur.s2t; s.last_scalar[1] = cur.alpha; s.last_scalar[2] = cur.sigma2;
    s.last_scalar[3] = nx.stopped ? cur.dxdr_prev : nx.dxdr_prev;
    return s;
}

// ---- persistent engine (amp_vamp_persist.hip) ----
// Denoiser policy over the LDS-resident rows of one persistent workgroup (vamp.py:84, 185).
struct PDenoisePolicy {
    const float* r;
    float* x;
    float* vnew;
    const float* vprev;
    float* sm;
    float* sa;
    int ldr, M, lspr, N;   // sections per row = 1 << lspr (N, M powers of two)
    float inv;
    __device__ __forceinline__ void load(int sec, int m, float& rr, float& ri, float& it) const {
        const int row = sec >> lspr, sj = sec & ((1 << lspr) - 1);
        const float2 v = *reinterpret_cast<const float2*>(r + row * ldr + 2 * (sj * M + m));
        rr = v.x; ri = v.y; it = inv;
    }
    __device__ __forceinline__ void store(int sec, int m, float xr, float xi, float var, PartAcc& pa) const {
        const int row = sec >> lspr, sj = sec & ((1 << lspr) - 1);
        *reinterpret_cast<float2*>(x + row * ldr + 2 * (sj * M + m)) = make_float2(xr, xi);
        const int vo = row * N + sj * M + m;
        vnew[vo] = var;
        pa.sumvar += (double)var;
        pa.notclose += torch_close(var, vprev[vo]) ? 0u : 1u;     // vamp.py:185
    }
    __device__ __forceinline__ void section(int sec, float smax, float sabs) const {
        sm[sec] = smax;
        sa[sec] = sabs;
    }
    float* dbg = nullptr;   // diagnostic: [16][2N] ze (columns < N) and vs (columns >= N), else null
};
__device__ __forceinline__ void den_debug(const PDenoisePolicy& p, int sec, int m, float ze, float vs) {
    if (p.dbg) {
        const int row = sec >> p.lspr, sj = sec & ((1 << p.lspr) - 1);
        p.dbg[row * 2 * p.N + sj * p.M + m] = ze;
        p.dbg[row * 2 * p.N + p.N + sj * p.M + m] = vs;
    }
}

constexpr int PBM = 16;   // trials per workgroup

bool vamp_persist_eligible(const amp_dims* d, int k, int ncu, int epochs = 1, int gemm = AMP_GEMM_AUTO);
int vamp_persist_max_epochs(const amp_dims* d, int k, int ncu, int gemm = AMP_GEMM_AUTO);
int vamp_persist_wg_per_cu(const amp_dims* d, int k, int gemm);   // resident workgroups per CU of the launch
int vamp_gemm_select(const amp_dims* d, int k, int gemm);   // 0 f32, 1 bf16x3, 2 fp16x2 (amp_vamp.hip)
bool vamp_persist_x3_fits(int N, int k, int L);
bool vamp_persist_ytil_in_kernel(const VampK& P);
bool vamp_persist_ytil_h2(const VampK& P);
int vamp_persist_launch(const VampK& P, const Const64& c64, const DecConst& dc, hipStream_t st, int ncu);
int device_cu_count();
float* debug_dump_ptr();   // amp_vamp_debug_dump's buffer (null: off)
bool gemm_f32_requested();   // AMP_VAMP_GEMM=f32 (amp_vamp.hip)
bool persist_wg2();   // AMP_PERSIST_WG2: two workgroups per CU at N = 64 (amp_vamp_persist.hip)

}  // namespace amp
