// amp_host.h — host-side helpers shared by the C entry points.
#pragma once

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <algorithm>
#include <stdlib.h>

#include "amp_common.h"

namespace amp {

void set_error(const char* fmt, ...);

#define AMP_REQUIRE(cond, ...)                      \
    do {                                            \
        if (!(cond)) {                              \
            ::amp::set_error(__VA_ARGS__);          \
            return AMP_E_ARG;                       \
        }                                           \
    } while (0)

#define AMP_LAUNCH_CHECK(what)                                                          \
    do {                                                                                \
        hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) {                                                         \
            ::amp::set_error("%s: %s", what, hipGetErrorString(e_));                    \
            return AMP_E_LAUNCH;                                                        \
        }                                                                               \
    } while (0)

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
inline int round_up(int v, int a) { return (v + a - 1) / a * a; }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline bool is_pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

// Bump allocator used twice: once with base == nullptr to size the workspace, once to carve it.
struct Carve {
    char* base;
    size_t off = 0;
    explicit Carve(void* b) : base((char*)b) {}
    template <typename T>
    T* take(size_t count) {
        off = align_up(off, 256);
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += count * sizeof(T);
        return p;
    }
};

// Diagnostic switches of the A/B tools (tools/*.sh, tools/*_bench.py): read from the environment
// only by a diagnostic build (`make DIAG=1` -> lib_diag/libampsparc_diag.so, loaded through
// AMP_LIB_PATH).  The shipped library ignores them, so no environment variable changes what the
// product computes (the GEMM arithmetic is an argument of the ABI and is reported back in
// amp_status.gemm).
inline const char* diag_env(const char* name) {
#if defined(AMP_DIAG_ENV) && AMP_DIAG_ENV
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// An engine form that only the A/B tools select (four waves at N = 256, one workgroup per CU at
// N = 64): instantiated in the diagnostic build only, so the shipped library does not carry it.
#if defined(AMP_DIAG_ENV) && AMP_DIAG_ENV
#define AMP_DIAG_ONLY(...) (__VA_ARGS__)
#else
#define AMP_DIAG_ONLY(...) (set_error("%s: an A/B form of the diagnostic build (make DIAG=1)", __func__), AMP_E_ARG)
#endif

// The product-grid form of the denoiser (amp_denoise.h) applies when the float32 points take
// R distinct real and R distinct imaginary values with K = R^2 (R = 2, 4, 8), the grid's four
// corners are in the table and the multiplicities follow a pattern the kernels know (every
// point once, or the reference's 16-QAM table).  QPSK, the reference's
// 16-QAM table (config.py:112: -1+3j twice, 1-3j missing) and square 64-QAM qualify; PSK and the
// real alphabets keep the direct form.  AMP_GRID_DENOISER=0 disables it (A/B runs).
inline bool grid_denoiser_enabled() {
    static const bool on = [] {
        const char* e = diag_env("AMP_GRID_DENOISER");
        return !(e && e[0] == '0');
    }();
    return on;
}

inline void grid_decompose(Const& k) {
    k.grid = 0;
    k.gfull = 0;
    for (int i = 0; i < 8; ++i) k.gre[i] = k.gim[i] = 0.f;
    if (!grid_denoiser_enabled()) return;
    float re[8], im[8];
    int nr = 0, ni = 0;
    for (int p = 0; p < k.K; ++p) {
        int a = 0, b = 0;
        while (a < nr && re[a] != k.re[p]) ++a;
        while (b < ni && im[b] != k.im[p]) ++b;
        if (a == nr) { if (nr == 8) return; re[nr++] = k.re[p]; }
        if (b == ni) { if (ni == 8) return; im[ni++] = k.im[p]; }
    }
    const int R = nr;
    if (ni != R || !(R == 2 || R == 4 || R == 8) || R * R != k.K) return;
    std::sort(re, re + R);
    std::sort(im, im + R);
    int cnt[8][8] = {};
    for (int p = 0; p < k.K; ++p) {
        const int a = (int)(std::find(re, re + R, k.re[p]) - re), b = (int)(std::find(im, im + R, k.im[p]) - im);
        if (++cnt[a][b] > 2) return;
    }
    if (!cnt[0][0] || !cnt[0][R - 1] || !cnt[R - 1][0] || !cnt[R - 1][R - 1]) return;
    bool full = true;
    for (int a = 0; a < R; ++a)
        for (int b = 0; b < R; ++b) full &= cnt[a][b] == 1;
    int pat = full ? 1 : 0;                       // GRID_FULL (amp_denoise.h)
    if (!full && R == 4) {
        // GRID_REF16: config.py:112 on the sorted grid (-1+3j twice, 1-3j missing)
        bool ref = true;
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                ref &= cnt[a][b] == ((a == 1 && b == 3) ? 2 : (a == 2 && b == 0) ? 0 : 1);
        if (ref) pat = 2;
    }
    if (!pat) return;
    for (int a = 0; a < R; ++a) { k.gre[a] = re[a]; k.gim[a] = im[a]; }
    k.grid = R;
    k.gfull = pat;
}

inline Const to_const(const amp_constellation* c) {
    Const k;
    k.K = c->K;
    for (int i = 0; i < AMP_MAX_K; ++i) {
        const bool v = i < c->K;
        k.re[i] = v ? c->re[i] : 0.f;
        k.im[i] = v ? c->im[i] : 0.f;
    }
    grid_decompose(k);
    return k;
}

inline Const64 to_const64(const amp_constellation* c) {
    Const64 k;
    k.K = c->K;
    k.real_alpha = 1;
    for (int i = 0; i < AMP_MAX_K; ++i) {
        const bool v = i < c->K;
        k.re[i] = v ? c->re64[i] : 0.0;
        k.im[i] = v ? c->im64[i] : 0.0;
        if (v && c->im64[i] != 0.0) k.real_alpha = 0;
    }
    return k;
}

// Batch-global values of one trial-sharded iteration (amp_vamp_run_sharded, amp_bamp_run_sharded):
// each stage's float64 words are all-reduced across the ranks by the registered hook between
// launches.
struct XState {
    double sum[2];    // SUM: sum var (VAMP, vamp.py:85), not-close count (vamp.py:185, bamp.py:140)
    double mx[2];     // MAX: max|xi| (NaN -> +inf), -min section max (vamp.py:112, bamp.py:70)
    double gmax[2];   // MAX: exact float64 max|xi| over the candidate sections (rare path); [1] pad
    double fix[4];    // SUM: rare-path var delta, not-close delta, recomputed sections; [3] pad
    int mode;         // 2: this iteration takes the rare path (xr3 / xr4 act), else 0
    int pad[3];
};

// The registered amp_allreduce_fn (amp_set_allreduce_hook, amp_weights.hip): all-reduce `count`
// float64 words at `buf` in place on `st` (op: AMP_ALLREDUCE_SUM / MAX).
bool allreduce_hook_set();
int call_allreduce_hook(double* buf, int count, int op, hipStream_t st);
int hook_failure(const char* what);   // sets the error text, returns AMP_E_LAUNCH

int check_dims(const amp_dims* d, const amp_constellation* c, bool tiled = true);
int device_cu_count();   // compute units of the current device (cached)
// amp_stream_create_cu_range's registry (amp_weights.hip): the CU range of a stream it made, and the
// claim of a range by one grid of a shard generation on an exchange buffer (false: the range
// overlaps one already claimed for that buffer and generation)
bool cu_range_of(hipStream_t st, int* cu0, int* cu1);
bool shard_claim_range(const void* xbuf, unsigned gen, int cu0, int cu1);
void shard_forget(const void* xbuf);   // amp_vamp_shard_reset: a new forward on this buffer

// Launch path of the persistent (grid-synchronising) engines: a plain launch after the
// co-residency check (default), or hipLaunchCooperativeKernel (AMP_PERSIST_LAUNCH=coop).
inline bool persist_coop() {
    static const bool c = [] {
        const char* e = getenv("AMP_PERSIST_LAUNCH");
        return e && e[0] == 'c';
    }();
    return c;
}

// One persistent grid: nwg workgroups of `threads`, `lds` bytes of dynamic LDS, kernel
// arguments `args` (hipLaunchCooperativeKernel's array form, also used for the plain launch
// through hipLaunchKernel).  per_cu: resident workgroups per CU from the occupancy query.
inline int persist_grid_launch(const char* what, const void* fn, int nwg, int threads, size_t lds, int per_cu,
                               void** args, hipStream_t st) {
    if (per_cu < 1 || (long)per_cu * device_cu_count() < nwg) {
        set_error("%s: grid of %d workgroups cannot be co-resident (%d per CU x %d CUs)", what, nwg, per_cu,
                  device_cu_count());
        return AMP_E_LAUNCH;
    }
    const hipError_t e = persist_coop()
        ? hipLaunchCooperativeKernel(fn, dim3(nwg), dim3(threads), args, (unsigned)lds, st)
        : hipLaunchKernel(fn, dim3(nwg), dim3(threads), args, lds, st);
    if (e != hipSuccess) {
        set_error("%s: %s launch (%d x %d, %zu B LDS): %s", what, persist_coop() ? "cooperative" : "plain", nwg,
                  threads, lds, hipGetErrorString(e));
        return AMP_E_LAUNCH;
    }
    return AMP_OK;
}

// Column tile width of the section-fused GEMMs: a multiple of 2M so no section straddles
// two workgroups.
// AMP_SECTION_BN=256: the wide column tile also where sections fit the narrow one (A/B runs)
inline bool section_bn_wide_env() {
    static const bool v = [] {
        const char* e = diag_env("AMP_SECTION_BN");
        return e && atoi(e) == 256;
    }();
    return v;
}
inline int section_bn(const amp_dims* d) { return (2 * d->M <= 128 && !section_bn_wide_env()) ? 128 : 256; }

// Expanded-weight builders (amp_weights.hip)
enum { WPACK_NONE = 0, WPACK32 = 1, WPACK16 = 2, WPACKX3 = 3, WPACKH2 = 4, WPACKH2_ABS2 = 5, WPACKI8 = 6, WPACKX3_ABS2 = 7 };
// X3 / H2: bf16x3 / fp16x2 planes of X, H2_ABS2: fp16x2 planes of the real |X|^2 (h2r_index),
// I8: int8x4 digit planes of X with per-column exponents (i8_index); kap = J, ncp = O
int build_cweight(const float2* src, long so, long sj, int conj, const float* rowscale, int O, int J,
                  float* wt, int kap, int ncp, hipStream_t st, int packed = WPACK32);
// One job of build_cweights: the expanded weight of X[o][j] = rowscale_o *
// (conj ? conj : id)(src[o * so + j * sj]), o < O, j < J, [ncp][kap] in layout `packed`.
struct CWeightJob {
    const float2* src;
    long so, sj;
    int conj;
    const float* rowscale;
    int O, J;
    float* wt;
    int kap, ncp;
    int packed;
    int ex = 14;        // WPACKH2: the operator's scale exponent (amp_persist.h H2_EX; SCAMP: SH2_EX)
};
// Up to CW_MAX_JOBS jobs in ONE launch (blockIdx.y = job; the side-by-side epochs with a channel
// each build three per epoch); the same launch zeroes `nzero` words at `zero` (or none).
constexpr int CW_MAX_JOBS = 24;

// The persistent engines fold the fused decision's per-workgroup counter records inside their own
// launch and write the host record themselves (amp_decide_fused.h); a diagnostic build with
// AMP_FOLD_LAUNCH=1 keeps the separate vamp_decide_fold launch (A/B runs; round 5: ~2 us per step
// slower).
inline bool fold_in_kernel() {
    const char* e = diag_env("AMP_FOLD_LAUNCH");
    return !(e && e[0] == '1');
}
int build_cweights(const CWeightJob* jobs, int njobs, unsigned* zero, int nzero, hipStream_t st);
int build_abs2_weight(const float2* src, long so, long sj, int O, int J, float* wt, int kap, int ncp,
                      hipStream_t st);
// For each BN-column tile of an MFMA-packed [ncp][kap] weight: the reduction range [kb, ke)
// (multiples of GBK) that holds all its nonzero entries -> band[2 c], band[2 c + 1] (kb = ke when
// the tile is all zero).  One pass over the weight (amp_weights.hip).
int weight_kband(const float* wp, int kap, int ncp, int BN, int* band, hipStream_t st);
int h2_kband(const void* wq, int PL, int G, int tpt, int ntiles, int n16, int* band, hipStream_t st);

// Grid of the launch engines' rare-path fix-up launches (grid-stride over `work` sections, one
// count slot per workgroup within the iteration's nblk partial slots): at most two workgroups per
// CU, since the launch runs every iteration and is a no-op unless a fix-up is pending, when its
// cost is the dispatch of its workgroups (4096 of them took 27 us at cfg5).
int fix_grid(int nblk, int work);
template <int BN>
int set_lds_attr(const void* fn);
int gemm_store(const float* a, int lda, int rows, int ka, const float* wt, int kap, int ncp, float* c, int ldc,
               int nc, hipStream_t st);

}  // namespace amp
