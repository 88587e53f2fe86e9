// amp_vamp_persist.hip — persistent VAMP engine: the whole iteration loop of
// VAMP.forward (vamp.py:159-187) in ONE cooperative launch.
//
// Each workgroup (256 threads = one wave per SIMD, one workgroup per CU) owns PBM = 16
// trials for the whole forward; their state lives in LDS across iterations:
//   r, xmmse (c64 rows), var of this and the previous iteration (ping-pong), the section
//   max / max|xi| of the last denoiser call, and the GEMM A operand (r~, then w).
// Per iteration t:
//   1. A <- r~ = (xmmse - dxdr r) * normScalar                         (vamp.py:89-91)
//   2. q = Vh r~ on v_mfma_f32_16x16x4_f32 (or the split-precision bf16x3 engine, below);
//      w = scale (y~ + vr q) - q                                         (vamp.py:67-72)
//   3. x~ - r~ = V w; r = (x~ - alpha r~) / (1 - alpha)                  (vamp.py:72-79)
//   4. section denoiser on r (amp_denoise.h)                           (vamp.py:84, 96-119)
//   5. one grid barrier: every workgroup reduces the same per-workgroup partials in the same
//      order, so every workgroup derives bit-identical batch scalars (mean var, allclose,
//      max|xi|, vamp.py:85-94 and 185) with no second exchange.  The rare exact-float64
//      path (amp_denoise.h: G out of range) takes two more barriers, uniformly.
// The weights are streamed from L2 by each wave in 16x16x4-packed order (amp_gemm.h,
// wpack16_index): a wave owns 16*NT output columns, NT independent accumulators.
// y~ = (s Uh) y comes from the launch engine's GEMM once per forward (amp_vamp.hip).
// X3 (default where the LDS fits): both GEMMs as 6-term bf16x3 products on
// v_mfma_f32_16x16x32_bf16 (amp_persist.h gemm_x3), A in LDS as six bf16 planes, the operators
// complex-planar (12 bytes per entry instead of the real expansion's 16); instantiated in
// amp_vamp_persist_x3.hip.  The kernel template lives in amp_vamp_persist_kernel.h.
//
// Co-residency: ceil(B/16) <= #CUs workgroups, one per CU by its LDS footprint; the launch
// checks occupancy x CUs >= grid first (or uses hipLaunchCooperativeKernel, which makes the
// same check); every barrier spin is bounded (2 s) and raises an abort word that releases
// every other workgroup.
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "amp_vamp_persist_kernel.h"

namespace amp {

// one workgroup per epoch: epoch e's n per-workgroup records -> out[e]
__global__ __launch_bounds__(1024) void vamp_decide_fold(const DecWG* w, int n, amp_counts* out) {
    __shared__ DecWG s[16];
    dec_fold_block(w + (size_t)blockIdx.x * n, n, out + blockIdx.x, s);
}

static std::once_flag g_pers_once;
static int g_ncu = 0;

int device_cu_count() {
    std::call_once(g_pers_once, [] {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&g_ncu, hipDeviceAttributeMultiprocessorCount,
                                                                      dev) != hipSuccess)
            g_ncu = 0;
    });
    return g_ncu;
}

bool vamp_persist_ytil_in_kernel(const VampK& P) {
    // y staged over the A/R/X region: 16 rows of 2n + 4 floats with n == 2N
    return P.n == 2 * P.N && PBM * (2 * P.n + 4) <= playout(P.N, P.k, P.L).offV0;
}

// the fp16x2 y~ prologue: n == 2N and the four y planes (16 rows x n fp16) within the A / R / X
// region of the split-precision carve
bool vamp_persist_ytil_h2(const VampK& P) {
    return P.n == 2 * P.N && P.k == P.N && 2 * PBM * pl_ldx(P.n) <= playout(P.N, P.k, P.L, true).offV0;
}

bool vamp_persist_x3_fits(int N, int k, int L) {
    return k == N && N % 64 == 0 && (size_t)playout(N, k, L, true).total * 4 + 2048 <= 160 * 1024;
}

// Workgroups per CU.  Two at N = 64 on the bf16x3 engine (its instantiation bounded for two
// waves per SIMD, 2 x 256 workgroups for 8 cfg2 epochs per launch; AMP_PERSIST_WG2=0 keeps one).
// The two-per-CU build runs the denoiser in scalar float32 (amp_denoise.h denoise_sections_sel):
// with the packed-math form, co-resident epochs were not reproducible run to run — the
// variance of a section's dominant position lost the Re or Im half of its packed
// sum |x - a_k|^2 eta_k in lanes 48-63 now and then (tools/epochs_diag.py, tools/var_check.py;
// DESIGN.md §3.8).
bool persist_wg2() {
    static const bool v = [] {
        const char* e = diag_env("AMP_PERSIST_WG2");
        return !(e && e[0] == '0') && !gemm_f32_requested();
    }();
    return v;
}
// Side-by-side epochs at two workgroups per CU only in the diagnostic build, with
// AMP_EPOCHS_TWO_PER_CU=1 (tools/occ2_repro.py, tests/test_gpu_epochs.py's 8-epoch cases).  The launches
// keep the two-per-CU build (same bits as one epoch), but by default an epoch group holds at most
// one workgroup per CU: gpurun r6c49 saw one 8-epoch cfg2 launch (two per CU) differ from its
// sequential forwards in one epoch's bit errors, on the tree whose full suite had passed (DESIGN.md
// §3.8, the unexplained two-per-CU corruption).
static bool persist_pair_epochs() {
    static const bool v = [] {
        const char* e = diag_env("AMP_EPOCHS_TWO_PER_CU");
        return e && e[0] == '1';
    }();
    return v;
}
// gemm_mode: the persistent GEMM arithmetic of the call (vamp_gemm_select: 0 f32, 1 bf16x3,
// 2 fp16x2); only the split-precision engines have a two-per-CU instantiation
static int persist_wg_cap(int N, int gemm_mode) {
    return (N == 64 && (gemm_mode == 1 || gemm_mode == 2) && persist_wg2() && persist_pair_epochs()) ? 2 : 1;
}

int vamp_persist_wg_per_cu(const amp_dims* d, int k, int gemm) {
    return persist_wg_cap(d->N, vamp_gemm_select(d, k, gemm));
}

int vamp_persist_max_epochs(const amp_dims* d, int k, int ncu, int gemm) {
    const int gemm_mode = vamp_gemm_select(d, k, gemm);
    if (k != d->N || !(d->N == 64 || d->N == 128 || d->N == 256) || d->M > 64) return 0;
    if ((size_t)playout(d->N, k, d->L).total * 4 + 2048 > 160 * 1024) return 0;
    const int wpe = cdiv(d->B, PBM);
    if (wpe > ncu) return 0;
    if (d->B % PBM != 0) return 1;
    return std::max(1, persist_wg_cap(d->N, gemm_mode) * ncu / wpe);
}

bool vamp_persist_eligible(const amp_dims* d, int k, int ncu, int epochs, int gemm) {
    if (k != d->N || !(d->N == 64 || d->N == 128 || d->N == 256) || d->M > 64) return false;
    if (epochs < 1 || (epochs > 1 && d->B % PBM != 0)) return false;
    if (cdiv(d->B, PBM) > ncu ||
        (long)epochs * cdiv(d->B, PBM) > (long)persist_wg_cap(d->N, vamp_gemm_select(d, k, gemm)) * ncu)
        return false;
    return (size_t)playout(d->N, k, d->L).total * 4 + 2048 <= 160 * 1024;
}

static int persist_dispatch(const VampK& P, const DecConst& dc, hipStream_t st);
int persist_dispatch_x3(const VampK& P, const DecConst& dc, hipStream_t st);   // amp_vamp_persist_x3.hip
int persist_dispatch_h2(const VampK& P, const DecConst& dc, hipStream_t st);   // amp_vamp_persist_h2.hip
int persist_dispatch_i8(const VampK& P, const DecConst& dc, hipStream_t st);   // amp_vamp_persist_i8.hip

// amp_debug_persist_timing: while on, a HIP event pair around every vamp_persist launch (bench.py
// times the kernel inside a loop of forwards, the conditions of its timed region).
static std::mutex g_tm_mu;
static bool g_tm_on = false;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_tm_ev;

// c64 is the rare path's float64 table; dc the decision's (dec_on) — one by-value table in the
// launch: dc's Const64 base is overwritten with c64.
int vamp_persist_launch(const VampK& P, const Const64& c64, const DecConst& dc, hipStream_t st, int ncu) {
    (void)ncu;
    DecConst d2 = dc;
    static_cast<Const64&>(d2) = c64;
    hipEvent_t te[2] = {nullptr, nullptr};
    {
        std::lock_guard<std::mutex> lk(g_tm_mu);
        if (g_tm_on && hipEventCreate(&te[0]) == hipSuccess && hipEventCreate(&te[1]) == hipSuccess) {
            g_tm_ev.emplace_back(te[0], te[1]);
            (void)hipEventRecord(te[0], st);
        } else {
            te[0] = te[1] = nullptr;
        }
    }
    // the decision's counter records are folded inside the launch (amp_decide_fused.h
    // dec_fold_gather; a shard folds its own workgroups), else by one block per epoch here
    const int rc = persist_dispatch(P, d2, st);
    if (te[1]) (void)hipEventRecord(te[1], st);
    if (rc || !P.dec_on || P.fold_in) return rc;
    hipLaunchKernelGGL(vamp_decide_fold, dim3(P.E), dim3(256), 0, st, (const DecWG*)P.dwg, P.nwg / P.E, P.counts);
    AMP_LAUNCH_CHECK("vamp_decide_fold");
    return AMP_OK;
}

static int persist_dispatch(const VampK& P, const DecConst& dc, hipStream_t st) {
    // the barrier words were zeroed by the prepare launch; the granules carry generation tags
    // NT = 2N / (16 * waves) column tiles of 16 per wave (both GEMMs are 2N x 2N: k == N)
    if (P.x3 == 3) return persist_dispatch_i8(P, dc, st);
    if (P.x3 == 2) return persist_dispatch_h2(P, dc, st);
    if (P.x3) return persist_dispatch_x3(P, dc, st);
    switch (P.N) {
    case 64: return persist_launch_nt<2, 4, false>(P, dc, st);
    case 128: return persist_launch_nt<4, 4, false>(P, dc, st);
    case 256: return persist_launch_nt<8, 4, false>(P, dc, st);
    default: break;
    }
    set_error("vamp_persist: N = %d not supported", P.N);
    return AMP_E_ARG;
}

}  // namespace amp

int amp_debug_persist_timing(int32_t on) {
    std::lock_guard<std::mutex> lk(amp::g_tm_mu);
    amp::g_tm_on = on != 0;
    return AMP_OK;
}

int amp_debug_persist_time(int32_t* n, float* mean_ms) {
    AMP_REQUIRE(n && mean_ms, "amp_debug_persist_time: null output");
    std::lock_guard<std::mutex> lk(amp::g_tm_mu);
    double tot = 0.0;
    int cnt = 0;
    for (auto& e : amp::g_tm_ev) {
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
            tot += ms;
            ++cnt;
        }
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    amp::g_tm_ev.clear();
    *n = cnt;
    *mean_ms = cnt ? (float)(tot / cnt) : 0.f;
    return AMP_OK;
}
