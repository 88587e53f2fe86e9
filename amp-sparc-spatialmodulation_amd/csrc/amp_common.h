// amp_common.h — shared device-side definitions for the gfx950 AMP kernels.
//
// Numerical conventions: kernels are compiled with
// -ffp-contract=off so every elementwise step rounds exactly where the
// reference's torch op rounds; FMAs appear only where written explicitly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/amp_sparc.h"

#define AMP_WAVE 64
#define AMP_WG 256

// float64 exp(x) underflows to exactly 0 for x < ln(2^-1075): the reference's
// section softmax exp(xi - max|xi|) (vamp.py:112) is 0/0 = NaN for a section
// whose every logit lies further than this below the batch-global max.
#define AMP_F64_EXP_UNDERFLOW (-745.13321910194122)

// vamp.py:51-54 (float32 0-dim tensors)
#define AMP_VAR_RATIO_MIN 1.0e-5f
#define AMP_VAR_MIN 1.0e-9f
#define AMP_VAR_MAX 1.0e5f

namespace amp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Per-workgroup partial results of one detector iteration.  The next kernel on
// the stream reduces them (kernel boundary = visibility), so no atomics and a
// fixed summation order: every workgroup that reduces them gets identical bits.
struct alignas(16) Partial {   // 32 B: also the persistent engine's granule pair
    double sumvar;     // sum of var (float64), NaN-propagating
    double maxabs;     // max |xi| over the block (float32 logits; NaN if any input is non-finite)
    double minsecmax;  // min over sections of the section max logit
    uint32_t notclose; // elements failing torch.allclose(var_new, var_prev)
    uint32_t pad;
};
static_assert(sizeof(Partial) == 32, "Partial is one 32-byte granule pair");


// Device-resident scalar state of one VAMP iteration (vamp.py:66-94).
struct alignas(16) VampIter {
    int32_t stopped;   // 1: the loop already broke (vamp.py:185-186); iteration is a no-op
    int32_t T;         // executed iterations once stopped
    int32_t fixed;     // sections of the previous iteration recomputed in exact float64 (-1: all NaN)
    int32_t fixed_all; // the previous iteration was set all-NaN (later ones stay NaN by propagation)
    float vr;          // var_ratio = noise_var / sigma2_tilde       (vamp.py:66)
    float alpha;       // clamped alpha                              (vamp.py:75-77)
    float inv1ma;      // 1 / (1 - alpha) (c64 / f32 == mul by recip) (vamp.py:79)
    float sigma2;      // clamped sigma2                             (vamp.py:80-82)
    float inv_sigma2;  // 1 / sigma2 (denoiser s / tau)              (vamp.py:111)
    float dxdr_prev;   // dxdr of iteration t-1 (0 at t = 0)         (vamp.py:85-87)
    float ns_prev;     // normScalar of iteration t-1 (1 at t = 0)   (vamp.py:89)
    float s2t;         // sigma2_tilde entering iteration t
    float pad1[3];
    double G;          // previous iteration's max|xi|
};

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---- NaN-propagating min/max with torch.maximum / torch.minimum semantics ----
__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || b != b) ? (a + b) : (a > b ? a : b); }
__device__ __forceinline__ float nan_min(float a, float b) { return (a != a || b != b) ? (a + b) : (a < b ? a : b); }
__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || b != b) ? (a + b) : (a > b ? a : b); }
__device__ __forceinline__ double nan_min(double a, double b) { return (a != a || b != b) ? (a + b) : (a < b ? a : b); }
__device__ __forceinline__ float clampf_t(float v, float lo, float hi) { return nan_min(nan_max(v, lo), hi); }

// torch.isclose(a, b, rtol=1e-5, atol=1e-8) in float32, no FMA contraction.
__device__ __forceinline__ bool torch_close(float a, float b) {
    if (a == b) return true;
    float actual = fabsf(__fsub_rn(a, b));
    float allowed = __fadd_rn(1.0e-8f, fabsf(__fmul_rn(1.0e-5f, b)));
    return isfinite(actual) && actual <= allowed;
}

// ---- reductions within aligned groups of G lanes (G power of two <= 64) ----
// Butterfly steps run with the partner distance O ascending, so before step O every aligned
// group of O lanes already holds one value and any pairing of the two halves of a 2O group
// works: DPP quad_perm for O = 1, 2, row_half_mirror / row_mirror for O = 4, 8 (no LDS
// traffic, foldable into the consuming VALU op), permlane16 / permlane32 swaps for 16, 32.
// Every lane ends with the same bits (the combining ops are commutative).
template <int O>
__device__ __forceinline__ int xl_i32(int v) {
    if constexpr (O == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);    // quad_perm [1,0,3,2]
    else if constexpr (O == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    else if constexpr (O == 4) return __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true); // row_half_mirror
    else if constexpr (O == 8) return __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true); // row_mirror
    else {
        // xor 16 / xor 32: gfx950's v_permlane16_swap / v_permlane32_swap (VALU, no LDS round
        // trip as ds_swizzle / ds_bpermute would take): r[0] holds the even half's value and
        // r[1] the odd half's in every lane; the partner's is the other half's
        const unsigned u = (unsigned)v;
        const auto r = (O == 16) ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                                 : __builtin_amdgcn_permlane32_swap(u, u, false, false);
        return (int)((threadIdx.x & O) ? r[0] : r[1]);
    }
}
template <int O> __device__ __forceinline__ float xl(float v) { return __int_as_float(xl_i32<O>(__float_as_int(v))); }
template <int O> __device__ __forceinline__ int xl(int v) { return xl_i32<O>(v); }
template <int O> __device__ __forceinline__ unsigned xl(unsigned v) { return (unsigned)xl_i32<O>((int)v); }
template <int O> __device__ __forceinline__ long long xl(long long v) {
    const int lo = xl_i32<O>((int)(unsigned)v), hi = xl_i32<O>((int)(v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int O> __device__ __forceinline__ double xl(double v) { return __longlong_as_double(xl<O>(__double_as_longlong(v))); }

// Compile-time group size: straight-line VALU (DPP for distances 1-8, gfx950's
// v_permlane16_swap / v_permlane32_swap for 16 and 32), no LDS round trip, no branches, so
// independent reductions interleave.  op(v, v ^ O) is formed as op(even half, odd half) in
// every lane, so all lanes of a group end with the same bits.
template <int O>
__device__ __forceinline__ void xl_pair(float v, float& lo, float& hi) {
    if constexpr (O == 16 || O == 32) {
        const unsigned u = __float_as_uint(v);
        const auto r = (O == 16) ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                                 : __builtin_amdgcn_permlane32_swap(u, u, false, false);
        lo = __uint_as_float(r[0]);   // the even 16/32-lane half's value, in every lane
        hi = __uint_as_float(r[1]);   // the odd half's value
    } else {
        const float p = xl<O>(v);
        const bool odd = (threadIdx.x & O) != 0;
        lo = odd ? p : v;
        hi = odd ? v : p;
    }
}
// Group max of float32 values as an integer max over order-preserving keys: the DPP row
// operations then fuse into v_max_i32_dpp (one instruction per butterfly step; fmaxf needs a
// canonicalising v_max_f32 after every DPP move in IEEE mode).  Key order:
// -NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN, so a (positive, default) NaN wins like
// torch.max; callers flag non-finite inputs separately (DenStat::st_bad).
__device__ __forceinline__ int fkey(float f) {
    const int b = __float_as_int(f);
    return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float funkey(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
template <int O>
__device__ __forceinline__ int imax_step(int v) {
    if constexpr (O == 16 || O == 32) {
        const unsigned u = (unsigned)v;
        const auto r = (O == 16) ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                                 : __builtin_amdgcn_permlane32_swap(u, u, false, false);
        return max((int)r[0], (int)r[1]);
    } else {
        return max(v, xl_i32<O>(v));
    }
}
template <int G>
__device__ __forceinline__ int group_imax_c(int v) {
    if constexpr (G > 1) v = imax_step<1>(v);
    if constexpr (G > 2) v = imax_step<2>(v);
    if constexpr (G > 4) v = imax_step<4>(v);
    if constexpr (G > 8) v = imax_step<8>(v);
    if constexpr (G > 16) v = imax_step<16>(v);
    if constexpr (G > 32) v = imax_step<32>(v);
    return v;
}
template <int G>
__device__ __forceinline__ float group_fmax_c(float v) { return funkey(group_imax_c<G>(fkey(v))); }
// Sum over the group (same bits in every lane: float addition is commutative) and, per lane,
// the sum of every OTHER lane of the group: a sum of non-negative terms when the inputs are,
// so Z - Z_m needs no subtraction.  DPP distances fuse into v_add_f32_dpp.
template <int O>
__device__ __forceinline__ void sum_excl_step(float& tot, float& excl) {
    if constexpr (O == 16 || O == 32) {
        float lo, hi;
        xl_pair<O>(tot, lo, hi);
        excl += (threadIdx.x & O) ? lo : hi;
        tot = lo + hi;
    } else {
        const float p = xl<O>(tot);
        excl += p;
        tot = tot + p;
    }
}
template <int G>
__device__ __forceinline__ void group_sum_excl_c(float& tot, float& excl) {
    if constexpr (G > 1) sum_excl_step<1>(tot, excl);
    if constexpr (G > 2) sum_excl_step<2>(tot, excl);
    if constexpr (G > 4) sum_excl_step<4>(tot, excl);
    if constexpr (G > 8) sum_excl_step<8>(tot, excl);
    if constexpr (G > 16) sum_excl_step<16>(tot, excl);
    if constexpr (G > 32) sum_excl_step<32>(tot, excl);
}

template <class T, class Op>
__device__ __forceinline__ T group_reduce(T v, int G, Op op) {
    if (G > 1) v = op(v, xl<1>(v));
    if (G > 2) v = op(v, xl<2>(v));
    if (G > 4) v = op(v, xl<4>(v));
    if (G > 8) v = op(v, xl<8>(v));
    if (G > 16) v = op(v, xl<16>(v));
    if (G > 32) v = op(v, xl<32>(v));
    return v;
}
template <typename T>
__device__ __forceinline__ T group_max(T v, int G) { return group_reduce(v, G, [](T a, T b) { return a > b ? a : b; }); }
template <typename T>
__device__ __forceinline__ T group_min(T v, int G) { return group_reduce(v, G, [](T a, T b) { return a < b ? a : b; }); }
template <typename T>
__device__ __forceinline__ T group_sum(T v, int G) { return group_reduce(v, G, [](T a, T b) { return a + b; }); }
__device__ __forceinline__ float group_fmax(float v, int G) {
    return group_reduce(v, G, [](float a, float b) { return fmaxf(a, b); });
}
// NaN-sticky variants (a NaN anywhere in the group wins)
template <typename T>
__device__ __forceinline__ T group_max_nan(T v, int G) {
    return group_reduce(v, G, [](T a, T b) { return nan_max(a, b); });
}
template <typename T>
__device__ __forceinline__ T group_min_nan(T v, int G) {
    return group_reduce(v, G, [](T a, T b) { return nan_min(a, b); });
}

// ---- workgroup-level reduction of a Partial (256 threads) ----
// Each thread contributes its own values; thread 0 returns the block result.
struct PartAcc {
    double sumvar = 0.0;
    double maxabs = 0.0;         // |xi| >= 0
    double minsecmax = INFINITY;
    uint32_t notclose = 0;
};

__device__ __forceinline__ void part_wave_reduce(PartAcc& p) {
    p.sumvar = group_sum(p.sumvar, 64);
    p.maxabs = group_max_nan(p.maxabs, 64);
    p.minsecmax = group_min_nan(p.minsecmax, 64);
    p.notclose = group_sum(p.notclose, 64);
}

// Reduces across the 4 waves through LDS scratch (>= 4*32 bytes) and stores the
// block partial from thread 0.
__device__ __forceinline__ void part_block_store(PartAcc p, Partial* dst, void* lds_scratch) {
    part_wave_reduce(p);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Partial* s = reinterpret_cast<Partial*>(lds_scratch);
    __syncthreads();
    if (lane == 0) {
        s[wave].sumvar = p.sumvar; s[wave].maxabs = p.maxabs;
        s[wave].minsecmax = p.minsecmax; s[wave].notclose = p.notclose;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial o;
        o.sumvar = s[0].sumvar; o.maxabs = s[0].maxabs; o.minsecmax = s[0].minsecmax; o.notclose = s[0].notclose;
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) {
            o.sumvar += s[w].sumvar; o.maxabs = nan_max(o.maxabs, s[w].maxabs);
            o.minsecmax = nan_min(o.minsecmax, s[w].minsecmax); o.notclose += s[w].notclose;
        }
        o.pad = 0;
        *dst = o;
    }
    __syncthreads();
}

// Deterministic reduction of nblk partials by one workgroup (every caller gets
// the same bits: fixed per-thread strides, fixed tree).
__device__ __forceinline__ PartAcc part_reduce_all(const Partial* src, int nblk, void* lds_scratch) {
    PartAcc p;
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
        Partial q = src[i];
        p.sumvar += q.sumvar; p.maxabs = nan_max(p.maxabs, q.maxabs);
        p.minsecmax = nan_min(p.minsecmax, q.minsecmax); p.notclose += q.notclose;
    }
    part_wave_reduce(p);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Partial* s = reinterpret_cast<Partial*>(lds_scratch);
    __syncthreads();
    if (lane == 0) {
        s[wave].sumvar = p.sumvar; s[wave].maxabs = p.maxabs;
        s[wave].minsecmax = p.minsecmax; s[wave].notclose = p.notclose;
    }
    __syncthreads();
    PartAcc o;
    o.sumvar = s[0].sumvar; o.maxabs = s[0].maxabs; o.minsecmax = s[0].minsecmax; o.notclose = s[0].notclose;
    for (int w = 1; w < (int)(blockDim.x / 64); ++w) {
        o.sumvar += s[w].sumvar; o.maxabs = nan_max(o.maxabs, s[w].maxabs);
        o.minsecmax = nan_min(o.minsecmax, s[w].minsecmax); o.notclose += s[w].notclose;
    }
    __syncthreads();
    return o;
}

// True in the workgroup that arrives last at `cnt` among the launch's `nblk` workgroups (the
// launch engines' "last block" fold: the batch reduction runs there instead of in a launch of its
// own).  Every workgroup's global stores before the call are visible to the last one (agent-scope
// release on arrival, acquire in the last); the last resets the counter for the next launch.
// Every workgroup of the launch must call it (or none: an early-exiting launch leaves it at 0).
__device__ __forceinline__ bool last_arrival(unsigned* cnt, unsigned nblk) {
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned k = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = k + 1 == nblk;
        if (last) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        s_last = last;
    }
    __syncthreads();
    return s_last != 0;
}

// A section whose max logit lies more than |AMP_DANGER| below the batch max|xi| leaves the
// normal float64 range in the reference's softmax exp(xi - max|xi|) (vamp.py:112): its
// normaliser Z is denormal or zero, so c128 / Z (= * (1/Z)) overflows to inf/NaN, and for
// real alphabets the true division is denormal-quantised or 0/0.  Such sections are
// recomputed with the reference's exact float64 arithmetic (exact_section_f64).
// The fast path's float32 logits carry a few ulp of |xi| of error: every decision on them
// (danger, batch max) is taken with this slack, and the exact path settles it in float64.
#define AMP_DANGER (-700.0)
__device__ __forceinline__ double logit_slack(double G) { return 1e-5 * fabs(G) + 2.0; }
__device__ __forceinline__ bool part_danger(const PartAcc& p) {
    return p.minsecmax - p.maxabs < AMP_DANGER + logit_slack(p.maxabs);
}

// torch's x.abs().max() propagates NaN: once any logit of the batch is NaN or +-inf the
// reference's shift G is NaN / inf and exp(xi - G) makes EVERY section NaN (0/0 or NaN).
__device__ __forceinline__ bool part_allnan(const PartAcc& p) { return !(p.maxabs <= 1.7976931348623157e308); }

// One workgroup writes NaN over n complex entries (and n var entries when var != nullptr).
__device__ __forceinline__ void nan_fill(float* xm, float* var, size_t n) {
    const float q = __int_as_float(0x7fc00000);
    for (size_t e = threadIdx.x; e < n; e += blockDim.x) {
        reinterpret_cast<float2*>(xm)[e] = make_float2(q, q);
        if (var) var[e] = q;
    }
}

// Constellation for the fast path (kept small: it lives in SGPRs of every fused kernel).
// Product-grid decomposition (amp_denoise.h, denoise_step_grid): grid = R when every point is
// (gre[i], gim[j]) of an R x R grid (R = 2, 4, 8, values ascending) with a multiplicity pattern
// the kernels know at compile time: gfull = 1 every point once (GRID_FULL), 2 the reference's
// 16-QAM table (GRID_REF16); otherwise grid = 0 and the direct form runs.
struct Const {
    int K;
    float re[AMP_MAX_K], im[AMP_MAX_K];
    int grid, gfull;
    float gre[8], gim[8];
};

// Constellation in float64 for the reference-exact rare path (never in a hot kernel's args).
struct Const64 {
    int K;
    int real_alpha;    // OOK / BPSK / 4ASK: float64 symbols in the reference (config.py:117)
    double re[AMP_MAX_K], im[AMP_MAX_K];
};

}  // namespace amp
