// amp_gemm.h — fp32 MFMA tile engine for the batched complex mat-vecs.
//
// Every per-iteration product of the detectors is   C[B x Nc] = A[B x Ka] . Wt[Nc x Ka]^T
// with A = one trial per row (the reference's [B, len, 1] batch of vectors, complex
// interleaved {re, im}) and Wt a weight matrix expanded ONCE per forward:
//   complex y = X x   ->  Wt[2o][2j] = Re X, Wt[2o][2j+1] = -Im X,
//                         Wt[2o+1][2j] = Im X, Wt[2o+1][2j+1] = Re X
// so the complex GEMM is a real GEMM whose A rows are the c64 vectors as they lie in
// memory and whose output rows come out interleaved re/im again (8 real flops per
// complex MAC: nothing is wasted).  One H/V is shared by all B trials,
// so this is a true GEMM and runs on v_mfma_f32_32x32x2_f32 (exact f32, 64 flop/clk/SIMD).
//
// Tile: BM = 32 trials x BN (128 | 256) output columns, 4 waves side by side in N, each
// wave owning BN/128 accumulators of 32 x 32.
//  * A (the trials, shared by the 4 waves) is staged ONCE per tile in LDS: the whole
//    32 x K block (K chunks of 512), so the main loop has no barrier and no LDS store.
//  * W is never staged: each wave owns its columns alone, so it streams them straight from
//    L2 in an MFMA-packed layout (below) — one fully coalesced 1 KB global_load_dwordx4
//    per wave feeds 4 MFMAs — through an 8-deep register ring.
// MFMA-packed weights: for a 32-column block cb and a group g of 8 reduction indices,
//   Wp[((cb * kap/8 + g) * 64 + lane) * 4 + s] = Wt[cb*32 + (lane & 31)][8g + 4*(lane >> 5) + s],
// i.e. MFMA s of group g reduces over k = 8g + s (lanes 0-31) and 8g + 4 + s (lanes 32-63);
// the A fragment is read with the same k mapping (one ds_read_b128 per group).
//
// The accumulators are written to an LDS C tile [32][BN+4] that aliases the A block, where
// the caller's fused epilogue (LMMSE step, Onsager update, section denoiser, ...) reads
// whole rows/sections.
#pragma once

#include "amp_common.h"

namespace amp {

constexpr int GBM = 32;       // trials per tile
constexpr int GBK = 64;       // reduction length granule (kap % GBK == 0)
constexpr int GKC = 512;      // A chunk staged in LDS
constexpr int GLDA = GKC + 4; // its row stride (floats): conflict-free ds_read_b128
constexpr int GRING = 8;      // W groups in flight per wave

// KC: the A chunk staged in LDS (GKC; 256 halves the footprint, so four tiles share a CU where
// the reduction ranges are short: the block-banded ISI operators)
template <int BN, int KC = GKC>
struct GemmCfg {
    static_assert(BN == 128 || BN == 256, "BN must be 128 or 256");
    static_assert(KC % GBK == 0 && KC <= GKC, "KC");
    static constexpr int NACC = BN / 128;                 // 32x32 accumulators per wave
    static constexpr int WN = BN / 4;                     // columns per wave
    static constexpr int LDC = BN + 4;                    // C tile row stride (floats)
    static constexpr int LDA = KC + 4;                    // A chunk row stride (floats)
    static constexpr int A_FLOATS = GBM * LDA;
    static constexpr int CTILE_FLOATS = GBM * LDC;
    static constexpr int LDS_FLOATS = A_FLOATS;           // C tile + epilogue scratch fit inside
    static_assert(CTILE_FLOATS + 2048 <= A_FLOATS, "epilogue scratch");
    static constexpr size_t LDS_BYTES = (size_t)LDS_FLOATS * 4;
};

// Packed index of Wt[n][k] (n = output column, k = reduction index) for a kap-long reduction.
__host__ __device__ __forceinline__ size_t wpack_index(int n, int k, int kap) {
    const int cb = n >> 5, jj = n & 31, g = k >> 3, w = k & 7;
    const int lane = jj + 32 * (w >> 2);
    return (((size_t)cb * (kap >> 3) + g) * 64 + lane) * 4 + (w & 3);
}

// Packing for the 16x16x4 form (persistent VAMP engine): 16-column block ct, group g of 16
// reduction indices; MFMA s of the group reduces over k = 16g + 4*(lane >> 4) + s.
__host__ __device__ __forceinline__ size_t wpack16_index(int n, int k, int kap) {
    const int ct = n >> 4, g = k >> 4, w = k & 15;
    const int lane = (n & 15) + 16 * (w >> 2);
    return (((size_t)ct * (kap >> 4) + g) * 64 + lane) * 4 + (w & 3);
}

// Packing for the split-precision complex form (gemm_x3, amp_persist.h): X[o][j] (o < O complex
// outputs, j < J complex inputs, J % 32 == 0) as bf16 pieces; 16-column tile ct = o >> 4, group
// g = j >> 5, plane f (0-2: Re x0 x1 x2, 3-5: Im x0 x1 x2), lane (o & 15) + 16 ((j & 31) >> 3),
// element j & 7: one 16-byte buffer load per lane and plane.
__host__ __device__ __forceinline__ size_t x3_index(int o, int j, int f, int J) {
    const int kk = j & 31;
    const int lane = (o & 15) + 16 * (kk >> 3);
    return ((((size_t)(o >> 4) * (J >> 5) + (j >> 5)) * 6 + f) * 64 + lane) * 8 + (kk & 7);
}

// The same for a real operator in the bf16x3 launch tile (amp_gemm_x3.h): three planes per
// (tile, group), f = 0-2: x0 x1 x2.
__host__ __device__ __forceinline__ size_t x3r_index(int o, int j, int f, int J) {
    const int kk = j & 31;
    const int lane = (o & 15) + 16 * (kk >> 3);
    return ((((size_t)(o >> 4) * (J >> 5) + (j >> 5)) * 3 + f) * 64 + lane) * 8 + (kk & 7);
}

// The same for the fp16x2 form (gemm_h2): four planes per (tile, group), f = 0-1: Re h0 h1,
// 2-3: Im h0 h1.
__host__ __device__ __forceinline__ size_t h2_index(int o, int j, int f, int J) {
    const int kk = j & 31;
    const int lane = (o & 15) + 16 * (kk >> 3);
    return ((((size_t)(o >> 4) * (J >> 5) + (j >> 5)) * 4 + f) * 64 + lane) * 8 + (kk & 7);
}

// The same for the int8x4 form (gemm_i8, amp_persist.h): X[o][j] 2^(30 - e_o) rounded to a 31-bit
// integer, written as four balanced base-256 digits; 16-column tile ct = o >> 4, group g = j >> 6
// (J % 64 == 0), plane f (0-3: Re digits top first, 4-7: Im), lane (o & 15) + 16 ((j & 63) >> 4),
// byte j & 15: one 16-byte buffer load per lane and plane (the i8 16x16x64 fragment).  The column
// exponents e_o follow the planes as ints (amp_persist.h i8_exp_offset bytes in).
__host__ __device__ __forceinline__ size_t i8_index(int o, int j, int f, int J) {
    const int kk = j & 63;
    const int lane = (o & 15) + 16 * (kk >> 4);
    return ((((size_t)(o >> 4) * (J >> 6) + (j >> 6)) * 8 + f) * 64 + lane) * 16 + (kk & 15);
}

// XCD-aware tile order.  Workgroups are dispatched in linear order (x fastest) round-robin over
// the 8 XCDs, each with its own 4 MB L2.  The row-block-fastest grid would make every XCD sweep
// ALL column blocks, i.e. the whole packed weight (8 MB for BAMP's H at cfg5) through each L2.
// Remapped, XCD x walks a contiguous run of tiles in column-block-major order: ~1/8 of the
// column blocks over all row blocks, so its share of the weight stays resident in its L2.
// A bijection of [0, gridDim.x * gridDim.y): every tile is computed exactly once.
struct GemmTile {
    int rb, cb;      // row block (trials), column block
};
__device__ __forceinline__ GemmTile xcd_tile() {
    constexpr int NXCD = 8;
    const int nr = gridDim.x, total = gridDim.x * gridDim.y;
    const int id = blockIdx.y * nr + blockIdx.x;
    const int x = id % NXCD, q = id / NXCD;
    const int base = total / NXCD, rem = total % NXCD;
    const int pos = x * base + min(x, rem) + q;
    return GemmTile{pos % nr, pos / nr};
}

// Row-block-major variant (the fp16x2 tiles, amp_gemm_h2.h): XCD x walks a contiguous run of
// tiles row block by row block, every column block of one row block in turn, so each XCD reads
// its rows' A planes once (they stay in its L2 while the column blocks pass) and serves the whole
// operator from its L2 (4 MB at cfg5's H as fp16x2 planes).  Also a bijection.
__device__ __forceinline__ GemmTile xcd_tile_rows() {
    constexpr int NXCD = 8;
    const int nr = gridDim.x, nc = gridDim.y, total = nr * nc;
    const int id = blockIdx.y * nr + blockIdx.x;
    const int x = id % NXCD, q = id / NXCD;
    const int base = total / NXCD, rem = total % NXCD;
    const int pos = x * base + min(x, rem) + q;
    return GemmTile{pos / nc, pos % nc};
}

// Plain A operand: rows of `lda` floats, `ka` valid columns (zero beyond, and for rows >= rows;
// ka % 4 == 0, ka >= 4, rows >= 1).  The tile stages its A chunks in two steps: raw() issues the
// load at a clamped, always valid address (no branch: a lane-divergent `if` around a load makes
// the other lanes' zero write wait for it, i.e. every load of a chunk waited out its full latency
// in turn), fin() zeroes the out-of-range elements once the value is needed (at the LDS store).
struct ALoadPlain {
    const float* __restrict__ a;
    int lda, rows, ka;
    using Raw = float4;
    __device__ __forceinline__ Raw raw(int row, int k) const {
        return *reinterpret_cast<const float4*>(a + (size_t)min(row, rows - 1) * lda + min(k, ka - 4));
    }
    __device__ __forceinline__ float4 fin(const Raw& v, int row, int k) const {
        const bool ok = row < rows && k < ka;
        return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
};

// Computes the C tile of rows [row0, row0+32) x cols [col0, col0+BN) into `lds` (as the C
// tile, row stride GemmCfg<BN>::LDC).  `wp` is the MFMA-packed [Ncp][kap] weight,
// kap % GBK == 0, col0 % BN == 0, col0 + BN <= Ncp.  [kb, ke): the reduction range that holds
// every nonzero weight of this column tile (multiples of GBK; weight_kband), default all of it:
// a block-banded operator (the ISI / spatially coupled channel, channel.py:75-95) skips its
// all-zero blocks.
template <int BN, class AL, int KC = GKC>
__device__ __forceinline__ void gemm_tile(const AL& al, const float* __restrict__ wp, int kap, int row0,
                                          int col0, float* lds, int kb = 0, int ke = -1) {
    using C = GemmCfg<BN, KC>;
    constexpr int LDA = C::LDA;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int G = kap >> 3;   // groups of 8 reduction indices

    f32x16 acc[C::NACC];
#pragma unroll
    for (int j = 0; j < C::NACC; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    const float4* wcol[C::NACC];
#pragma unroll
    for (int j = 0; j < C::NACC; ++j)
        wcol[j] = reinterpret_cast<const float4*>(wp) + ((size_t)((col0 >> 5) + wave * C::NACC + j) * G) * 64 + lane;

    if (ke < 0) ke = kap;
    const int glast = (ke >> 3) - 1;   // last group of the range
    // The W ring runs across the chunks: a slot refilled GRING groups ahead past the end of a
    // chunk already holds the next chunk's group (every chunk is a whole number of rings), so a
    // chunk starts without waiting on its first operator loads.
    float4 ring[GRING][C::NACC];
#pragma unroll
    for (int d = 0; d < GRING; ++d)
#pragma unroll
        for (int j = 0; j < C::NACC; ++j) ring[d][j] = wcol[j][(size_t)((kb >> 3) + d) * 64];
    // A chunk staging: all loads of a batch in flight before its LDS stores.  Short chunks
    // (KC <= 256: 8 float4 per thread) load the NEXT chunk into registers while this one's MFMAs
    // run; 512-wide chunks stage in two half-batches between the chunks.  Every chunk is staged
    // with the full chunk's compile-time geometry and no branch (AL::raw / fin): a tail chunk's
    // columns past ke are loaded at clamped addresses and land in LDS, but no group reads them.
    // (Masking those loads instead put the staging back inside branches, where the compiler
    // drains the weight ring before the stores: cfg5 BAMP 18.3 -> 20.5 ms, same box.)
    constexpr int PER = GBM * (KC / 4) / AMP_WG;    // float4 per thread for a full chunk
    constexpr bool PF = PER <= 8;
    using Raw = typename AL::Raw;
    Raw nxt[PF ? PER : 1];
    auto load_chunk = [&](int c0, Raw* t4, int h, int cnt) {
#pragma unroll
        for (int i = 0; i < cnt; ++i) {
            const int e = tid + (h + i) * AMP_WG;
            const int row = e / (KC / 4), k4 = e % (KC / 4);
            t4[i] = al.raw(row0 + row, c0 + 4 * k4);
        }
    };
    auto store_chunk = [&](int c0, const Raw* t4, int h, int cnt) {
#pragma unroll
        for (int i = 0; i < cnt; ++i) {
            const int e = tid + (h + i) * AMP_WG;
            const int row = e / (KC / 4), k4 = e % (KC / 4);
            *reinterpret_cast<float4*>(lds + row * LDA + 4 * k4) = al.fin(t4[i], row0 + row, c0 + 4 * k4);
        }
    };
    if constexpr (PF) {
        load_chunk(kb, nxt, 0, PER);
        store_chunk(kb, nxt, 0, PER);
    }
    for (int kc0 = kb; kc0 < ke; kc0 += KC) {
        const int kc = min(KC, ke - kc0);
        const int g0 = kc0 >> 3, gc = kc >> 3;   // gc % GRING == 0 (kap % 64 == 0)
        if constexpr (PF) {
            __syncthreads();   // this chunk's LDS stores are visible
            if (kc0 + KC < ke) load_chunk(kc0 + KC, nxt, 0, PER);
        } else {
            if (kc0 > kb) __syncthreads();   // every wave is done with the previous chunk
#pragma unroll
            for (int h = 0; h < PER; h += PER / 2) {
                Raw t4[PER / 2];
                load_chunk(kc0, t4, h, PER / 2);
                store_chunk(kc0, t4, h, PER / 2);
            }
            __syncthreads();
        }
        // Per group: read the NEXT group's A fragment, issue this group's MFMAs, then refill this
        // ring slot GRING groups ahead.  The scheduling barrier pins that order (left alone, the
        // scheduler sinks all refills behind the MFMAs and drains them at once).
        const float* a_s = lds + li * LDA + 4 * lh;
        float4 acur = *reinterpret_cast<const float4*>(a_s);
        for (int gb = 0; gb < gc; gb += GRING) {
#pragma unroll
            for (int d = 0; d < GRING; ++d) {
                const int g = gb + d;
                const float4 anext = *reinterpret_cast<const float4*>(a_s + 8 * min(g + 1, gc - 1));
#pragma unroll
                for (int j = 0; j < C::NACC; ++j) {
                    acc[j] = mfma32x32x2(acur.x, ring[d][j].x, acc[j]);
                    acc[j] = mfma32x32x2(acur.y, ring[d][j].y, acc[j]);
                    acc[j] = mfma32x32x2(acur.z, ring[d][j].z, acc[j]);
                    acc[j] = mfma32x32x2(acur.w, ring[d][j].w, acc[j]);
                }
                // refill GRING groups ahead, into the next chunk (clamped: the tail of the range
                // re-reads its last group)
                const int gn = min(g0 + g + GRING, glast);
#pragma unroll
                for (int j = 0; j < C::NACC; ++j) ring[d][j] = wcol[j][(size_t)gn * 64];
                acur = anext;
                // the next group's A read goes out BEFORE this group's MFMAs: left alone the
                // scheduler put it after them, into the registers they read, and every group then
                // waited out the LDS latency with one wave per SIMD (lgkmcnt(0) before its MFMAs)
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 4 * C::NACC, 0);      // MFMA
                __builtin_amdgcn_sched_group_barrier(0x020, C::NACC, 0);          // VMEM read
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (PF) {
            if (kc0 + KC < ke) {
                __syncthreads();   // every wave is done with this chunk
                store_chunk(kc0 + KC, nxt, 0, PER);
            }
        }
    }
    __syncthreads();   // the C tile aliases the A block
    float* ct = lds;
#pragma unroll
    for (int j = 0; j < C::NACC; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            const int col = wave * C::WN + j * 32 + li;
            ct[row * C::LDC + col] = acc[j][r];
        }
    __syncthreads();
}

}  // namespace amp
