// amp_decide_fused.h — the MAP decision and error counters fused into the end of a persistent
// engine (vamp_persist, scamp_persist): each workgroup decides its own rows from LDS and writes
// one DecWG record; vamp_decide_fold (one workgroup per epoch) folds them in a fixed order.
// PK: the engine's parameter struct (VampK / ScampK) with M, L, N, Na, Lin, ibits, xtrue, sym, idx
// and dwg.
#pragma once

#include "amp_decide.h"
#include "amp_persist.h"

namespace amp {

// Fused MAP decision + error counters (Loss.error_rate, loss.py:67-179, via amp_decide.h) on
// this workgroup's rows while the decision input (VAMP: r, vamp.py:187; SCAMP: xmap,
// scamp.py:107) and xmmse are still in LDS (sR / sX, row stride ldr);
// per-workgroup records, folded by the last workgroup to finish (threadfence reduction).
// lab_lds: lab_cap bytes of free LDS (at least nrows * L for the mismatch flags; the labels are
// staged there too when 17 nrows L bytes fit, else read from global memory in the decision loop);
// scr: >= 16 * sizeof(DecWG) bytes.
// row0: first row of the concatenated [E * B] tensors; lrow0: the same trial within its epoch
// (the flat indices and channel uses the counters compare are per batch, loss.py:105-179).
// PUB with a nonzero pub_tag (the persistent engines, which fold the records themselves:
// dec_fold_gather): the record is published as 13 tagged 16-byte granules of 8 bytes each (sc1
// write-through stores, like the per-iteration partials, amp_persist.h part_publish) at
// P.dwg + 256 blockIdx.x bytes; else stored plainly for vamp_decide_fold.
template <int PWG, int KK, bool PUB = false, class PK>
__device__ __forceinline__ void decide_epilogue(const PK& P, const DecConst& dc, const float* sR, const float* sX, int ldr, int row0,
                                int lrow0, int nrows, float* sT, void* lab_lds, int lab_cap, void* scr,
                                unsigned pub_tag = 0) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int M = P.M, L = P.L, N = P.N;
    const int S = nrows * L;
    // one coalesced bulk load of this workgroup's truth rows and labels into LDS (a per-section
    // global load inside the decision loop left every round waiting on HBM latency); labels that
    // do not fit the free region (17 bytes per section: small M, many sections per row) stay in
    // global memory
    const bool stage = 17 * S <= lab_cap;   // workgroup-uniform
    long long* lsym = reinterpret_cast<long long*>(lab_lds);
    long long* lidx = lsym + S;
    unsigned char* mism = stage ? reinterpret_cast<unsigned char*>(lidx + S) : reinterpret_cast<unsigned char*>(lab_lds);
    const long long* gsym = P.sym + (size_t)row0 * L;
    const long long* gidx = P.idx + (size_t)row0 * L;
    {
        // PBM rows of 2N floats = PBM * N / 2 float4: all eight loads in flight before the LDS
        // stores, at a clamped index with no branch (a lane past the end rewrites the last element
        // with the same value).  Named values, not an array: inlined into the engines, a float4[8]
        // stayed a 128-byte scratch array per lane (written by every workgroup: ~17 MB of
        // WRITE_SIZE per cfg4 launch)
        const int tot = nrows * (N >> 1);
        auto at = [&](int e) {
            e = min(e, tot - 1);
            const int row = e / (N >> 1);
            return make_int2(row, 4 * (e - row * (N >> 1)));
        };
        auto ldv = [&](int e) {
            const int2 rc = at(e);
            return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(P.xtrue) +
                                                    (size_t)(row0 + rc.x) * 2 * N + rc.y);
        };
        auto stv = [&](int e, const float4& v) {
            const int2 rc = at(e);
            *reinterpret_cast<float4*>(sT + rc.x * ldr + rc.y) = v;
        };
        for (int e0 = tid; e0 < tot; e0 += 8 * PWG) {
            const float4 v0 = ldv(e0), v1 = ldv(e0 + PWG), v2 = ldv(e0 + 2 * PWG), v3 = ldv(e0 + 3 * PWG);
            const float4 v4 = ldv(e0 + 4 * PWG), v5 = ldv(e0 + 5 * PWG), v6 = ldv(e0 + 6 * PWG), v7 = ldv(e0 + 7 * PWG);
            stv(e0, v0); stv(e0 + PWG, v1); stv(e0 + 2 * PWG, v2); stv(e0 + 3 * PWG, v3);
            stv(e0 + 4 * PWG, v4); stv(e0 + 5 * PWG, v5); stv(e0 + 6 * PWG, v6); stv(e0 + 7 * PWG, v7);
        }
    }
    if (stage) {
        for (int e = tid; e < S; e += PWG) {
            lsym[e] = gsym[e];
            lidx[e] = gidx[e];
        }
    }
    __syncthreads();
    const long long ibmask = dec_ibmask(P.ibits);
    DecPart q = decpart_zero();
    // one section per group of DG = 4 lanes (two DPP steps per reduction), float32 prefilter
    constexpr int DG = 4;
    const int g = lane % DG;
    for (int base = wave * (64 / DG); base < S; base += (PWG / 64) * (64 / DG)) {   // wave-uniform
        const int ls = base + lane / DG;
        const bool act = ls < S;
        const int lsc = act ? ls : S - 1;
        const int row = lsc / L, l = lsc - row * L;
        const float* rp = sR + row * ldr + 2 * l * M;
        const float* xp = sX + row * ldr + 2 * l * M;
        const float* tp = sT + row * ldr + 2 * l * M;
        auto ld = [&](int m, float2& xv, float2& xt, float2& xe) {
            xv = *reinterpret_cast<const float2*>(rp + 2 * m);
            xe = *reinterpret_cast<const float2*>(xp + 2 * m);
            xt = *reinterpret_cast<const float2*>(tp + 2 * m);
        };
        int bi, mm;
        double se;
        decide_section<KK, DG, true>(dc, M, g, ld, bi, mm, se);
        if (act && g == 0) {
            const long long s = (long long)(lrow0 + row) * L + l;
            mism[lsc] = (unsigned char)mm;
            count_section<KK>(dc, s, M, L, P.Na, P.Lin, bi, se, stage ? lsym[lsc] : gsym[lsc],
                              stage ? lidx[lsc] : gidx[lsc], ibmask, q);
        }
    }
    __syncthreads();
    // channel uses (Na sections each) and trials with any mismatch (loss.py:133-136, 150)
    long long ver = 0, verf = 0, verm = 0, verL = 0, fer = 0;
    for (int row = tid; row < nrows; row += PWG) {
        int trial = 0;
        for (int lin = 0; lin < P.Lin; ++lin) {
            int cu = 0;
            for (int a = 0; a < P.Na; ++a) cu |= mism[row * L + lin * P.Na + a];
            ver += cu;
            if (lin == 0) verf += cu;
            if (lin == P.Lin / 2) verm += cu;
            if (lin == P.Lin - 1) verL += cu;
            trial |= cu;
        }
        fer += trial;
    }
    q.ier = group_sum(q.ier, 64); q.ser = group_sum(q.ser, 64); q.iber = group_sum(q.iber, 64);
    q.sber = group_sum(q.sber, 64);
    q.mse = group_sum(q.mse, 64); q.msef = group_sum(q.msef, 64); q.msem = group_sum(q.msem, 64);
    q.mseL = group_sum(q.mseL, 64);
    ver = group_sum(ver, 64); verf = group_sum(verf, 64); verm = group_sum(verm, 64); verL = group_sum(verL, 64);
    fer = group_sum(fer, 64);
    DecWG* sw = reinterpret_cast<DecWG*>(scr);
    if (lane == 0) {
        DecWG w;
        w.p = q; w.ver = ver; w.verf = verf; w.verm = verm; w.verL = verL; w.fer = fer;
        w.pad[0] = w.pad[1] = w.pad[2] = 0;
        sw[wave] = w;
    }
    __syncthreads();
    if (tid == 0) {
        DecWG o = sw[0];
        for (int v = 1; v < PWG / 64; ++v) {
            decpart_add(o.p, sw[v].p);
            o.ver += sw[v].ver; o.verf += sw[v].verf; o.verm += sw[v].verm; o.verL += sw[v].verL; o.fer += sw[v].fer;
        }
        if (PUB && pub_tag != 0u) {
            const unsigned long long v[13] = {
                (unsigned long long)o.p.ier, (unsigned long long)o.p.ser, (unsigned long long)o.p.iber,
                (unsigned long long)o.p.sber, (unsigned long long)__double_as_longlong(o.p.mse),
                (unsigned long long)__double_as_longlong(o.p.msef), (unsigned long long)__double_as_longlong(o.p.msem),
                (unsigned long long)__double_as_longlong(o.p.mseL), (unsigned long long)o.ver,
                (unsigned long long)o.verf, (unsigned long long)o.verm, (unsigned long long)o.verL,
                (unsigned long long)o.fer};
            const __amdgpu_buffer_rsrc_t rs = gran_rsrc(P.dwg, (unsigned)(gridDim.x * 256u));
#pragma unroll
            for (int j = 0; j < 13; ++j) {
                const u32x4 g = {(unsigned)v[j], (unsigned)(v[j] >> 32), (unsigned)j, pub_tag};
                __builtin_amdgcn_raw_buffer_store_b128(g, rs, (int)(blockIdx.x * 256u + 16u * j), 0, 16);   // sc1
            }
        } else {
            P.dwg[blockIdx.x] = o;   // folded by vamp_decide_fold after this launch (no cross-XCD fence here:
                                     // an agent-scope release writes back the L2 and cost ~90 us)
        }
    }
}

// The fold of the n published records of workgroups [base, base + n) of this launch (one epoch),
// by waves 0-3 of the calling workgroup, in vamp_decide_fold's order (thread i < 256 folds records
// i, i + 256, ..., a 64-lane sum per wave, thread 0 adds the four wave sums in order: the same
// bits).  Each thread polls its records' granules until all 13 carry `tag` (a workgroup that has
// not yet reached its epilogue); a bounded spin (2 s).  Thread 0 writes *out.  Returns false (every thread) on a timeout.
template <class PK>
__device__ bool dec_fold_gather(const PK& P, int base, int n, unsigned tag, amp_counts* out, void* lds, int* s_flag) {
    const int tid = threadIdx.x;
    DecWG a;
    a.p = decpart_zero();
    a.ver = a.verf = a.verm = a.verL = a.fer = 0;
    if (tid == 0) *s_flag = 1;
    __syncthreads();
    if (tid < 256) {
        // thread i folds records i, i + 256, ... in order: vamp_decide_fold's order at 256 threads
        const __amdgpu_buffer_rsrc_t rs = gran_rsrc(P.dwg, (unsigned)((base + n) * 256));
        for (int i = tid; i < n; i += 256) {
            const int off = (base + i) * 256;
            u32x4 g[13];
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                bool all = true;
#pragma unroll
                for (int j = 0; j < 13; ++j) {
                    g[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * j, 0, 16);
                    all &= g[j].w == tag;
                }
                if (all) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {   // 2 s at 100 MHz
                    *s_flag = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            auto u64 = [&](int j) { return ((unsigned long long)g[j].y << 32) | g[j].x; };
            DecWG q;
            q.p.ier = (long long)u64(0); q.p.ser = (long long)u64(1); q.p.iber = (long long)u64(2);
            q.p.sber = (long long)u64(3);
            q.p.mse = __longlong_as_double((long long)u64(4)); q.p.msef = __longlong_as_double((long long)u64(5));
            q.p.msem = __longlong_as_double((long long)u64(6)); q.p.mseL = __longlong_as_double((long long)u64(7));
            q.ver = (long long)u64(8); q.verf = (long long)u64(9); q.verm = (long long)u64(10);
            q.verL = (long long)u64(11); q.fer = (long long)u64(12);
            decpart_add(a.p, q.p);
            a.ver += q.ver; a.verf += q.verf; a.verm += q.verm; a.verL += q.verL; a.fer += q.fer;
        }
        a.p.ier = group_sum(a.p.ier, 64); a.p.ser = group_sum(a.p.ser, 64);
        a.p.iber = group_sum(a.p.iber, 64); a.p.sber = group_sum(a.p.sber, 64);
        a.p.mse = group_sum(a.p.mse, 64); a.p.msef = group_sum(a.p.msef, 64);
        a.p.msem = group_sum(a.p.msem, 64); a.p.mseL = group_sum(a.p.mseL, 64);
        a.ver = group_sum(a.ver, 64); a.verf = group_sum(a.verf, 64); a.verm = group_sum(a.verm, 64);
        a.verL = group_sum(a.verL, 64); a.fer = group_sum(a.fer, 64);
    }
    DecWG* sw = reinterpret_cast<DecWG*>(lds);
    __syncthreads();
    if (tid < 256 && (tid & 63) == 0) sw[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        amp_counts c;
        c.ier = c.ser = c.iber = c.sber = 0;
        c.ver = c.verf = c.verm = c.verL = c.fer = 0;
        c.mse = c.msef = c.msem = c.mseL = 0.0;
        for (int v = 0; v < 4; ++v) {
            const DecWG& q = sw[v];
            c.ier += q.p.ier; c.ser += q.p.ser; c.iber += q.p.iber; c.sber += q.p.sber;
            c.mse += q.p.mse; c.msef += q.p.msef; c.msem += q.p.msem; c.mseL += q.p.mseL;
            c.ver += q.ver; c.verf += q.verf; c.verm += q.verm; c.verL += q.verL; c.fer += q.fer;
        }
        *out = c;
    }
    __syncthreads();
    const bool ok = *s_flag != 0;
    __syncthreads();
    return ok;
}

// A record (status, counters) written to page-locked host memory (the caller's
// amp_vamp_decide_args.host_record): status at byte 0, counters at byte 64, as nine 16-byte
// non-temporal stores by thread 0 (the buffer is host memory the device maps uncached; the
// stream's completion signal follows the kernel's stores).
__device__ __forceinline__ void host_record_write(unsigned char* rec, const amp_status& s, const amp_counts& c) {
    u32x4 w[11];
    static_assert(sizeof(amp_status) == 32 && sizeof(amp_counts) == 104, "record layout");
    __builtin_memcpy(&w[0], &s, 32);
    w[2] = w[3] = u32x4{0u, 0u, 0u, 0u};
    w[10] = u32x4{0u, 0u, 0u, 0u};
    __builtin_memcpy(&w[4], &c, 104);
#pragma unroll
    for (int i = 0; i < 11; ++i) {
        if (i == 2 || i == 3) continue;
        __builtin_nontemporal_store(w[i], reinterpret_cast<u32x4*>(rec) + i);
    }
}

__global__ __launch_bounds__(1024) void vamp_decide_fold(const DecWG* w, int n, amp_counts* out);

}  // namespace amp
