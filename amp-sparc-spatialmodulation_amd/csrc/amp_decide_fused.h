// amp_decide_fused.h — the MAP decision and error counters fused into the end of a persistent
// engine (vamp_persist, scamp_persist): each workgroup decides its own rows from LDS and writes
// one DecWG record; vamp_decide_fold (one workgroup per epoch) folds them in a fixed order.
// PK: the engine's parameter struct (VampK / ScampK) with M, L, N, Na, Lin, ibits, xtrue, sym, idx
// and dwg.
#pragma once

#include "amp_decide.h"

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
template <int PWG, int KK, class PK>
__device__ __forceinline__ void decide_epilogue(const PK& P, const DecConst& dc, const float* sR, const float* sX, int ldr, int row0,
                                int lrow0, int nrows, float* sT, void* lab_lds, int lab_cap, void* scr) {
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
        // PBM rows of 2N floats = PBM * N / 2 float4: all loads in flight before the LDS stores
        constexpr int CH = 8;
        const int tot = nrows * (N >> 1);
        for (int e0 = 0; e0 < tot; e0 += PWG * CH) {
            float4 v[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int e = e0 + u * PWG + tid;
                if (e < tot) {
                    const int row = e / (N >> 1), c4 = 4 * (e - row * (N >> 1));
                    v[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(P.xtrue) +
                                                            (size_t)(row0 + row) * 2 * N + c4);
                }
            }
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int e = e0 + u * PWG + tid;
                if (e < tot) {
                    const int row = e / (N >> 1), c4 = 4 * (e - row * (N >> 1));
                    *reinterpret_cast<float4*>(sT + row * ldr + c4) = v[u];
                }
            }
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
        P.dwg[blockIdx.x] = o;   // folded by vamp_decide_fold after this launch (no cross-XCD fence here:
                                 // an agent-scope release writes back the L2 and cost ~90 us)
    }
}

__global__ __launch_bounds__(1024) void vamp_decide_fold(const DecWG* w, int n, amp_counts* out);

}  // namespace amp
