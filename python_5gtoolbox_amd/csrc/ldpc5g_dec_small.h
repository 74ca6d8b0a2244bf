// ldpc5g_dec_small.h — flooding min-sum decoder for small codeblocks (Zc <= 64), one codeblock per
// workgroup: the launch shape of the per-codeblock drop-ins (BASELINE config 1: ONE BG2 Zc=8 codeblock
// per nr_decode_ldpc call).  Same arithmetic in the same order as ldpc_flood_kernel
// (ldpc5g_dec_flood.h), so float64 is bit-identical to py5gphy/ldpc/nr_ldpc_decode.py:51-143 with
// _min_sum_process :178-227; only the mapping differs:
//   * a thread per check node (base row i, z) for all base rows at once — MB*Zc nodes over at most
//     1024 threads (<= 4 per thread) — so no wave walks a serial chain of rows;
//   * phase A (every row from LQ_old, syndrome of LQ_old) writes each core edge's new message r into a
//     per-edge LDS array at its column position (z + V mod Zc), and a column pass (a thread per core
//     column entry) sums those messages in ascending row order, as Lr.sum(axis=0) (:126):
//     TWO barriers per iteration instead of one per group of column-disjoint rows (32 BG1 / 28 BG2) of
//     the batch kernel's 16-part small configuration;
//   * the edge list (column, V mod Zc, message slot) and the core columns' row-ascending slot lists are
//     staged into LDS once per launch (lane-varying rows read their edges by LDS broadcast).
// LDS: LQ of the core columns + one message per core edge, KC*Zc + Ec*Zc values (BG1 Zc=64 float64:
// 153.6 KB of the CU's 160 KB).
#pragma once
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {
namespace {

constexpr int kSmallMaxZc = 64;
constexpr int kSmallMaxThreads = 1024;
constexpr int kSmallRpt = 4;   // check nodes per thread: MB*Zc <= 46*64 = 2944 <= 4*1024
constexpr int kSmallCpt = 3;   // core column entries per thread: KC*Zc <= 26*64 over >= MB*Zc/4 threads

// core-edge message slots (edges in row-major order, the degree-1 extension edges skipped) and each
// core column's slots in ascending row order (the order Lr.sum(axis=0) adds them)
template <int BG>
struct SmallPlan {
    int16_t cstart[BGT<BG>::KC + 1] = {};
    int16_t cslot[BGT<BG>::E] = {};
    int ncore = 0;
    constexpr SmallPlan() {
        using P = BGT<BG>;
        int slot[P::E] = {};
        for (int e = 0; e < P::E; ++e) slot[e] = P::COL[e] < P::KC ? ncore++ : -1;
        int n = 0;
        for (int j = 0; j < P::KC; ++j) {
            cstart[j] = (int16_t)n;
            for (int i = 0; i < P::MB; ++i)
                for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                    if (P::COL[e] == j) cslot[n++] = (int16_t)slot[e];
        }
        cstart[P::KC] = (int16_t)n;
    }
};
template <int BG>
__device__ constexpr SmallPlan<BG> kSmallPlanD{};
template <int BG>
constexpr SmallPlan<BG> kSmallPlanH{};

template <int BG, typename T>
constexpr size_t small_lds_bytes_t(int Zc) {
    using P = BGT<BG>;
    return (size_t)(P::KC + kSmallPlanH<BG>.ncore) * Zc * sizeof(T) +
           (size_t)(P::E + P::MB + 1 + P::KC + 1 + kSmallPlanH<BG>.ncore + 4) * 4;
}

template <int BG, typename T, bool OFS>
__global__ __launch_bounds__(kSmallMaxThreads) void ldpc_small_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int Zc, int zi, int64_t ldl, int64_t ldc, int L, T alpha, T beta,
    int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E;
    constexpr int NCE = kSmallPlanH<BG>.ncore;
    extern __shared__ __align__(16) unsigned char smem[];
    T* LQ = (T*)smem;                          // [KC][Zc]  LQ of the core columns
    T* LR = LQ + KC * Zc;                      // [NCE][Zc] message of core edge slot, column position
    uint32_t* ew = (uint32_t*)(LR + NCE * Zc); // [E] column | slot << 8 | (V mod Zc) << 20
    uint32_t* rs = ew + E;                     // [MB + 1] row starts
    uint32_t* cst = rs + MB + 1;               // [KC + 1] column list starts
    uint32_t* csl = cst + KC + 1;              // [NCE] slots, rows ascending per column
    int* flag = (int*)(csl + NCE);             // "some row failed" epoch, then the final verdict

    const int cb = blockIdx.x;
    const T* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    const int t = threadIdx.x, NT = blockDim.x;
    const int NR = MB * Zc, NC = KC * Zc;

    // ---- stage the edge tables; LQ = LLRin (:94), punctured columns 0 (:43)
    if (t < MB) {
        const int e0 = row_start_d<BG>(t), e1 = row_start_d<BG>(t + 1);
        int sl = e0 - (t > 4 ? t - 4 : 0);   // core slot of e0: one extension edge per earlier row >= 4
        for (int e = e0; e < e1; ++e) {
            const int j = col_d<BG>(e);
            const uint32_t s = (uint32_t)shift_of<BG>(zi, e);
            ew[e] = (uint32_t)j | ((j < KC ? (uint32_t)sl : 0xfffu) << 8) | (s << 20);
            sl += j < KC;
        }
        rs[t] = (uint32_t)e0;
        if (t == MB - 1) rs[MB] = (uint32_t)e1;
    }
    for (int x = t; x < NCE; x += NT) csl[x] = (uint32_t)kSmallPlanD<BG>.cslot[x];
    if (t <= KC) cst[t] = (uint32_t)kSmallPlanD<BG>.cstart[t];
    if (t == 0) flag[0] = 0, flag[1] = 0;
    // own core column entries c = j*Zc + z': their channel LLRs stay in registers
    T lf[kSmallCpt];
    int cj[kSmallCpt], cz[kSmallCpt];
#pragma unroll
    for (int k = 0; k < kSmallCpt; ++k) {
        const int c = t + k * NT;
        cj[k] = c < NC ? c / Zc : 0;
        cz[k] = c - cj[k] * Zc;
        lf[k] = (c < NC && cj[k] >= pc) ? lrow[(cj[k] - pc) * Zc + cz[k]] : T(0);
        if (c < NC) LQ[c] = lf[k];
    }
    // own check nodes r = i*Zc + z: row state (nA, nB, signs | argmin << 24), extension LLR
    T nA[kSmallRpt], nB[kSmallRpt], xl[kSmallRpt];
    uint32_t wd[kSmallRpt];
    int ri[kSmallRpt], rz[kSmallRpt];
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k) {
        const int r = t + k * NT;
        ri[k] = r < NR ? r / Zc : 0;
        rz[k] = r - ri[k] * Zc;
        nA[k] = T(0), nB[k] = T(0), wd[k] = 0u;
        xl[k] = (r < NR && ri[k] >= 4) ? lrow[(KB + ri[k] - pc) * Zc + rz[k]] : T(0);
    }
    lds_barrier();
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR v_bitop3 is full rate)
    asm volatile("" : "+v"(mv));
    // LQ entry (column j, row z + s mod Zc)
    auto rot = [&](int z, uint32_t s) -> int {
        const int zz = z + (int)s;
        return zz >= Zc ? zz - Zc : zz;
    };

    uint32_t hdx = 0;   // bit k: extension decision of own node k (LQ_old < 0) in the last phase A
    int it = 0;
    for (; it < L; ++it) {
        // ---- phase A: new row state from LQ_old (:117-123, _min_sum_process :186-202), the
        //      syndrome of LQ_old's hard decisions (:107-114) from the same reads
        bool fail = false;
        hdx = 0;
#pragma unroll
        for (int k = 0; k < kSmallRpt; ++k) {
            if (t + k * NT >= NR) continue;
            const int i = ri[k], z = rz[k];
            const int e0 = (int)rs[i], d = (int)rs[i + 1] - e0;
            uint32_t u = wd[k] << (32 - d);
            const uint32_t idxo = wd[k] >> 24;
            const T mA = nA[k], mB = nB[k];
            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0;
            bool par = false;
            for (int q0 = 0; q0 < d; ++q0) {
                const uint32_t w = ew[e0 + q0];
                const int j = (int)(w & 0xffu);
                const T rold = xsign_v(idxo == (uint32_t)q0 ? mB : mA, u, mv);
                u <<= 1;
                T a;
                if (j < KC) {
                    a = LQ[j * Zc + rot(z, w >> 20)];
                } else {
                    a = xl[k] + rold;   // LQ of a degree-1 column = LLR + its only r
                    hdx |= (uint32_t)(a < T(0)) << k;
                }
                par ^= a < T(0);
                const T q = a - rold;
                const T aq = fabs(q);
                idx = aq < min1 ? (uint32_t)q0 : idx;
                negs = (negs << 1) | (FT<T>::sbits(q) >> 31);
                two_min(min1, min2, aq);
                sx ^= FT<T>::sbits(q);
            }
            fail |= par;
            T x1 = min1, x2 = min2;
            if constexpr (OFS) {
                x1 = min1 - beta, x2 = min2 - beta;   // max(minv - beta, 0) (:201)
                x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
            }
            const uint32_t flip = (uint32_t)((int32_t)sx >> 31) & ((1u << d) - 1u);
            nA[k] = alpha * x1, nB[k] = alpha * x2;
            wd[k] = (negs ^ flip) | (idx << 24);
            // the new messages of the core edges, at their column positions
            uint32_t un = wd[k] << (32 - d);
            for (int q0 = 0; q0 < d; ++q0) {
                const uint32_t w = ew[e0 + q0];
                const int j = (int)(w & 0xffu);
                if (j < KC) {
                    const T r = xsign_v(idx == (uint32_t)q0 ? nB[k] : nA[k], un, mv);
                    LR[(int)((w >> 8) & 0xfffu) * Zc + rot(z, w >> 20)] = r;
                }
                un <<= 1;
            }
        }
        if (fail) flag[0] = it + 1;
        lds_barrier();
        if (flag[0] != it + 1) {
            // ---- the syndrome of LQ_old holds (:112-114): its hard decisions are the output
#pragma unroll
            for (int k = 0; k < kSmallCpt; ++k)
                if (t + k * NT < NC) crow[cj[k] * Zc + cz[k]] = (int8_t)(LQ[t + k * NT] < T(0));
#pragma unroll
            for (int k = 0; k < kSmallRpt; ++k)
                if (t + k * NT < NR && ri[k] >= 4) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)((hdx >> k) & 1u);
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        // ---- LQ = LLRin + Lr.sum(axis=0) (:126): core columns, rows ascending
#pragma unroll
        for (int k = 0; k < kSmallCpt; ++k) {
            if (t + k * NT >= NC) continue;
            const int j = cj[k], z = cz[k];
            const int p0 = (int)cst[j], p1 = (int)cst[j + 1];
            T acc = T(0) + LR[(int)csl[p0] * Zc + z];
            for (int p = p0 + 1; p < p1; ++p) acc = acc + LR[(int)csl[p] * Zc + z];
            LQ[t + k * NT] = (j < pc ? T(0) : lf[k]) + acc;   // punctured columns: LLR 0 (:43)
        }
        lds_barrier();
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    bool fail = false;
    uint32_t ox = 0;
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k) {
        if (t + k * NT >= NR) continue;
        const int i = ri[k], z = rz[k];
        const int e0 = (int)rs[i], d = (int)rs[i + 1] - e0;
        bool par = false;
        if (i >= 4) {   // the extension edge is the row's last: LLR + its r
            const T rx = xsign_v((wd[k] >> 24) == (uint32_t)(d - 1) ? nB[k] : nA[k], wd[k] << 31, mv);
            const bool b = xl[k] + rx <= T(0);
            ox |= (uint32_t)b << k;
            par = b;
        }
        for (int q0 = 0; q0 < d; ++q0) {
            const uint32_t w = ew[e0 + q0];
            const int j = (int)(w & 0xffu);
            if (j < KC) par ^= LQ[j * Zc + rot(z, w >> 20)] <= T(0);
        }
        fail |= par;
    }
    if (fail) flag[1] = 1;
    lds_barrier();
#pragma unroll
    for (int k = 0; k < kSmallCpt; ++k)
        if (t + k * NT < NC) crow[cj[k] * Zc + cz[k]] = (int8_t)(LQ[t + k * NT] <= T(0));
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k)
        if (t + k * NT < NR && ri[k] >= 4) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)((ox >> k) & 1u);
    if (t == 0) status[cb] = flag[1] == 0, iters[cb] = L;
}

template <int BG, typename T, bool OFS>
constexpr auto small_kernel() { return ldpc_small_kernel<BG, T, OFS>; }

template <int BG, typename T>
bool small_fits(int Zc) {
    return Zc <= kSmallMaxZc && small_lds_bytes_t<BG, T>(Zc) <= kLdsPerCU;
}

// one codeblock per workgroup, B workgroups; the caller checks small_fits
template <int BG, typename T>
int launch_small_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                   int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    const bool ofs = beta != 0.0;
    auto kern = ofs ? ldpc_small_kernel<BG, T, true> : ldpc_small_kernel<BG, T, false>;
    const int nodes = BGT<BG>::MB * Zc;
    const int threads = std::min(kSmallMaxThreads, ((nodes + 63) / 64) * 64);
    if (!small_fits<BG, T>(Zc) || nodes > kSmallRpt * threads || BGT<BG>::KC * Zc > kSmallCpt * threads)
        return fail(LDPC5G_ESIZE, "small-codeblock decoder: Zc=%d does not fit", Zc);
    const size_t lds = small_lds_bytes_t<BG, T>(64);   // one attribute value for every Zc <= 64
    if (int rc = ofs ? set_lds_once<small_kernel<BG, T, true>()>(lds) : set_lds_once<small_kernel<BG, T, false>()>(lds))
        return rc;
    const size_t lds_zc = small_lds_bytes_t<BG, T>(Zc);
    hipLaunchKernelGGL(kern, dim3(B), dim3(threads), lds_zc, st, llr, ck, status, iters, Zc,
                       zi, ldl, ldc, L, (T)alpha, (T)beta, pc);
    return check_hip(hipGetLastError(), "ldpc_small_kernel launch");
}

}  // namespace
}  // namespace ldpc5g_impl
