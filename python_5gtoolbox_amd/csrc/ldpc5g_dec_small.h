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
//   * messages are stored in CSC order (column j's edges rows ascending), so a column sums consecutive
//     slots whose reads are all independent; the edge words (column, CSC slot, V mod Zc) are staged
//     into LDS once per launch, a thread per edge (lane-varying rows read them by LDS broadcast), and
//     a row's LQ reads are issued 8 at a time before any is used.
// LDS: LQ of the core columns + one message per core edge, KC*Zc + Ec*Zc values (BG1 Zc=64 float64:
// 153.6 KB of the CU's 160 KB).
#pragma once
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {
namespace {

constexpr int kSmallMaxZc = 64;
constexpr int kSmallMaxThreads = 1024;
// check nodes per thread RPT (a template argument: 1 for Zc <= 22, up to 3 for BG1 Zc = 64, since
// MB*Zc <= 46*64 = 2944 <= 3*1024) and core column entries per thread (KC*Zc <= KC/MB * RPT threads)
constexpr int kSmallMaxRpt = 3;
template <int RPT>
constexpr int small_cpt() { return RPT == 1 ? 1 : 2; }

// the core edges' messages live in CSC order: position p of column j's list (rows ascending, the
// order Lr.sum(axis=0) adds them) is message slot p, so the column pass reads consecutive slots
template <int BG>
struct SmallPlan {
    int16_t cstart[BGT<BG>::KC + 1] = {};
    uint16_t ew[BGT<BG>::E] = {};   // static part of an edge word: column | CSC position << 8
    int ncore = 0, dmax = 0;
    constexpr SmallPlan() {
        using P = BGT<BG>;
        int n = 0;
        for (int j = 0; j < P::KC; ++j) {
            cstart[j] = (int16_t)n;
            for (int i = 0; i < P::MB; ++i)
                for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                    if (P::COL[e] == j) ew[e] = (uint16_t)(j | (n++ << 8));
        }
        cstart[P::KC] = (int16_t)n;
        ncore = n;
        for (int e = 0; e < P::E; ++e)
            if (P::COL[e] >= P::KC) ew[e] = (uint16_t)P::COL[e];
        for (int i = 0; i < P::MB; ++i) dmax = dmax > P::RS[i + 1] - P::RS[i] ? dmax : P::RS[i + 1] - P::RS[i];
    }
};
template <int BG>
__device__ constexpr SmallPlan<BG> kSmallPlanD{};
template <int BG>
constexpr SmallPlan<BG> kSmallPlanH{};

template <int BG, typename T>
constexpr size_t small_lds_bytes_t(int Zc) {
    using P = BGT<BG>;
    return (size_t)(P::KC + kSmallPlanH<BG>.ncore) * Zc * sizeof(T) + (size_t)(P::E + 4) * 4;
}

template <int BG, typename T, bool OFS, int kSmallRpt>
__global__ __launch_bounds__(kSmallMaxThreads) void ldpc_small_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int Zc, int zi, int64_t ldl, int64_t ldc, int L, T alpha, T beta,
    int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E;
    constexpr int NCE = kSmallPlanH<BG>.ncore, DMAX = kSmallPlanH<BG>.dmax;
    constexpr int CH = 8;   // edges whose LQ reads are in flight together
    constexpr int kSmallCpt = small_cpt<kSmallRpt>();
    extern __shared__ __align__(16) unsigned char smem[];
    T* LQ = (T*)smem;                           // [KC][Zc]  LQ of the core columns
    T* LR = LQ + KC * Zc;                       // [NCE][Zc] message at CSC position p, column row z'
    uint32_t* ew = (uint32_t*)(LR + NCE * Zc);  // [E] column | CSC position << 8 | (V mod Zc) << 20
    int* flag = (int*)(ew + E);                 // "some row failed" epoch, then the final verdict

    const int cb = blockIdx.x;
    const T* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    const int t = threadIdx.x, NT = blockDim.x;
    const int NR = MB * Zc, NC = KC * Zc;

    // ---- edge words (one thread per edge: a single round trip to the constant tables); LQ =
    //      LLRin (:94), punctured columns 0 (:43)
    for (int e = t; e < E; e += NT)
        ew[e] = (uint32_t)kSmallPlanD<BG>.ew[e] | ((uint32_t)shift_of<BG>(zi, e) << 20);
    if (t == 0) flag[0] = 0, flag[1] = 0;
    // own core column entries c = j*Zc + z': channel LLR and CSC range stay in registers
    T lf[kSmallCpt];
    int cz[kSmallCpt], cp0[kSmallCpt], cp1[kSmallCpt];
    bool cpun[kSmallCpt];
#pragma unroll
    for (int k = 0; k < kSmallCpt; ++k) {
        const int c = t + k * NT;
        const int j = c < NC ? c / Zc : 0;
        cz[k] = c - j * Zc;
        cp0[k] = kSmallPlanD<BG>.cstart[j], cp1[k] = kSmallPlanD<BG>.cstart[j + 1];
        cpun[k] = j < pc;
        lf[k] = (c < NC && j >= pc) ? lrow[(j - pc) * Zc + cz[k]] : T(0);
        if (c < NC) LQ[c] = lf[k];
    }
    // own check nodes r = i*Zc + z: row state (nA, nB, signs | argmin << 24), extension LLR
    T nA[kSmallRpt], nB[kSmallRpt], xl[kSmallRpt];
    uint32_t wd[kSmallRpt];
    int ri[kSmallRpt], rz[kSmallRpt], re0[kSmallRpt], rd[kSmallRpt];
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k) {
        const int r = t + k * NT;
        ri[k] = r < NR ? r / Zc : 0;
        rz[k] = r - ri[k] * Zc;
        re0[k] = row_start_d<BG>(ri[k]);
        rd[k] = row_start_d<BG>(ri[k] + 1) - re0[k];
        nA[k] = T(0), nB[k] = T(0), wd[k] = 0u;
        xl[k] = (r < NR && ri[k] >= 4) ? lrow[(KB + ri[k] - pc) * Zc + rz[k]] : T(0);
    }
    lds_barrier();
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR v_bitop3 is full rate)
    asm volatile("" : "+v"(mv));
    // entry (z + s) mod Zc of a column
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
            const int z = rz[k], e0 = re0[k], d = rd[k];
            // the row's edge words, all requested at once (LDS broadcast within a row)
            uint32_t W[DMAX];
#pragma unroll
            for (int x = 0; x < DMAX; ++x) W[x] = x < d ? ew[e0 + x] : (uint32_t)KC;
            uint32_t u = wd[k] << (32 - d);
            const uint32_t idxo = wd[k] >> 24;
            const T mA = nA[k], mB = nB[k];
            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0;
            bool par = false;
#pragma unroll
            for (int c0 = 0; c0 < DMAX; c0 += CH) {
                T a[CH];
#pragma unroll
                for (int x = 0; x < CH && c0 + x < DMAX; ++x) {
                    const uint32_t w = W[c0 + x];
                    const int j = (int)(w & 0xffu);
                    a[x] = LQ[(j < KC ? j : 0) * Zc + rot(z, w >> 20)];
                }
#pragma unroll
                for (int x = 0; x < CH && c0 + x < DMAX; ++x) {
                    const int q0 = c0 + x;
                    if (q0 >= d) break;
                    const int j = (int)(W[q0] & 0xffu);
                    const T rold = xsign_v(idxo == (uint32_t)q0 ? mB : mA, u, mv);
                    u <<= 1;
                    T av = a[x];
                    if (j >= KC) {
                        av = xl[k] + rold;   // LQ of a degree-1 column = LLR + its only r
                        hdx |= (uint32_t)(av < T(0)) << k;
                    }
                    par ^= av < T(0);
                    const T q = av - rold;
                    const T aq = fabs(q);
                    idx = aq < min1 ? (uint32_t)q0 : idx;
                    negs = (negs << 1) | (FT<T>::sbits(q) >> 31);
                    two_min(min1, min2, aq);
                    sx ^= FT<T>::sbits(q);
                }
            }
            fail |= par;
            T x1 = min1, x2 = min2;
            if constexpr (OFS) {
                x1 = min1 - beta, x2 = min2 - beta;   // max(minv - beta, 0) (:201)
                x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
            }
            const uint32_t flip = (uint32_t)((int32_t)sx >> 31) & ((1u << d) - 1u);
            const T nAk = alpha * x1, nBk = alpha * x2;
            nA[k] = nAk, nB[k] = nBk;
            wd[k] = (negs ^ flip) | (idx << 24);
            // the new messages of the core edges, at their CSC position and column row
            uint32_t un = wd[k] << (32 - d);
#pragma unroll
            for (int q0 = 0; q0 < DMAX; ++q0) {
                if (q0 >= d) break;
                const uint32_t w = W[q0];
                if ((int)(w & 0xffu) < KC) {
                    const T r = xsign_v(idx == (uint32_t)q0 ? nBk : nAk, un, mv);
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
                if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(LQ[t + k * NT] < T(0));
#pragma unroll
            for (int k = 0; k < kSmallRpt; ++k)
                if (t + k * NT < NR && ri[k] >= 4) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)((hdx >> k) & 1u);
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        // ---- LQ = LLRin + Lr.sum(axis=0) (:126): core columns, rows ascending (consecutive
        //      CSC slots, four reads in flight)
#pragma unroll
        for (int k = 0; k < kSmallCpt; ++k) {
            if (t + k * NT >= NC) continue;
            const int z = cz[k], p1 = cp1[k];
            int p = cp0[k];
            T acc = T(0) + LR[p * Zc + z];
            for (++p; p + 4 <= p1; p += 4) {
                const T v0 = LR[p * Zc + z], v1 = LR[(p + 1) * Zc + z];
                const T v2 = LR[(p + 2) * Zc + z], v3 = LR[(p + 3) * Zc + z];
                acc = acc + v0;
                acc = acc + v1;
                acc = acc + v2;
                acc = acc + v3;
            }
            for (; p < p1; ++p) acc = acc + LR[p * Zc + z];
            LQ[t + k * NT] = (cpun[k] ? T(0) : lf[k]) + acc;   // punctured columns: LLR 0 (:43)
        }
        lds_barrier();
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    bool fail = false;
    uint32_t ox = 0;
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k) {
        if (t + k * NT >= NR) continue;
        const int i = ri[k], z = rz[k], e0 = re0[k], d = rd[k];
        bool par = false;
        if (i >= 4) {   // the extension edge is the row's last: LLR + its r
            const T rx = xsign_v((wd[k] >> 24) == (uint32_t)(d - 1) ? nB[k] : nA[k], wd[k] << 31, mv);
            const bool b = xl[k] + rx <= T(0);
            ox |= (uint32_t)b << k;
            par = b;
        }
        uint32_t W[DMAX];
#pragma unroll
        for (int x = 0; x < DMAX; ++x) W[x] = x < d ? ew[e0 + x] : (uint32_t)KC;
#pragma unroll
        for (int x = 0; x < DMAX; ++x) {
            const int j = (int)(W[x] & 0xffu);
            if (j < KC) par ^= LQ[j * Zc + rot(z, W[x] >> 20)] <= T(0);
        }
        fail |= par;
    }
    if (fail) flag[1] = 1;
    lds_barrier();
#pragma unroll
    for (int k = 0; k < kSmallCpt; ++k)
        if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(LQ[t + k * NT] <= T(0));
#pragma unroll
    for (int k = 0; k < kSmallRpt; ++k)
        if (t + k * NT < NR && ri[k] >= 4) crow[(KB + ri[k]) * Zc + rz[k]] = (int8_t)((ox >> k) & 1u);
    if (t == 0) status[cb] = flag[1] == 0, iters[cb] = L;
}

template <int BG, typename T, bool OFS, int RPT>
constexpr auto small_kernel() { return ldpc_small_kernel<BG, T, OFS, RPT>; }

template <int BG, typename T>
bool small_fits(int Zc) {
    return Zc <= kSmallMaxZc && small_lds_bytes_t<BG, T>(Zc) <= kLdsPerCU;
}

template <int BG, typename T, int RPT>
int launch_small_rpt(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                     int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, int threads,
                     hipStream_t st) {
    const bool ofs = beta != 0.0;
    auto kern = ofs ? ldpc_small_kernel<BG, T, true, RPT> : ldpc_small_kernel<BG, T, false, RPT>;
    const size_t lds = small_lds_bytes_t<BG, T>(64);   // one attribute value for every Zc <= 64
    if (int rc = ofs ? set_lds_once<small_kernel<BG, T, true, RPT>()>(lds) : set_lds_once<small_kernel<BG, T, false, RPT>()>(lds))
        return rc;
    const size_t lds_zc = small_lds_bytes_t<BG, T>(Zc);
    hipLaunchKernelGGL(kern, dim3(B), dim3(threads), lds_zc, st, llr, ck, status, iters, Zc, zi, ldl, ldc, L,
                       (T)alpha, (T)beta, pc);
    return check_hip(hipGetLastError(), "ldpc_small_kernel launch");
}

// one codeblock per workgroup, B workgroups; the caller checks small_fits
template <int BG, typename T>
int launch_small_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                   int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    const int nodes = BGT<BG>::MB * Zc;
    const int threads = std::min(kSmallMaxThreads, ((nodes + 63) / 64) * 64);
    const int rpt = (nodes + threads - 1) / threads;
    if (!small_fits<BG, T>(Zc) || rpt > kSmallMaxRpt || BGT<BG>::KC * Zc > (rpt == 1 ? 1 : 2) * threads)
        return fail(LDPC5G_ESIZE, "small-codeblock decoder: Zc=%d does not fit", Zc);
    if (rpt == 1)
        return launch_small_rpt<BG, T, 1>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
    if (rpt == 2)
        return launch_small_rpt<BG, T, 2>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
    return launch_small_rpt<BG, T, 3>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
}

}  // namespace
}  // namespace ldpc5g_impl
