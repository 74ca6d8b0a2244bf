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
    uint32_t ew[BGT<BG>::E] = {};   // static part of an edge word: column | CSC position << 8
    int ncore = 0, dmax = 0;
    constexpr SmallPlan() {
        using P = BGT<BG>;
        int n = 0;
        for (int j = 0; j < P::KC; ++j) {
            cstart[j] = (int16_t)n;
            for (int i = 0; i < P::MB; ++i)
                for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                    if (P::COL[e] == j) ew[e] = (uint32_t)(j | (n++ << 8));
        }
        cstart[P::KC] = (int16_t)n;
        ncore = n;
        for (int e = 0; e < P::E; ++e)
            if (P::COL[e] >= P::KC) ew[e] = (uint32_t)P::COL[e];
        for (int i = 0; i < P::MB; ++i) dmax = dmax > P::RS[i + 1] - P::RS[i] ? dmax : P::RS[i + 1] - P::RS[i];
    }
};
template <int BG>
__device__ constexpr SmallPlan<BG> kSmallPlanD{};
template <int BG>
constexpr SmallPlan<BG> kSmallPlanH{};

// LDS bytes: LQ twice per core column (entries z and z + Zc hold LQ of row z, so a read at z + V
// mod Zc needs no wrap), one message per core edge, two edge words per edge, flags
template <int BG, typename T>
constexpr size_t small_lds_bytes_t(int Zc) {
    using P = BGT<BG>;
    return (size_t)(2 * P::KC + kSmallPlanH<BG>.ncore) * Zc * sizeof(T) + (size_t)(2 * P::E + 4) * 4;
}

template <int BG, typename T, bool OFS, int RPT>
__global__ __launch_bounds__(kSmallMaxThreads) void ldpc_small_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int Zc, int zi, int64_t ldl, int64_t ldc, int L, T alpha, T beta,
    int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E, TS = sizeof(T);
    constexpr int NCE = kSmallPlanH<BG>.ncore, DMAX = kSmallPlanH<BG>.dmax;
    constexpr int CPT = small_cpt<RPT>();
    constexpr int CH = 10;   // LQ reads in flight together (BG2's widest row; BG1's rows 0-3 in two)
    extern __shared__ __align__(16) unsigned char smem[];
    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem != 0u)
        __builtin_trap();   // the byte-offset LDS addressing below assumes a zero base
    using lds_T = __attribute__((address_space(3))) T;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    auto at = [&](uint32_t byte) -> lds_T& { return *(lds_T*)(uintptr_t)byte; };
    auto word = [&](uint32_t byte) -> lds_u32& { return *(lds_u32*)(uintptr_t)byte; };
    const uint32_t ZT = (uint32_t)(Zc * TS);
    // byte offsets: LQ2 [KC][2 Zc] | LR [NCE][Zc] | read words [E] | write words [E] | flags
    const uint32_t LR_B = 2u * KC * ZT, RW_B = LR_B + (uint32_t)NCE * ZT, WW_B = RW_B + 4u * E;
    const uint32_t FL_B = WW_B + 4u * E;

    const int cb = blockIdx.x;
    const T* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    const int t = threadIdx.x, NT = blockDim.x;
    const int NR = MB * Zc, NC = KC * Zc;

    // ---- edge words, one thread per edge (a single round trip to the constant tables): read word
    //      = byte offset of LQ2 entry (column j, row V mod Zc) relative to row z; write word = byte
    //      offset of the edge's message slot (CSC position p) | (V mod Zc) * TS << 18
    for (int e = t; e < E; e += NT) {
        const uint32_t w0 = kSmallPlanD<BG>.ew[e];
        const uint32_t j = w0 & 0xffu, pp = w0 >> 8;
        const uint32_t sb = (uint32_t)shift_of<BG>(zi, e) * TS;
        const bool core = j < (uint32_t)KC;
        word(RW_B + 4u * e) = core ? 2u * j * ZT + sb : 0u;
        word(WW_B + 4u * e) = core ? (LR_B + pp * ZT) | (sb << 18) : 0u;
    }
    if (t == 0) word(FL_B) = 0u, word(FL_B + 4) = 0u;
    // own core column entries c = j*Zc + z': LLR, CSC range, LQ2 / message byte offsets
    T lf[CPT];
    uint32_t cq[CPT], cr[CPT];
    int cn[CPT];
    bool cpun[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const int c = t + k * NT;
        const int j = c < NC ? c / Zc : 0, z = c - j * Zc;
        const int p0 = kSmallPlanD<BG>.cstart[j];
        cn[k] = kSmallPlanD<BG>.cstart[j + 1] - p0;
        cq[k] = 2u * (uint32_t)j * ZT + (uint32_t)z * TS;
        cr[k] = LR_B + (uint32_t)p0 * ZT + (uint32_t)z * TS;
        cpun[k] = j < pc;
        lf[k] = (c < NC && j >= pc) ? lrow[(j - pc) * Zc + z] : T(0);
        if (c < NC) at(cq[k]) = lf[k], at(cq[k] + ZT) = lf[k];
    }
    // own check nodes r = i*Zc + z: row state (nA, nB, signs | argmin << 24), extension LLR
    T nA[RPT], nB[RPT], xl[RPT];
    uint32_t wd[RPT], zb[RPT];
    int ri[RPT], re0[RPT], rd[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = t + k * NT;
        ri[k] = r < NR ? r / Zc : 0;
        const int z = r - ri[k] * Zc;
        zb[k] = (uint32_t)z * TS;
        re0[k] = row_start_d<BG>(ri[k]);
        rd[k] = row_start_d<BG>(ri[k] + 1) - re0[k];
        nA[k] = T(0), nB[k] = T(0), wd[k] = 0u;
        xl[k] = (r < NR && ri[k] >= 4) ? lrow[(KB + ri[k] - pc) * Zc + z] : T(0);
    }
    lds_barrier();
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR v_bitop3 is full rate)
    asm volatile("" : "+v"(mv));

    uint32_t hdx = 0;   // bit k: extension decision of own node k (LQ_old < 0) in the last phase A
    int it = 0;
    for (; it < L; ++it) {
        // ---- phase A: new row state from LQ_old (:117-123, _min_sum_process :186-202), the
        //      syndrome of LQ_old's hard decisions (:107-114) from the same reads
        bool fail = false;
        hdx = 0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (t + k * NT >= NR) continue;
            const int e0 = re0[k], d = rd[k];
            const bool xe = ri[k] >= 4;         // rows >= 4: the last edge is the extension column
            const int dc = d - (xe ? 1 : 0);    // core edges
            // the row's LQ reads, all in flight before the first is used (read words are LDS
            // broadcasts within a row)
            uint32_t W[DMAX];
#pragma unroll
            for (int x = 0; x < DMAX; ++x) W[x] = word(RW_B + 4u * (uint32_t)(e0 + (x < dc ? x : 0)));
            uint32_t u = wd[k] << (32 - d);
            const uint32_t idxo = wd[k] >> 24;
            const T mA = nA[k], mB = nB[k];
            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0;
            bool par = false;
            auto edge = [&](int q0, T av, T rold) {
                par ^= av < T(0);
                const T q = av - rold;
                const T aq = fabs(q);
                idx = aq < min1 ? (uint32_t)q0 : idx;
                negs = __builtin_amdgcn_alignbit(negs, FT<T>::sbits(q), 31);
                two_min(min1, min2, aq);
                sx ^= FT<T>::sbits(q);
            };
            // LQ reads in chunks of CH, all of a chunk in flight before the first is used
            sfor<0, (DMAX + CH - 1) / CH>([&](auto cc) {
                constexpr int c0 = decltype(cc)::value * CH, c1 = c0 + CH < DMAX ? c0 + CH : DMAX;
                T a[CH];
                sfor<c0, c1>([&](auto xc) { a[decltype(xc)::value - c0] = at(W[decltype(xc)::value] + zb[k]); });
                sfor<c0, c1>([&](auto xc) {
                    constexpr int q0 = decltype(xc)::value;
                    if (q0 < dc) {
                        const T rold = xsign_v(idxo == (uint32_t)q0 ? mB : mA, u, mv);
                        u <<= 1;
                        edge(q0, a[q0 - c0], rold);
                    }
                });
            });
            if (xe) {   // LQ of the degree-1 column = LLR + its only r
                const T rold = xsign_v(idxo == (uint32_t)dc ? mB : mA, u, mv);
                const T av = xl[k] + rold;
                hdx |= (uint32_t)(av < T(0)) << k;
                edge(dc, av, rold);
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
            // the new messages of the core edges into their slots, at row (z + V) mod Zc
            uint32_t un = wd[k] << (32 - d);
            uint32_t V[DMAX];
#pragma unroll
            for (int x = 0; x < DMAX; ++x) V[x] = word(WW_B + 4u * (uint32_t)(e0 + (x < dc ? x : 0)));
            sfor<0, DMAX>([&](auto xc) {
                constexpr int q0 = decltype(xc)::value;
                if (q0 < dc) {
                    const T r = xsign_v(idx == (uint32_t)q0 ? nBk : nAk, un, mv);
                    un <<= 1;
                    const uint32_t zz = zb[k] + (V[q0] >> 18);
                    at((V[q0] & 0x3ffffu) + min(zz, zz - ZT)) = r;
                }
            });
        }
        if (fail) word(FL_B) = (uint32_t)(it + 1);
        lds_barrier();
        if (word(FL_B) != (uint32_t)(it + 1)) {
            // ---- the syndrome of LQ_old holds (:112-114): its hard decisions are the output
#pragma unroll
            for (int k = 0; k < CPT; ++k)
                if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(at(cq[k]) < T(0));
#pragma unroll
            for (int k = 0; k < RPT; ++k)
                if (t + k * NT < NR && ri[k] >= 4)
                    crow[(KB + ri[k]) * Zc + (int)(zb[k] / TS)] = (int8_t)((hdx >> k) & 1u);
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        // ---- LQ = LLRin + Lr.sum(axis=0) (:126): core columns, rows ascending (consecutive
        //      message slots, four reads in flight)
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            if (t + k * NT >= NC) continue;
            const int n = cn[k];
            uint32_t o = cr[k];
            T acc = T(0) + at(o);
            int p = 1;
            for (; p + 4 <= n; p += 4) {
                const T v0 = at(o + ZT), v1 = at(o + 2 * ZT), v2 = at(o + 3 * ZT), v3 = at(o + 4 * ZT);
                o += 4 * ZT;
                acc = acc + v0;
                acc = acc + v1;
                acc = acc + v2;
                acc = acc + v3;
            }
            for (; p < n; ++p) {
                o += ZT;
                acc = acc + at(o);
            }
            const T v = (cpun[k] ? T(0) : lf[k]) + acc;   // punctured columns: LLR 0 (:43)
            at(cq[k]) = v, at(cq[k] + ZT) = v;
        }
        lds_barrier();
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    bool fail = false;
    uint32_t ox = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (t + k * NT >= NR) continue;
        const int e0 = re0[k], d = rd[k];
        const bool xe = ri[k] >= 4;
        const int dc = d - (xe ? 1 : 0);
        bool par = false;
        if (xe) {   // the extension edge is the row's last: LLR + its r
            const T rx = xsign_v((wd[k] >> 24) == (uint32_t)dc ? nB[k] : nA[k], wd[k] << 31, mv);
            const bool b = xl[k] + rx <= T(0);
            ox |= (uint32_t)b << k;
            par = b;
        }
        uint32_t W[DMAX];
#pragma unroll
        for (int x = 0; x < DMAX; ++x) W[x] = word(RW_B + 4u * (uint32_t)(e0 + (x < dc ? x : 0)));
        sfor<0, DMAX>([&](auto xc) {
            constexpr int x = decltype(xc)::value;
            const bool b = at(W[x] + zb[k]) <= T(0);
            par ^= x < dc && b;
        });
        fail |= par;
    }
    if (fail) word(FL_B + 4) = 1u;
    lds_barrier();
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(at(cq[k]) <= T(0));
#pragma unroll
    for (int k = 0; k < RPT; ++k)
        if (t + k * NT < NR && ri[k] >= 4) crow[(KB + ri[k]) * Zc + (int)(zb[k] / TS)] = (int8_t)((ox >> k) & 1u);
    if (t == 0) status[cb] = word(FL_B + 4) == 0u, iters[cb] = L;
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
    const size_t lds = kLdsPerCU;   // one attribute value for every Zc (the launch asks for what it needs)
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
