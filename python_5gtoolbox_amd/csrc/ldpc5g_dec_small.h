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
// LDS (small_lds_bytes_t): the doubled LQ of the core columns, the +inf / discard / zero rows and one
// message per core edge, (2*KC + 2 + Ec + 2)*Zc values, plus the edge words: 2,640*Zc + 7,008 B for
// BG1 float64, so the largest BG1 float64 lifting size that fits the CU's 160 KB is Zc = 56 (154.8 KB;
// BG1 float64 Zc = 60 / 64 run the batch kernel's 16-part configuration instead).
#pragma once
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {
namespace {

constexpr int kSmallMaxZc = 64;
// development instrumentation (tools/small_dev): thread 0's cycle counter at phase boundaries
#ifdef LDPC5G_SMALL_TS
#define SMALL_TS(n) \
    if (t == 0 && (n) < 16) tsv[(n)] = __builtin_amdgcn_s_memtime()
#define SMALL_TS_DUMP() \
    if (t == 0) { for (int q_ = 0; q_ < 16; ++q_) ((uint64_t*)crow)[q_] = tsv[q_]; }
#else
#define SMALL_TS(n)
#define SMALL_TS_DUMP()
#endif
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
    int ncore = 0, dmax = 0, cmax = 0;
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
        for (int j = 0; j < P::KC; ++j) cmax = cmax > cstart[j + 1] - cstart[j] ? cmax : cstart[j + 1] - cstart[j];
    }
};
template <int BG>
__device__ constexpr SmallPlan<BG> kSmallPlanD{};
template <int BG>
constexpr SmallPlan<BG> kSmallPlanH{};

// LDS bytes: LQ twice per core column (entries z and z + Zc hold LQ of row z, so a read at z + V
// mod Zc needs no wrap), a +inf column (the reads of a row's padding edges), one message per core
// edge and a discard slot row (the padding edges' writes), two words per (row, edge < DMAX), flags
template <int BG, typename T>
constexpr size_t small_lds_bytes_t(int Zc) {
    using P = BGT<BG>;
    return (size_t)(2 * P::KC + 2 + kSmallPlanH<BG>.ncore + 2) * Zc * sizeof(T) +
           (size_t)(2 * P::MB * kSmallPlanH<BG>.dmax + 4) * 4;
}

template <int BG, typename T, bool OFS, int RPT, int NP>
__global__ __launch_bounds__(kSmallMaxThreads) void ldpc_small_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int Zc, int zi, int64_t ldl, int64_t ldc, int L, T alpha, T beta,
    int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E, TS = sizeof(T);
    constexpr int NCE = kSmallPlanH<BG>.ncore, DMAX = kSmallPlanH<BG>.dmax;
    constexpr int CPT = small_cpt<RPT>();
    static_assert(NP == 1 || (NP == 2 && RPT == 1), "two parts per check node only with one node per pair");
    // NP = 2: a check node's edges are split between two neighbouring lanes (edges [0, DH) and
    // [DH, 2 DH)), whose partial two-min / argmin / sign states are merged with one DPP exchange —
    // half the serial chain per node for the smallest codes (BASELINE config 1)
    constexpr int DH = (DMAX + NP - 1) / NP;
    constexpr int CH = RPT == 1 ? 10 : 5;   // LQ reads in flight together
    constexpr int CMAX = kSmallPlanH<BG>.cmax, CCH = RPT == 1 ? 10 : 5;   // column degree; reads in flight
    extern __shared__ __align__(16) unsigned char smem[];
    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem != 0u)
        __builtin_trap();   // the byte-offset LDS addressing below assumes a zero base
    using lds_T = __attribute__((address_space(3))) T;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    auto at = [&](uint32_t byte) -> lds_T& { return *(lds_T*)(uintptr_t)byte; };
    auto word = [&](uint32_t byte) -> lds_u32& { return *(lds_u32*)(uintptr_t)byte; };
    const uint32_t ZT = (uint32_t)(Zc * TS);
    // byte offsets: LQ2 [KC][2 Zc] | +inf [2 Zc] | LR [NCE][Zc] | discard [Zc] | zeros [Zc] |
    // read words [MB][DMAX] | write words [MB][DMAX] | flags
    const uint32_t INF_B = 2u * KC * ZT, LR_B = INF_B + 2u * ZT, DIS_B = LR_B + (uint32_t)NCE * ZT;
    const uint32_t ZR_B = DIS_B + ZT;   // a row of +0.0: the padding reads of the column pass
    const uint32_t RW_B = ZR_B + ZT, WW_B = RW_B + 4u * MB * DMAX, FL_B = WW_B + 4u * MB * DMAX;

    const int cb = blockIdx.x;
    const T* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    const int t = threadIdx.x, NT = blockDim.x;
    const int NR = MB * Zc * NP, NC = KC * Zc;   // NR: (check node, part) slots
    const int part = NP == 2 ? (t & 1) : 0;
#ifdef LDPC5G_SMALL_TS
    uint64_t tsv[16] = {};
#endif
    SMALL_TS(0);

    // ---- edge words per (row i, edge x < DMAX), one thread each (a single round trip to the
    //      constant tables).  Read word: byte offset of LQ2 entry (column j, row V mod Zc) relative to
    //      row z; write word: byte offset of the message slot (CSC position p) | (V mod Zc)*TS << 18.
    //      Padding edges (x >= the row's core degree) read +inf and write the discard row, so every
    //      row runs the same branch-free DMAX-edge sequence.
    for (int q = t; q < MB * DMAX; q += NT) {
        const int i = q / DMAX, x = q - i * DMAX;
        const int e0 = row_start_d<BG>(i), dc = row_start_d<BG>(i + 1) - e0 - (i >= 4 ? 1 : 0);
        uint32_t rw = INF_B, ww = DIS_B;
        if (x < dc) {
            const uint32_t w0 = kSmallPlanD<BG>.ew[e0 + x];
            const uint32_t sb = (uint32_t)shift_of<BG>(zi, e0 + x) * TS;
            rw = 2u * (w0 & 0xffu) * ZT + sb;
            ww = (LR_B + (w0 >> 8) * ZT) | (sb << 18);
        }
        word(RW_B + 4u * q) = rw;
        word(WW_B + 4u * q) = ww;
    }
    for (int z = t; z < 2 * Zc; z += NT) at(INF_B + (uint32_t)z * TS) = FT<T>::inf();
    for (int z = t; z < Zc; z += NT) at(ZR_B + (uint32_t)z * TS) = T(0);
    if (t == 0) word(FL_B) = 0u, word(FL_B + 4) = 0u;
    // own core column entries c = j*Zc + z': LLR, CSC range, LQ2 / message byte offsets
    T lf[CPT];
    uint32_t cq[CPT], cr[CPT], cz0[CPT];
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
        cz0[k] = ZR_B + (uint32_t)z * TS;
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
        const int r = (t + k * NT) / NP;   // check node
        ri[k] = r < NR / NP ? r / Zc : 0;
        const int z = r - ri[k] * Zc;
        zb[k] = (uint32_t)z * TS;
        re0[k] = (int)(RW_B + 4u * (uint32_t)(ri[k] * DMAX));   // the row's read words
        rd[k] = row_start_d<BG>(ri[k] + 1) - row_start_d<BG>(ri[k]);
        nA[k] = T(0), nB[k] = T(0), wd[k] = 0u;
        xl[k] = (r < NR / NP && ri[k] >= 4) ? lrow[(KB + ri[k] - pc) * Zc + z] : T(0);
    }
    lds_barrier();
    SMALL_TS(1);
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
            const uint32_t rwb = (uint32_t)re0[k];
            const int d = rd[k];
            const bool xe = ri[k] >= 4;   // rows >= 4: the last edge is the extension column
            const int dc = d - (xe ? 1 : 0);
            // the row's DMAX read words (LDS broadcasts within a row) and LQ reads, all in flight
            // before the first is used; padding edges read +inf, which leaves the two-min, the argmin,
            // the sign product and the parity unchanged
            // this part's edges [x0, x0 + DH)
            const uint32_t x0 = (uint32_t)(part * DH);
            uint32_t W[DH];
            sfor<0, DH>([&](auto xc) {
                constexpr int x = decltype(xc)::value;
                W[x] = x < DMAX - (NP - 1) * DH || NP == 1 ? word(rwb + 4u * (x0 + x))
                                                           : (part ? word(RW_B + 4u * MB * DMAX - 4u) : word(rwb + 4u * x));
            });
            uint32_t u = (wd[k] << (32 - d)) << x0;
            const uint32_t idxo = wd[k] >> 24;
            const T mA = nA[k], mB = nB[k];
            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0;
            bool par = false;
            auto edge = [&](uint32_t q0, T av, T rold) {
                par ^= av < T(0);
                const T q = av - rold;
                const T aq = fabs(q);
                idx = aq < min1 ? q0 : idx;
                asm volatile("" : "+v"(idx));   // update in place (no sunk select chain)
                negs = __builtin_amdgcn_alignbit(negs, FT<T>::sbits(q), 31);
                two_min(min1, min2, aq);
                sx ^= FT<T>::sbits(q);
            };
            sfor<0, (DH + CH - 1) / CH>([&](auto cc) {
                constexpr int c0 = decltype(cc)::value * CH, c1 = c0 + CH < DH ? c0 + CH : DH;
                T a[CH];
                sfor<c0, c1>([&](auto xc) { a[decltype(xc)::value - c0] = at(W[decltype(xc)::value] + zb[k]); });
                sfor<c0, c1>([&](auto xc) {
                    constexpr int x = decltype(xc)::value;
                    const uint32_t q0 = x0 + x;
                    const T rold = xsign_v(idxo == q0 ? mB : mA, u, mv);
                    asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1, all-VGPR form
                    edge(q0, a[x - c0], rold);
                });
            });
            if constexpr (NP == 2) {
                // merge with the partner lane (t ^ 1): part 0 holds edges [0, DH), part 1 [DH, 2DH)
                auto xchg = [](uint32_t v) -> uint32_t {
                    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
                };
                auto xchgT = [&](T v) -> T {
                    if constexpr (sizeof(T) == 8) {
                        const uint32_t lo = xchg((uint32_t)__double2loint(v)), hi = xchg((uint32_t)__double2hiint(v));
                        return __hiloint2double((int)hi, (int)lo);
                    } else {
                        return __uint_as_float(xchg(__float_as_uint(v)));
                    }
                };
                const T o1 = xchgT(min1), o2 = xchgT(min2);
                const uint32_t oidx = xchg(idx), onegs = xchg(negs), osx = xchg(sx), opar = xchg((uint32_t)par);
                const T a1 = part ? o1 : min1, b1 = part ? min1 : o1;   // a: edges [0, DH), b: [DH, 2DH)
                const T a2 = part ? o2 : min2, b2 = part ? min2 : o2;
                const uint32_t ia = part ? oidx : idx, ib = part ? idx : oidx;
                const uint32_t na = part ? onegs : negs, nb = part ? negs : onegs;
                idx = b1 < a1 ? ib : ia;   // the first occurrence of the minimum (ties: part a)
                min2 = fmin(fmin(a2, b2), fmax(a1, b1));
                min1 = fmin(a1, b1);
                negs = (na << DH) | nb;
                sx ^= osx;
                par ^= (opar & 1u) != 0;
            }
            // the extension edge (the row's last: sign bit 0 of the stored word); rows 0..3 run it
            // on +inf like a padding edge.  LQ of the degree-1 column = LLR + its only r
            negs >>= (uint32_t)(NP * DH - dc);   // drop the padding edges' (positive) sign bits
            {
                const T rold = xsign_v(idxo == (uint32_t)dc ? mB : mA, wd[k] << 31, mv);
                const T av = xe ? xl[k] + rold : FT<T>::inf();
                hdx |= (uint32_t)(av < T(0)) << k;
                edge(dc, av, rold);
            }
            negs >>= (uint32_t)(xe ? 0 : 1);   // rows 0..3: no extension edge
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
            // the new messages of the core edges into their slots at row (z + V) mod Zc (padding
            // edges: the discard row)
            uint32_t un = (wd[k] << (32 - d)) << x0;
            uint32_t V[DH];
            sfor<0, DH>([&](auto xc) {
                constexpr int x = decltype(xc)::value;
                V[x] = x < DMAX - (NP - 1) * DH || NP == 1 ? word(rwb + (WW_B - RW_B) + 4u * (x0 + x))
                                                           : (part ? (uint32_t)DIS_B : word(rwb + (WW_B - RW_B) + 4u * x));
            });
            sfor<0, DH>([&](auto xc) {
                constexpr int x = decltype(xc)::value;
                const T r = xsign_v(idx == x0 + x ? nBk : nAk, un, mv);
                asm("v_add_u32 %0, %1, %1" : "=v"(un) : "v"(un));
                const uint32_t zz = zb[k] + (V[x] >> 18);
                at((V[x] & 0x3ffffu) + min(zz, zz - ZT)) = r;
            });
        }
        if (fail) word(FL_B) = (uint32_t)(it + 1);
        lds_barrier();
        SMALL_TS(3 + 3 * it);
        if (word(FL_B) != (uint32_t)(it + 1)) {
            // ---- the syndrome of LQ_old holds (:112-114): its hard decisions are the output
#pragma unroll
            for (int k = 0; k < CPT; ++k)
                if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(at(cq[k]) < T(0));
#pragma unroll
            for (int k = 0; k < RPT; ++k)
                if (t + k * NT < NR && ri[k] >= 4 && part == 0)
                    crow[(KB + ri[k]) * Zc + (int)(zb[k] / TS)] = (int8_t)((hdx >> k) & 1u);
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        // ---- LQ = LLRin + Lr.sum(axis=0) (:126): core columns, rows ascending (consecutive
        //      message slots).  Every column runs CMAX adds, the ones past its degree adding +0.0
        //      from the zero row: exact (acc = 0 + r0 + ... is never -0.0), and branch-free, so
        //      the reads of a chunk are all in flight together
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            if (t + k * NT >= NC) continue;
            const int n = cn[k];
            const uint32_t o = cr[k], oz = cz0[k];
            T acc = T(0);
            sfor<0, (CMAX + CCH - 1) / CCH>([&](auto cc) {
                constexpr int p0 = decltype(cc)::value * CCH, p1 = p0 + CCH < CMAX ? p0 + CCH : CMAX;
                T v[CCH];
                sfor<p0, p1>([&](auto pc) {
                    constexpr int p = decltype(pc)::value;
                    v[p - p0] = at(p < n ? o + (uint32_t)p * ZT : oz);
                });
                sfor<p0, p1>([&](auto pc) { acc = acc + v[decltype(pc)::value - p0]; });
            });
            const T v = (cpun[k] ? T(0) : lf[k]) + acc;   // punctured columns: LLR 0 (:43)
            at(cq[k]) = v, at(cq[k] + ZT) = v;
        }
        SMALL_TS(4 + 3 * it);
        lds_barrier();
    }
    SMALL_TS(14);

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    bool fail = false;
    uint32_t ox = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (t + k * NT >= NR) continue;
        const uint32_t rwb = (uint32_t)re0[k];
        const int d = rd[k];
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
        sfor<0, DMAX>([&](auto xc) { W[decltype(xc)::value] = word(rwb + 4u * decltype(xc)::value); });
        sfor<0, DMAX>([&](auto xc) { par ^= at(W[decltype(xc)::value] + zb[k]) <= T(0); });   // +inf: false
        fail |= par;
    }
    if (fail) word(FL_B + 4) = 1u;
    lds_barrier();
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        if (t + k * NT < NC) crow[t + k * NT] = (int8_t)(at(cq[k]) <= T(0));
#pragma unroll
    for (int k = 0; k < RPT; ++k)
        if (t + k * NT < NR && ri[k] >= 4 && part == 0)
            crow[(KB + ri[k]) * Zc + (int)(zb[k] / TS)] = (int8_t)((ox >> k) & 1u);
    if (t == 0) status[cb] = word(FL_B + 4) == 0u, iters[cb] = L;
    SMALL_TS(15);
    SMALL_TS_DUMP();
}

template <int BG, typename T, bool OFS, int RPT, int NP>
constexpr auto small_kernel() { return ldpc_small_kernel<BG, T, OFS, RPT, NP>; }

template <int BG, typename T>
bool small_fits(int Zc) {
    return Zc <= kSmallMaxZc && small_lds_bytes_t<BG, T>(Zc) <= kLdsPerCU;
}

template <int BG, typename T, int RPT, int NP>
int launch_small_rpt(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                     int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, int threads,
                     hipStream_t st) {
    const bool ofs = beta != 0.0;
    auto kern = ofs ? ldpc_small_kernel<BG, T, true, RPT, NP> : ldpc_small_kernel<BG, T, false, RPT, NP>;
    const size_t lds = kLdsPerCU;   // one attribute value for every Zc (the launch asks for what it needs)
    if (int rc = ofs ? set_lds_once<small_kernel<BG, T, true, RPT, NP>()>(lds)
                     : set_lds_once<small_kernel<BG, T, false, RPT, NP>()>(lds))
        return rc;
    const size_t lds_zc = small_lds_bytes_t<BG, T>(Zc);
    hipLaunchKernelGGL(kern, dim3(B), dim3(threads), lds_zc, st, llr, ck, status, iters, Zc, zi, ldl, ldc, L,
                       (T)alpha, (T)beta, pc);
    return check_hip(hipGetLastError(), "ldpc_small_kernel launch");
}

// one codeblock per workgroup, B workgroups; the caller checks small_fits.  Check nodes per thread
// RPT = 1..3 as Zc grows; for the smallest codes (2 * MB * Zc <= 1024) two lanes per node.
template <int BG, typename T>
int launch_small_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                   int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    const int nodes = BGT<BG>::MB * Zc;
    if (2 * nodes <= kSmallMaxThreads)
        return launch_small_rpt<BG, T, 1, 2>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc,
                                             ((2 * nodes + 63) / 64) * 64, st);
    const int threads = std::min(kSmallMaxThreads, ((nodes + 63) / 64) * 64);
    const int rpt = (nodes + threads - 1) / threads;
    if (!small_fits<BG, T>(Zc) || rpt > kSmallMaxRpt || BGT<BG>::KC * Zc > (rpt == 1 ? 1 : 2) * threads)
        return fail(LDPC5G_ESIZE, "small-codeblock decoder: Zc=%d does not fit", Zc);
    if (rpt == 1)
        return launch_small_rpt<BG, T, 1, 1>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
    if (rpt == 2)
        return launch_small_rpt<BG, T, 2, 1>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
    return launch_small_rpt<BG, T, 3, 1>(llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, threads, st);
}

}  // namespace
}  // namespace ldpc5g_impl
