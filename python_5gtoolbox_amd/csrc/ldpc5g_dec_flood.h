// ldpc5g_dec_flood.h — flooding min-sum decoder (py5gphy/ldpc/nr_ldpc_decode.py:51-143 with
// _min_sum_process :178-227), float64 (bit-identical to the reference) and float32.
//
// One iteration of the reference computes every check-to-variable message Lr from Lq = LQ_old - Lr_old
// (:117-123), then LQ_new = LLRin + Lr.sum(axis=0) (:126), a row-ascending sum per column.  The
// kernel splits it the same way:
//   phase A  every base row reads LQ_old (LDS, read-only in this phase, no barrier between rows),
//            forms q = LQ_old - r_old edge by edge and keeps only the new compressed row state
//            (nA = alpha*max(min1-beta,0), nB = ... min2, per-edge signs, argmin);  the syndrome
//            of the hard decisions of LQ_old (:107-114) falls out of the same reads;
//   phase B  the messages r are rebuilt from the new state and summed into the SAME LDS array
//            (LQ_old is dead now) in row-ascending order, one barrier per group of column-disjoint
//            rows; the first row of each column writes 0 + r instead of adding;
//   then     LQ = LLR + sum for the thread's own entries.
// So one f64 array of the Kb+4 core columns (80 KB at Zc = 384) is the whole LDS image of LQ, and
// the remaining LDS holds the state of the first rows.  Every thread slot (z, codeblock) has two
// threads, one per half of the 768-thread workgroup (6 waves each, 3 waves per SIMD): the base rows
// are split between the halves (phase-A edge counts balanced, the rows of a multi-row group on
// different halves so phase B stays balanced), so each thread holds the state of ~half the rows
// in VGPRs.  Rows whose state lives in LDS are summed by both halves (alternate edges) in phase B.
#pragma once
#include "ldpc5g_dec_body.h"

namespace ldpc5g_impl {
namespace {

constexpr size_t kLdsPerCU = 160 * 1024;
// 1: float64 Zc = 384 batches run the frame kernel (ldpc5g_dec_frame.h) and this header's Zc = 384
// float64 instantiation is not built; 0 (tools/flood_dev A/B builds): this kernel again
#ifndef LDPC5G_FLOOD_FRAME
#define LDPC5G_FLOOD_FRAME 1
#endif
#ifndef LDPC5G_FLOOD_XPRE
#define LDPC5G_FLOOD_XPRE 4
#endif
// extension-column LLRs are loaded this many ext rows ahead of their use in phase A
constexpr int kXPre = LDPC5G_FLOOD_XPRE;
// phase A: core-edge LQ reads issued this many edges ahead (0: at their use), and whether a
// scheduling barrier pins each read before the arithmetic of the edge it overlaps (r04: one edge
// ahead + barrier 4.205 -> 4.041 ms per 4096 f64 codeblocks; 2 or 3 ahead 4.06 ms)
#ifndef LDPC5G_FLOOD_APRE
#define LDPC5G_FLOOD_APRE 1
#endif
#ifndef LDPC5G_FLOOD_ASB
#define LDPC5G_FLOOD_ASB 1
#endif
constexpr int kAPre = LDPC5G_FLOOD_APRE;
// phase A: the row sign product from the parity of the packed sign bits (one v_bcnt per row instead
// of an XOR per edge: r05 3.627 -> 3.549 ms per 4096 f64 codeblocks)
#ifndef LDPC5G_FLOOD_SXPOP
#define LDPC5G_FLOOD_SXPOP 1
#endif
constexpr bool kSxPop = LDPC5G_FLOOD_SXPOP != 0;
// (variants measured and dropped — rows of a part paired with interleaved edges, phase-B sign words
// shifted per added edge, phase-B table offsets, sign-word syndrome parity: DESIGN.md §4.2b)
constexpr bool kASb = LDPC5G_FLOOD_ASB != 0;
// phase A takes its rotated core-edge offsets from an LDS wrap table (one LDS read issued two edges
// ahead instead of the add/add/min arithmetic: 3 half-rate VALU ops per edge) in the batch
// kernels (2 parts x 384 slots), whose LDS has room for it (2 x 384 u32 entries; the numbers of
// LDS state rows do not change; float64 BG2 Zc=384 2.97 -> 2.78 ms per 4096 codeblocks, float32
// BG1 Zc=384 1.18 -> 1.31 M CB/s).
// r04: 4.04 -> 3.93 ms per 4096 codeblocks.  (Phase B keeps the arithmetic: a table read there
// adds an LDS round trip to each barrier-separated row group, measured 4.08 ms.)
template <int BG, typename T, int NP, int CS>
constexpr bool flood_wtab() { return NP == 2 && CS == 384; }
template <int BG, typename T, int NP, int CS>
constexpr int flood_wtab_bytes() { return flood_wtab<BG, T, NP, CS>() ? 2 * CS * 4 : 0; }
// ZCC > 0 (zc_shift, ldpc5g_dec_body.h): a kernel for the one lifting size Zc = 384 = CS, one
// codeblock per workgroup, r04: 3.93 -> 3.64 ms per 4096 codeblocks

// Row plan of a workgroup of NP parts x CS slots (constexpr): which part runs each row, where its
// state lives, and the packing of its sign word.  NP = 2, CS = 384 for batches; NP = 16, CS = 64 for
// the small launches of the per-codeblock drop-ins (16 waves share one codeblock's rows).
template <int BG, typename T, int NP, int CS>
struct FloodPlan {
    int nls = 0;          // rows 0..nls-1 keep their state in LDS
    int owner[64] = {};   // part that runs phase A of row i (and phase B of a VGPR row)
    int slot[64] = {};    // VGPR state slot of row i in its owner part (-1: LDS row)
    int nslot = 0;
    int pw[64] = {};      // VGPR sign word of row i: rows of degree <= 12 share a word (16-bit fields)
    int ph[64] = {};      // 0: whole word (negs | idx << 24), 1: low field, 2: high field (negs | idx << 12)
    int npw = 0;
    int first_row[32] = {};   // lowest base row of core column j (writes 0 + r in phase B)
    int xpos[64] = {};        // rank of ext row i (i >= 4) among its owner part's ext rows
    int xlist[NP][64] = {};   // ext rows of each part, ascending
    int nx[NP] = {};
    static constexpr int deg(int i) { return BGT<BG>::RS[i + 1] - BGT<BG>::RS[i]; }
    constexpr FloodPlan() {
        using P = BGT<BG>;
        const auto& G = kGroups<BG>;
        const size_t fixed = (size_t)P::KC * CS * sizeof(T) + (2 * kMaxG + 4) * 4 + flood_wtab_bytes<BG, T, NP, CS>();
        const int fit = (int)((kLdsPerCU - fixed) / (CS * (2 * sizeof(T) + 4)));
        int lead = 0;   // leading single-row groups: their phase B is split only if in LDS
        while (lead < G.n && G.start[lead + 1] - G.start[lead] == 1 && G.start[lead] == lead) ++lead;
        nls = fit < lead ? fit : lead;
        int load[NP] = {};
        bool done[64] = {};
        // rows of a multi-row group on different parts (phase B balance), then every other row
        // by decreasing degree onto the least loaded part (phase A balance)
        for (int g = 0; g < G.n; ++g) {
            if (G.start[g + 1] - G.start[g] < 2) continue;
            int gl[NP] = {};
            for (;;) {
                int best = -1;
                for (int i = G.start[g]; i < G.start[g + 1]; ++i)
                    if (!done[i] && (best < 0 || deg(i) > deg(best))) best = i;
                if (best < 0) break;
                int h = 0;
                for (int q = 1; q < NP; ++q)
                    if (gl[q] < gl[h] || (gl[q] == gl[h] && load[q] < load[h])) h = q;
                owner[best] = h, gl[h] += deg(best), load[h] += deg(best), done[best] = true;
            }
        }
        for (;;) {
            int best = -1;
            for (int i = 0; i < P::MB; ++i)
                if (!done[i] && (best < 0 || deg(i) > deg(best))) best = i;
            if (best < 0) break;
            int h = 0;
            for (int q = 1; q < NP; ++q)
                if (load[q] < load[h]) h = q;
            owner[best] = h, load[h] += deg(best), done[best] = true;
        }
        int ns[NP] = {};
        for (int i = 0; i < P::MB; ++i) slot[i] = i < nls ? -1 : ns[owner[i]]++;
        for (int q = 0; q < NP; ++q) nslot = nslot > ns[q] ? nslot : ns[q];
        for (int hh = 0; hh < NP; ++hh) {
            int n = 0, open = -1;
            for (int i = nls; i < P::MB; ++i) {
                if (owner[i] != hh) continue;
                if (deg(i) > 12) {
                    pw[i] = n++, ph[i] = 0;
                } else if (open >= 0) {
                    pw[i] = open, ph[i] = 2, open = -1;
                } else {
                    open = n, pw[i] = n++, ph[i] = 1;
                }
            }
            npw = npw > n ? npw : n;
        }
        for (int i = 4; i < P::MB; ++i) {
            xpos[i] = nx[owner[i]];
            xlist[owner[i]][nx[owner[i]]++] = i;
        }
        for (int j = 0; j < P::KC; ++j) {
            first_row[j] = -1;
            for (int i = 0; i < P::MB && first_row[j] < 0; ++i)
                for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                    if (P::COL[e] == j) first_row[j] = i;
        }
    }
};
template <int BG, typename T, int NP, int CS>
constexpr FloodPlan<BG, T, NP, CS> kFloodPlan{};

// every core column's first row is one of rows 0..3 (which have no extension column): a dead
// extension row never initialises a column sum in phase B, so skipping its adds is exact
template <int BG>
constexpr bool first_rows_core() {
    for (int j = 0; j < BGT<BG>::KC; ++j) {
        int f = -1;
        for (int i = 0; i < BGT<BG>::MB && f < 0; ++i)
            for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i + 1]; ++e)
                if (BGT<BG>::COL[e] == j) f = i;
        if (f < 0 || f >= 4) return false;
    }
    return true;
}
static_assert(first_rows_core<1>() && first_rows_core<2>(), "dead-row skipping needs core first rows");

template <int BG, typename T, int NP, int CS>
constexpr size_t flood_lds_bytes_t() {
    return (size_t)BGT<BG>::KC * CS * sizeof(T) + (size_t)kFloodPlan<BG, T, NP, CS>.nls * CS * (2 * sizeof(T) + 4) +
           (2 * kMaxG + 4) * 4 + flood_wtab_bytes<BG, T, NP, CS>();
}

// x with its sign flipped by bit 31 of u (all-VGPR v_bitop3: x ^ (u & mv), mv = 0x80000000)
__device__ __forceinline__ float xsign_v(float x, uint32_t u, uint32_t mv) {
    return __uint_as_float(__builtin_amdgcn_bitop3_b32(u, __float_as_uint(x), mv, 0x6c));
}
__device__ __forceinline__ double xsign_v(double x, uint32_t u, uint32_t mv) {
    const uint32_t hi = __builtin_amdgcn_bitop3_b32(u, (uint32_t)__double2hiint(x), mv, 0x6c);
    return __hiloint2double((int)hi, __double2loint(x));
}
template <int BG>
__device__ __forceinline__ const uint32_t* shift_row(int zi) {
    if constexpr (BG == 1) return kBG1ShiftMod[zi];
    else return kBG2ShiftMod[zi];
}
// c ? a : b on values (a conditional on two lvalues may become a select of their addresses, which
// keeps the state arrays out of registers)
template <typename T>
__device__ __forceinline__ T pick(bool c, T a, T b) { return c ? a : b; }
// two-min update with min1 <= min2 (values are selected, never rounded: any form is exact)
__device__ __forceinline__ void two_min(float& m1, float& m2, float a) {
    m2 = __builtin_amdgcn_fmed3f(m1, m2, a);
    m1 = fminf(m1, a);
}
__device__ __forceinline__ void two_min(double& m1, double& m2, double a) {
    m2 = fmin(m2, fmax(m1, a));
    m1 = fmin(m1, a);
}

template <int BG, typename T, bool OFS, int NP, int CS, bool DEAD, int ZCC = 0>
__device__ __forceinline__ void flood_body(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int B, int Zc_u, int zi_u, int G_u, int64_t ldl, int64_t ldc,
    int L, T alpha, T beta, int pc, const DecWork* __restrict__ work,
    const CbRef* __restrict__ cbs) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, TS = sizeof(T);
    constexpr int NLS = kFloodPlan<BG, T, NP, CS>.nls;
    constexpr int NS = kFloodPlan<BG, T, NP, CS>.nslot > 0 ? kFloodPlan<BG, T, NP, CS>.nslot : 1;
    constexpr int NPW = kFloodPlan<BG, T, NP, CS>.npw > 0 ? kFloodPlan<BG, T, NP, CS>.npw : 1;
    constexpr int ST_B = KC * CS * TS;               // LDS rows: (mA, mB) pairs
    constexpr int PK_B = ST_B + NLS * CS * 2 * TS;   // LDS rows: sign/argmin words
    constexpr int FLAG_B = PK_B + NLS * CS * 4;
    constexpr int KH = (KC + NP - 1) / NP;   // own columns [h*KH, (h+1)*KH) are part h's
    extern __shared__ __align__(16) unsigned char smem[];

    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem != 0u)
        __builtin_trap();   // the byte-offset LDS addressing below assumes a zero base
    int Zc = Zc_u, zi = zi_u, G = G_u;
    const int t = threadIdx.x;
    const int H = (int)blockDim.x / NP;   // slots per part, a multiple of 64 (<= CS)
    const int h = __builtin_amdgcn_readfirstlane(t / H);
    const int s = t - h * H;
    if (work) {
        DecWork w = work[blockIdx.x];
        Zc = w.Zc, zi = w.zi, G = w.G;
    }
    constexpr bool kZ = ZCC > 0;   // compile-time lifting size (see zc_shift)
    static_assert(!kZ || (ZCC == CS && flood_wtab<BG, T, NP, CS>()), "Zc-specialised kernel: Zc = CS, wrap table");
    constexpr bool WT = flood_wtab<BG, T, NP, CS>();
    if constexpr (kZ) Zc = ZCC, G = 1;
    // slot s = z*G + cl owns row z of codeblock slot cl; LDS column entries are interleaved the
    // same way (entry (z, cl) at byte (z*G + cl)*TS), so a cyclic shift never crosses CB slots
    const int z = s / G;
    const int cbl = s - z * G;
    bool valid = z < Zc;
    const T* lrow = llr;
    int8_t* crow = ck;
    int out = 0;
    if (valid) {
        if (work) {
            CbRef r = cbs[work[blockIdx.x].first + cbl];
            lrow = llr + r.llr_off;
            crow = ck + r.ck_off;
            out = r.out;
        } else {
            const int cb = blockIdx.x * G + cbl;   // slots past the batch keep lrow = llr
            valid = cb < B;
            if (valid) {
                lrow = llr + (int64_t)cb * ldl;
                crow = ck + (int64_t)cb * ldc;
                out = cb;
            }
        }
    }
    const int cl = valid ? cbl : 0;
    // LLR loads as saddr accesses: a workgroup-uniform base (the work item's first codeblock, its
    // lowest row: build_plan sorts them) plus a 32-bit per-lane byte offset (< 4 GiB: checked by
    // launch_flood_cfg / the plan) — as the layered kernel (ldpc5g_dec_body.h)
    const T* lbase;
    uint32_t lofs = 0;
    if (work) {
        lbase = llr + cbs[work[blockIdx.x].first].llr_off;
        if (valid) lofs = (uint32_t)((lrow - lbase) * TS);
    } else {
        lbase = llr + (int64_t)blockIdx.x * G * ldl;
        if (valid) lofs = (uint32_t)((int64_t)cl * ldl * TS);
    }
    // element e of column-major row position (uniform part `u`, this lane's entry `z`)
    auto ldl_at = [&](int u, int zz) -> T {
        using gT = const __attribute__((address_space(1))) T;
        using gB = const __attribute__((address_space(1))) unsigned char;
        gB* rowb = (gB*)(uintptr_t)lbase + (uint32_t)(u * TS);
        return *(gT*)(rowb + (lofs + (uint32_t)zz * (uint32_t)TS));
    };
    const int so = valid ? s : 0;
    const int tzb = so * TS;   // byte offset of this slot's own column entry
    const int zg = valid ? z : 0;   // loads issued without a branch stay in row 0 of CB 0
    int zv = zg, ziv = zi;
    constexpr int TBL_B = FLAG_B + (2 * kMaxG + 4) * 4;   // wrap table (WT)
    int* flagA = (int*)(smem + FLAG_B);
    int* anyf = flagA + 2 * kMaxG;
    int epoch = 0;
    auto block_any = [&](bool p) -> bool {
        ++epoch;
        if (p) *anyf = epoch;
        lds_barrier();
        return *anyf == epoch;
    };
    using lds_T = __attribute__((address_space(3))) T;
    using lds_V2 = __attribute__((address_space(3))) V2<T>;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    auto at = [&](int byte) -> lds_T& { return *(lds_T*)(uintptr_t)(uint32_t)byte; };
    auto own = [&](int j) -> lds_T& { return at(j * CS * TS + tzb); };
    auto llrx = [&](int i) -> T { return ldl_at((KB + i - pc) * Zc, zv); };   // ext column of row i
    auto per_half_init = [&](auto&& f) {
        sfor<0, NP>([&](auto pc_) {
            if (h == decltype(pc_)::value) f(pc_);
        });
    };

    // row state: (mA, mB) magnitudes, the signs of r_k (edge 0 in bit d-1) and the argmin edge;
    // VGPR rows of degree <= 12 keep signs | argmin << 12 in one 16-bit field of a shared word
    T sA[NS], sB[NS];
    uint32_t sP[NPW];
#pragma unroll
    for (int x = 0; x < NS; ++x) sA[x] = T(0), sB[x] = T(0);
#pragma unroll
    for (int x = 0; x < NPW; ++x) sP[x] = 0u;
    // u: bit 31 = sign of r_0 (u << k: of r_k), idx: argmin edge
    auto get_state = [&](auto ic, T& a, T& b, uint32_t& u, uint32_t& idx) {
        constexpr int i = decltype(ic)::value;
        constexpr int d = BGT<BG>::RS[i + 1] - BGT<BG>::RS[i];
        if constexpr (i < NLS) {
            const V2<T> v = *(lds_V2*)(uintptr_t)(uint32_t)(ST_B + (i * CS) * 2 * TS + 2 * tzb);
            a = v.x, b = v.y;
            const uint32_t p = *(lds_u32*)(uintptr_t)(uint32_t)(PK_B + (i * CS) * 4 + so * 4);
            u = p << (32 - d), idx = p >> 24;
            asm volatile("" : "+v"(idx));   // compare idx itself with inline constants k
        } else {
            constexpr int x = kFloodPlan<BG, T, NP, CS>.slot[i];
            constexpr int w = kFloodPlan<BG, T, NP, CS>.pw[i];
            constexpr int f = kFloodPlan<BG, T, NP, CS>.ph[i];
            a = sA[x], b = sB[x];
            const uint32_t p = sP[w];
            if constexpr (f == 0) u = p << (32 - d), idx = p >> 24;
            else if constexpr (f == 1) u = p << (32 - d), idx = (p >> 12) & 0xfu;
            else u = p << (16 - d), idx = p >> 28;
            asm volatile("" : "+v"(idx));
        }
    };
    auto put_state = [&](auto ic, T a, T b, uint32_t negs, uint32_t idx) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NLS) {
            V2<T> v;
            v.x = a, v.y = b;
            *(lds_V2*)(uintptr_t)(uint32_t)(ST_B + (i * CS) * 2 * TS + 2 * tzb) = v;
            *(lds_u32*)(uintptr_t)(uint32_t)(PK_B + (i * CS) * 4 + so * 4) = negs | (idx << 24);
        } else {
            constexpr int x = kFloodPlan<BG, T, NP, CS>.slot[i];
            constexpr int w = kFloodPlan<BG, T, NP, CS>.pw[i];
            constexpr int f = kFloodPlan<BG, T, NP, CS>.ph[i];
            sA[x] = a, sB[x] = b;
            if constexpr (f == 0) sP[w] = negs | (idx << 24);
            else if constexpr (f == 1) sP[w] = (sP[w] & 0xffff0000u) | negs | (idx << 12);
            else sP[w] = (sP[w] & 0xffffu) | (negs << 16) | (idx << 28);
        }
    };

    // ---- load: LQ = LLRin (:94), punctured columns 0 (:43); LDS row state 0; wrap table
    uint64_t nzx = 0;   // extension columns of this half's rows whose LLR is not +0.0 at this z
    if (valid) {
        // all loads issued before any is used: one HBM round trip (a conditional load per
        // punctured column made KH dependent round trips per workgroup)
        T v0[KH];
        sfor<0, KH>([&](auto jc) {
            const int j = min(h * KH + decltype(jc)::value, KC - 1);
            v0[decltype(jc)::value] = lrow[(j < pc ? 0 : j - pc) * Zc + z];
        });
        sfor<0, KH>([&](auto jc) {
            const int j = h * KH + decltype(jc)::value;
            if (j < KC) own(j) = j < pc ? T(0) : v0[decltype(jc)::value];
        });
        if constexpr (DEAD)
            per_half_init([&](auto hc) {
                sfor<4, MB>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (kFloodPlan<BG, T, NP, CS>.owner[i] == decltype(hc)::value)
                        nzx |= (uint64_t)(FT<T>::bits(llrx(i)) != 0) << (i - 4);
                });
            });
    }
    for (int w = t; w < NLS * CS; w += (int)blockDim.x) {
        V2<T> v;
        v.x = T(0), v.y = T(0);
        *(lds_V2*)(uintptr_t)(uint32_t)(ST_B + w * 2 * TS) = v;
        *(lds_u32*)(uintptr_t)(uint32_t)(PK_B + w * 4) = 0u;
    }
    if (s == 0 && h == 0)
        for (int c = 0; c < G; ++c) flagA[c] = 0;
    if constexpr (WT) {   // entry e (e < 2*Zc*G): byte offset of column entry e mod (Zc*G)
        const int ZG = Zc * G;
        if (t < ZG) {
            *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(uint32_t)(TBL_B + t * 4) = (uint32_t)(t * TS);
            *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(uint32_t)(TBL_B + (t + ZG) * 4) = (uint32_t)(t * TS);
        }
    }
    uint32_t* livew = (uint32_t*)(anyf + 2);   // workgroup OR of nzx (2 words)
    if (t == 0) *anyf = 0;
    if constexpr (DEAD)
        if (t == 0) livew[0] = 0u, livew[1] = 0u;
    bool active = valid;
    lds_barrier();
    // Dead extension rows (LLR +0.0 in every slot of the workgroup: untransmitted parity at high
    // code rates): q_ext = (0 + r) - r = +0, so every core message of the row is +-0 and its phase-B
    // adds change no column sum (their first rows are rows 0..3); only r_ext and the row's syndrome
    // bit matter.  rowA_dead computes exactly those; dead rows add nothing in phase B, and a group
    // of dead rows needs no barrier.  Bit-identical to running them (flooding has no ordering
    // between rows in phase A).
    uint64_t live_x = ~0ull;
    if constexpr (DEAD) {
        if (nzx & 0xffffffffu) atomicOr(&livew[0], (uint32_t)nzx);
        if (nzx >> 32) atomicOr(&livew[1], (uint32_t)(nzx >> 32));
        lds_barrier();
        live_x = ((uint64_t)__builtin_amdgcn_readfirstlane(livew[1]) << 32) |
                 (uint64_t)__builtin_amdgcn_readfirstlane(livew[0]);
    }
    auto rdead = [&](auto ic) -> bool {
        constexpr int i = decltype(ic)::value;
        if constexpr (!DEAD || i < 4) return false;
        else return ((live_x >> (i - 4)) & 1u) == 0;
    };
    auto gdead = [&](auto gc) -> bool {
        constexpr uint64_t m = group_xmask<BG>(decltype(gc)::value);
        if constexpr (!DEAD || m == 0) return false;
        else return (live_x & m) == 0;
    };

    // byte offset (without column base) of entry ((z + sft) mod Zc, cl): the unwrapped candidate,
    // or the wrapped one when it is valid (smaller as unsigned).  Arithmetic, not the layered
    // kernel's LDS wrap table: phase B is a chain of dependent LDS round trips per row group, and
    // a table lookup adds one (measured: 4.85 -> 4.53 ms per 4096 f64 codeblocks without it)
    const uint32_t GT = (uint32_t)(G * TS), tzbw = (uint32_t)tzb - (uint32_t)(Zc * G * TS);
    const uint32_t G4 = (uint32_t)(G * 4), tzT = (uint32_t)(TBL_B + so * 4);
    uint32_t tzbR = (uint32_t)tzb, tzbwR = tzbw;   // kZ: made opaque per iteration (no LICM)
    uint32_t tzTR = tzT;   // opaque: the table's base stays in the VGPR, shift offsets are immediates
    auto rot = [&](int sft) -> int {
        const uint32_t S = (uint32_t)sft * GT;
        if constexpr (kZ) return (int)min(tzbR + S, tzbwR + S);
        else return (int)min((uint32_t)tzb + S, tzbw + S);
    };
    // the same on the VALU (v_mul_u32_u24 with an opaque VGPR stride) for the final syndrome pass:
    // the scalar unit is shared by the workgroup's 12 waves
    uint32_t GTv = GT;
    asm volatile("" : "+v"(GTv));
    auto rot_v = [&](int sft) -> int {
        const uint32_t S = __umul24((uint32_t)sft, GTv);
        return (int)min((uint32_t)tzb + S, tzbw + S);
    };
    // f(integral_constant<half>): each half's rows form one basic block, so the scheduler can
    // overlap a row's LDS reads with the previous row's arithmetic
    auto per_half = [&](auto&& f) {
        sfor<0, NP>([&](auto pc_) {
            if (h == decltype(pc_)::value) f(pc_);
        });
    };
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)
    asm volatile("" : "+v"(mv));

    uint64_t hdx_keep = 0;   // extension decisions of a slot decided by the syndrome test
    int it = 0;
    for (; it < L; ++it) {
        // zv / ziv opaque per iteration: otherwise LICM hoists the ~300 loop-invariant shift
        // words and column addresses out of the loop into registers
        zv = zg;
        ziv = zi;
        asm volatile("" : "+v"(zv));
        asm volatile("" : "+s"(ziv));
        if constexpr (kZ) {
            tzbR = (uint32_t)tzb, tzbwR = tzbw;
            asm volatile("" : "+v"(tzbR));
            asm volatile("" : "+v"(tzbwR));
        }
        if constexpr (WT) {
            tzTR = tzT;
            asm volatile("" : "+v"(tzTR));
        }
        bool fail = false;
        uint64_t hdx = 0;   // hard decisions of the owned extension columns (LQ_old)
        // shift words of this lifting size: one base pointer (SGPR pair), immediate offsets
        const uint32_t* __restrict__ swrow = shift_row<BG>(ziv);
        auto sh = [&](int e) -> int {   // e compile-time after unrolling
            if constexpr (kZ) return zc_shift<BG, ZCC>(e);
            const uint32_t w = swrow[e >> 1];
            return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
        };

        // ext LLR ring: slot p % XP holds the LLR of the half's ext row p, loaded XP rows ahead
        constexpr int XP = kXPre > 0 ? kXPre : 1;
        T xr[XP];
        auto xload = [&](auto hc, auto pc_) {
            constexpr int hh = decltype(hc)::value, p = decltype(pc_)::value;
            if constexpr (kXPre > 0 && p < kFloodPlan<BG, T, NP, CS>.nx[hh])
                xr[p % XP] = llrx(kFloodPlan<BG, T, NP, CS>.xlist[hh][p]);
        };
        // ---- phase A: new row state from LQ_old (:117-123, _min_sum_process :186-202)
        // core-edge LQ reads issued kAPre edges ahead of their use (ring ab)
        constexpr int AP = kAPre > 0 ? kAPre : 1;
        struct RowSt {
            T mA, mB, min1, min2;
            uint32_t u, idxo, sx, idx, negs;   // u: bit 31 = sign of r_k for the edge k being visited
            bool par;
            T ab[AP];
            uint32_t tb[AP + 1];   // WT: wrap-table entries of the next AP + 1 edges
        };
        auto aloadt = [&](RowSt& r, auto ic, auto kc3) {
            constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = P::RS[i + 1] - e0;
            constexpr int k3 = decltype(kc3)::value;
            if constexpr (WT && k3 < d) {
                if constexpr (P::COL[e0 + k3] < KC)
                    r.tb[k3 % (AP + 1)] = *(lds_u32*)(uintptr_t)(tzTR + (uint32_t)sh(e0 + k3) * G4);
            }
        };
        auto aload = [&](RowSt& r, auto ic, auto kc2) {
            constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = P::RS[i + 1] - e0;
            constexpr int k2 = decltype(kc2)::value;
            if constexpr (kAPre > 0 && k2 < d) {
                if constexpr (P::COL[e0 + k2] < KC) {
                    if constexpr (WT) r.ab[k2 % AP] = at(P::COL[e0 + k2] * CS * TS + (int)r.tb[k2 % (AP + 1)]);
                    else r.ab[k2 % AP] = at(P::COL[e0 + k2] * CS * TS + rot(sh(e0 + k2)));
                }
            }
        };
        auto rbegin = [&](RowSt& r, auto ic) {
            get_state(ic, r.mA, r.mB, r.u, r.idxo);
            r.min1 = FT<T>::inf(), r.min2 = FT<T>::inf();
            r.sx = 0, r.idx = 0, r.negs = 0;
            r.par = false;
            if constexpr (WT) sfor<0, AP + 1>([&](auto kc3) { aloadt(r, ic, kc3); });
            sfor<0, AP>([&](auto kc2) { aload(r, ic, kc2); });
        };
        auto rstep = [&](RowSt& r, auto ic, auto kc) {
            constexpr int i = decltype(ic)::value, e0 = P::RS[i];
            constexpr int k = decltype(kc)::value;
            constexpr int j = P::COL[e0 + k];
            const T rold = xsign_v(pick(r.idxo == (uint32_t)k, r.mB, r.mA), r.u, mv);
            asm("v_add_u32 %0, %1, %1" : "=v"(r.u) : "v"(r.u));   // u <<= 1, all-VGPR form
            T a;
            if constexpr (j < KC) {
                if constexpr (kAPre > 0) {
                    a = r.ab[k % AP];
                    aload(r, ic, std::integral_constant<int, k + AP>{});
                    aloadt(r, ic, std::integral_constant<int, k + AP + 1>{});
                    if constexpr (kASb) __builtin_amdgcn_sched_barrier(0);
                } else {
                    a = at(j * CS * TS + rot(sh(e0 + k)));
                }
            } else {
                constexpr int hh = kFloodPlan<BG, T, NP, CS>.owner[i], p = kFloodPlan<BG, T, NP, CS>.xpos[i];
                if constexpr (kXPre > 0) {
                    a = xr[p % XP] + rold;   // LQ of a degree-1 column = LLR + its only r
                    xload(std::integral_constant<int, hh>{}, std::integral_constant<int, p + XP>{});
                } else {
                    a = llrx(i) + rold;
                }
                hdx |= (uint64_t)(a < T(0)) << (i - 4);
            }
            r.par ^= a < T(0);
            const T q = a - rold;
            const T aq = fabs(q);
            r.idx = aq < r.min1 ? (uint32_t)k : r.idx;
            asm volatile("" : "+v"(r.idx));   // update in place: a sunk select chain keeps all
                                              // the compare masks live (scratch spills)
            r.negs = __builtin_amdgcn_alignbit(r.negs, FT<T>::sbits(q), 31);
            two_min(r.min1, r.min2, aq);
            if constexpr (!kSxPop) r.sx ^= FT<T>::sbits(q);
        };
        auto rend = [&](RowSt& r, auto ic) {
            constexpr int i = decltype(ic)::value, d = P::RS[i + 1] - P::RS[i];
            fail |= r.par;
            T x1 = r.min1, x2 = r.min2;
            if constexpr (OFS) {
                x1 = r.min1 - beta, x2 = r.min2 - beta;   // max(minv - beta, 0) (:201)
                x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
            }
            // the row's sign product: the parity of the d sign bits packed in negs (or bit 31 of the
            // XOR of the q sign words)
            const uint32_t sgn = kSxPop ? 0u - (__builtin_popcount(r.negs) & 1u) : (uint32_t)((int32_t)r.sx >> 31);
            const uint32_t flip = sgn & ((1u << d) - 1u);
            put_state(ic, alpha * x1, alpha * x2, r.negs ^ flip, r.idx);
        };
        auto rowA = [&](auto ic) {
            constexpr int i = decltype(ic)::value, d = P::RS[i + 1] - P::RS[i];
            RowSt r;
            rbegin(r, ic);
            sfor<0, d>([&](auto kc) { rstep(r, ic, kc); });
            rend(r, ic);
        };
        // dead extension row: LQ_ext = 0 + r_old_ext (its syndrome bit), q_core = LQ - (+-0);
        // new state as the full update leaves it up to zero signs: nA = 0, nB = alpha * max(
        // min |q_core| - beta, 0), argmin = the extension edge, whose sign bit is the row sign
        auto rowA_dead = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int e0 = P::RS[i];
            constexpr int d = P::RS[i + 1] - e0;
            T mA, mB;
            uint32_t u, idxo;
            get_state(ic, mA, mB, u, idxo);
            const T rext = xsign_v(pick(idxo == (uint32_t)(d - 1), mB, mA), u << (d - 1), mv);
            if constexpr (kXPre > 0) {   // keep the half's ext-LLR ring moving (row p + XP's load)
                constexpr int hh = kFloodPlan<BG, T, NP, CS>.owner[i], p = kFloodPlan<BG, T, NP, CS>.xpos[i];
                xload(std::integral_constant<int, hh>{}, std::integral_constant<int, p + XP>{});
            }
            const T ax = T(0) + rext;
            hdx |= (uint64_t)(ax < T(0)) << (i - 4);
            bool par = ax < T(0);
            T mn = FT<T>::inf();
            uint32_t sx = 0;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                if constexpr (j < KC) {
                    const T a = at(j * CS * TS + rot(sh(e0 + k)));
                    par ^= a < T(0);
                    mn = fmin(mn, fabs(a));
                    sx ^= FT<T>::sbits(a);
                }
            });
            fail |= par;
            T x2 = mn;
            if constexpr (OFS) {
                x2 = mn - beta;
                x2 = x2 > T(0) ? x2 : T(0);
            }
            put_state(ic, T(0), alpha * x2, sx >> 31, (uint32_t)(d - 1));
        };
        if (active) {
            per_half([&](auto hc) { sfor<0, XP>([&](auto pc_) { xload(hc, pc_); }); });
            sfor<0, MB>([&](auto ic) {   // one branch per row: bounded live ranges
                constexpr int i = decltype(ic)::value;
                if (h == kFloodPlan<BG, T, NP, CS>.owner[i]) {
                    if constexpr (DEAD && i >= 4) {
                        if (rdead(ic)) rowA_dead(ic);
                        else rowA(ic);
                    } else {
                        rowA(ic);
                    }
                }
            });
            if (fail) flagA[cl] = 1;
        }
        // phase B's shift words are loaded one row group ahead (scalar loads issued before the
        // barrier that precedes the group, so their latency hides behind it)
        constexpr int NPW = max_group_nw<BG>();
        uint32_t nsw[NPW];
        auto prefetch = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            sfor<0, group_nw<BG>(g)>([&](auto wc) {
                constexpr int w = decltype(wc)::value;
                nsw[w] = swrow[group_w0<BG>(g) + w];
            });
        };
        // the LDS-held state of the next group's row (rows < NLS are single-row groups) is read
        // one group ahead as well: phase A wrote it before the barrier that precedes phase B
        T qA = T(0), qB = T(0);
        uint32_t qu = 0, qidx = 0;
        auto prefetch_state = [&](auto gc) {
            constexpr int r = kGroups<BG>.start[decltype(gc)::value];
            if constexpr (r < NLS) get_state(std::integral_constant<int, r>{}, qA, qB, qu, qidx);
        };
        prefetch(std::integral_constant<int, 0>{});
        lds_barrier();
        prefetch_state(std::integral_constant<int, 0>{});
        // ---- the syndrome of LQ_old decides (:107-114): output its hard decisions
        if (active && flagA[cl] == 0) {
            // decided: its LQ entries stay frozen in LDS (no phase B / LQ update for an inactive
            // slot) and its extension decisions are kept, for the staged ck store at the end
            hdx_keep = hdx;
            if (z == 0 && h == 0) status[out] = 1, iters[out] = it;
            active = false;
        }

        // ---- phase B: Lr.sum(axis=0) in row order into the LQ array (:126)
        auto rowB = [&](auto ic, auto splitc, auto& gshift, T nA, T nB, uint32_t u, uint32_t idxn) {
            constexpr int i = decltype(ic)::value;
            constexpr int e0 = P::RS[i];
            constexpr int d = P::RS[i + 1] - e0;
            constexpr int split = decltype(splitc)::value;   // -1: all edges, else edges of parity
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                constexpr int cidx = [] {
                    int n = 0;
                    for (int kk = 0; kk < k; ++kk) n += P::COL[e0 + kk] < KC;
                    return n;
                }();
                if constexpr (j < KC && (split < 0 || cidx % NP == split)) {
                    const T r = xsign_v(pick(idxn == (uint32_t)k, nB, nA), u, mv);
                    lds_T& acc = at(j * CS * TS + rot(gshift(e0 + k)));
                    if constexpr (kFloodPlan<BG, T, NP, CS>.first_row[j] == i) {
                        acc = T(0) + r;
                    } else if constexpr (sizeof(T) == 8) {
                        // ds_add_f64 without return: the LDS unit does the read-add-write (same
                        // IEEE round-to-nearest double add), so a row group is not a chain of
                        // dependent round trips (4.38 -> 4.17 ms per 4096 codeblocks).  The f32
                        // ds_add_f32 measured 4x slower than read-add-write; f32 keeps the latter.
                        __hip_atomic_fetch_add(&acc, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        acc = acc + r;
                    }
                }
                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));
            });
        };
        // the core LLRs of the LQ update, loaded now so phase B hides their latency
        T lf[KH];
        if (active)
            sfor<0, KH>([&](auto jc) {
                constexpr int jj = decltype(jc)::value;
                const int j = h * KH + jj;
                const int jl = min(j, KC - 1);   // unconditional: all loads in flight at once
                lf[jj] = ldl_at((jl < pc ? 0 : jl - pc) * Zc, zv);
            });
        sfor<0, kGroups<BG>.n>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            uint32_t csw[NPW];
#pragma unroll
            for (int x = 0; x < NPW; ++x) csw[x] = nsw[x];
            const T cA = qA, cB = qB;
            const uint32_t cu = qu, cidx = qidx;
            if constexpr (g + 1 < kGroups<BG>.n) {
                prefetch(std::integral_constant<int, g + 1>{});
                prefetch_state(std::integral_constant<int, g + 1>{});
            }
            auto gshift = [&](int e) -> int {   // e compile-time after unrolling
                if constexpr (kZ) return zc_shift<BG, ZCC>(e);
                const uint32_t w = csw[(e >> 1) - group_w0<BG>(g)];
                return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
            };
            const bool gd = gdead(gc);   // a dead group adds nothing: no barrier either
            if (active && !gd) {
                per_half([&](auto hc) {
                    sfor<kGroups<BG>.start[g], kGroups<BG>.start[g + 1]>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        if (rdead(ic)) return;   // +-0 adds (a partly dead group)
                        if constexpr (i < NLS) {   // LDS state: both halves, alternate edges
                            rowB(ic, hc, gshift, cA, cB, cu, cidx);
                        } else if constexpr (kFloodPlan<BG, T, NP, CS>.owner[i] == decltype(hc)::value) {
                            T a, b;
                            uint32_t u, x;
                            get_state(ic, a, b, u, x);
                            rowB(ic, std::integral_constant<int, -1>{}, gshift, a, b, u, x);
                        }
                    });
                });
            }
            if (!gd) lds_barrier();
        });
        // ---- LQ = LLRin + sum (:126) for the own entries
        if (active)
            sfor<0, KH>([&](auto jc) {
                constexpr int jj = decltype(jc)::value;
                const int j = h * KH + jj;
                if (j < KC) {
                    lds_T& x = own(j);
                    x = (j < pc ? T(0) : lf[jj]) + x;   // punctured columns: LLR 0 (:43)
                }
            });
        if (s == 0 && h == 0)
            for (int c = 0; c < G; ++c) flagA[c] = 0;   // read before the phase-B barriers
        if (!block_any(active)) break;
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    zv = zg;
    asm volatile("" : "+v"(zv));   // keep the output addresses out of the loop (no hoist/spill)
    auto rfinal = [&](auto ic, int k) -> T {
        constexpr int i = decltype(ic)::value;
        T a, b;
        uint32_t u, idx;
        get_state(ic, a, b, u, idx);
        return xsign_v(pick(idx == (uint32_t)k, b, a), u << k, mv);
    };
    uint32_t oc = 0;          // own core columns (bit j - h*KH): LQ <= 0, or LQ_old < 0 if decided
    uint64_t ox = hdx_keep;   // own extension columns
    if (active) {
        // the owned rows' extension decisions first, their LLRs requested in batches of 8 before any
        // is used (the row state is dead before the syndrome pass)
        ox = 0;
        per_half([&](auto hc) {
            constexpr int hh = decltype(hc)::value;
            constexpr int NX = kFloodPlan<BG, T, NP, CS>.nx[hh], XB = 8;
            sfor<0, (NX + XB - 1) / XB>([&](auto bc) {
                constexpr int x0 = decltype(bc)::value * XB, x1 = x0 + XB < NX ? x0 + XB : NX;
                T vx[XB];
                sfor<x0, x1>([&](auto xc) {
                    vx[decltype(xc)::value - x0] = llrx(kFloodPlan<BG, T, NP, CS>.xlist[hh][decltype(xc)::value]);
                });
                __builtin_amdgcn_sched_barrier(0);
                sfor<x0, x1>([&](auto xc) {
                    constexpr int i = kFloodPlan<BG, T, NP, CS>.xlist[hh][decltype(xc)::value];
                    constexpr int dl = P::RS[i + 1] - P::RS[i] - 1;   // ext column = last edge
                    ox |= (uint64_t)(vx[decltype(xc)::value - x0] + rfinal(std::integral_constant<int, i>{}, dl) <= T(0))
                          << (i - 4);
                });
            });
        });
        bool fail = false;
        per_half([&](auto hc) {
            constexpr int hh = decltype(hc)::value;
            constexpr uint64_t rows = [] {
                uint64_t m = 0;
                for (int i = 0; i < P::MB; ++i)
                    if (kFloodPlan<BG, T, NP, CS>.owner[i] == hh) m |= 1ull << i;
                return m;
            }();
            fail = syndrome_fails<BG, rows, false, T>(
                [&](auto ic, auto kc) -> T {
                    constexpr int e = P::RS[decltype(ic)::value] + decltype(kc)::value;
                    return at(P::COL[e] * CS * TS + rot_v(shift_of<BG>(zi, e)));
                },
                [&](auto ic) -> bool { return (ox >> (decltype(ic)::value - 4)) & 1u; });
        });
        if (fail) flagA[cl] = 1;
    }
    if (valid)
        sfor<0, KH>([&](auto jc) {
            const int j = h * KH + decltype(jc)::value;
            if (j < KC) {
                const T v = own(j);
                oc |= (uint32_t)(active ? v <= T(0) : v < T(0)) << decltype(jc)::value;
            }
        });
    lds_barrier();   // every LQ / state read is done: LDS below FLAG_B is free from here
    if (active && z == 0 && h == 0) {
        status[out] = flagA[cl] == 0;
        iters[out] = L;
    }
    // ---- ck through LDS (ck_store_staged, ldpc5g_dec_body.h); direct byte stores when the
    //      workgroup's rows exceed the space below the flags (small-CS configurations)
    const int NFZ = P::NB * Zc;
    const bool staged = G * ck_stage_stride(NFZ) <= FLAG_B;
    if (valid) {
        const uint32_t sb = (uint32_t)(cl * ck_stage_stride(NFZ) + zv);
        auto put = [&](int col, uint32_t bit) {
            if (staged) ck_stage_byte(sb + (uint32_t)(col * Zc), bit);
            else crow[col * Zc + zv] = (int8_t)bit;
        };
        sfor<0, KH>([&](auto jc) {
            const int j = h * KH + decltype(jc)::value;
            if (j < KC) put(j, (oc >> decltype(jc)::value) & 1u);
        });
        per_half([&](auto hc) {
            sfor<4, MB>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (kFloodPlan<BG, T, NP, CS>.owner[i] == decltype(hc)::value)
                    put(KB + i, (uint32_t)(ox >> (i - 4)) & 1u);
            });
        });
    }
    if (staged) {
        const bool slow = block_any(valid && !ck_row_aligned(NFZ, crow));   // orders the staging too
        const int nslots = work ? G : min(G, B - (int)blockIdx.x * G);
        ck_store_staged(NFZ, nslots, [&](int sl) -> int8_t* {
            if (work) return ck + cbs[work[blockIdx.x].first + sl].ck_off;
            return ck + (int64_t)((int)blockIdx.x * G + sl) * ldc;
        }, slow, t, (int)blockDim.x);
    }
}

// NP parts x CS slots: 768 threads (3 waves per SIMD) for batches, 1024 (4 per SIMD) for the
// 16-part configuration of small launches
template <int BG, typename T, bool OFS, int NP, int CS, bool DEAD = false, int ZCC = 0>
__global__ __launch_bounds__(NP * CS) __attribute__((amdgpu_waves_per_eu(NP * CS / 256))) void
ldpc_flood_kernel(LDPC5G_DEC_PARAMS) {
    flood_body<BG, T, OFS, NP, CS, DEAD, ZCC>(LDPC5G_DEC_ARGS);
}

template <int BG, typename T, bool OFS, int NP, int CS, bool DEAD = false, int ZCC = 0>
constexpr auto flood_kernel() { return ldpc_flood_kernel<BG, T, OFS, NP, CS, DEAD, ZCC>; }

template <int BG, typename T, int NP, int CS>
size_t flood_lds_bytes() {
    static_assert(flood_lds_bytes_t<BG, T, NP, CS>() <= kLdsPerCU, "LDS budget of one CU");
    return flood_lds_bytes_t<BG, T, NP, CS>();
}

template <int BG, typename T, int NP, int CS, bool DEAD = false, int ZCC = 0>
int set_flood_lds(bool ofs) {
    const size_t lds = flood_lds_bytes<BG, T, NP, CS>();
    return ofs ? set_lds_once<flood_kernel<BG, T, true, NP, CS, DEAD, ZCC>()>(lds)
               : set_lds_once<flood_kernel<BG, T, false, NP, CS, DEAD, ZCC>()>(lds);
}

// G codeblocks per workgroup (G * Zc <= CS); NP parts of H = G*Zc rounded up to a wave
template <int BG, typename T, int NP, int CS, bool DEAD = false, int ZCC = 0>
int launch_flood_cfg(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                     int G, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                     hipStream_t st) {
    const bool ofs = beta != 0.0;
    auto kern = ofs ? ldpc_flood_kernel<BG, T, true, NP, CS, DEAD, ZCC> : ldpc_flood_kernel<BG, T, false, NP, CS, DEAD, ZCC>;
    const int H = ((G * Zc + 63) / 64) * 64;
    if (G < 1 || H > CS) return fail(LDPC5G_ESIZE, "flooding launch: %d codeblocks of Zc=%d per workgroup", G, Zc);
    if (ZCC > 0 && (Zc != ZCC || G != 1)) return fail(LDPC5G_ESIZE, "Zc=%d kernel launched for Zc=%d, G=%d", ZCC, Zc, G);
    if ((int64_t)G * ldl * (int64_t)sizeof(T) >= ((int64_t)1 << 32))   // 32-bit lane offsets (flood_body)
        return fail(LDPC5G_ESIZE, "ldl=%lld: a workgroup's %d LLR rows span >= 4 GiB", (long long)ldl, G);
    if (int rc = set_flood_lds<BG, T, NP, CS, DEAD, ZCC>(ofs)) return rc;
    const size_t lds = flood_lds_bytes<BG, T, NP, CS>();
    hipLaunchKernelGGL(kern, dim3((B + G - 1) / G), dim3(NP * H), lds, st, llr, ck, status, iters, B, Zc,
                       zi, G, ldl, ldc, L, (T)alpha, (T)beta, pc, (const DecWork*)nullptr,
                       (const CbRef*)nullptr);
    return check_hip(hipGetLastError(), "ldpc_flood_kernel launch");
}

constexpr int kFloodNP = 2, kFloodCS = kDecThreads;   // batch configuration: 2 x 384 slots
constexpr int kFloodSmallNP = 16, kFloodSmallCS = 64;  // small launches: 16 x 64 slots

template <int BG, typename T, bool DEAD = false>
int launch_flood_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                   int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    // small batches (the per-codeblock drop-ins): no more slots than codeblocks
    const int G = std::min(dec_G(Zc, false), B);
    if constexpr (flood_wtab<BG, T, kFloodNP, kFloodCS>() && !(LDPC5G_FLOOD_FRAME && std::is_same_v<T, double>))
        if (Zc == kFloodCS)   // the largest lifting size has its own kernel (zc_shift)
            return launch_flood_cfg<BG, T, kFloodNP, kFloodCS, DEAD, kFloodCS>(
                llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha, beta, pc, st);
    return launch_flood_cfg<BG, T, kFloodNP, kFloodCS, DEAD>(llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L,
                                                             alpha, beta, pc, st);
}

// ZCC > 0: every work item is a Zc = ZCC item (G = 1; ldpc5g_capi.hip build_plan puts them last)
template <int BG, typename T, bool DEAD = false, int ZCC = 0>
int launch_flood_mixed_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                         const DecWork* work, const CbRef* cbs, int L, double alpha, double beta,
                         int pc, hipStream_t st) {
    const bool ofs = beta != 0.0;
    auto kern = ofs ? ldpc_flood_kernel<BG, T, true, kFloodNP, kFloodCS, DEAD, ZCC>
                    : ldpc_flood_kernel<BG, T, false, kFloodNP, kFloodCS, DEAD, ZCC>;
    if (int rc = set_flood_lds<BG, T, kFloodNP, kFloodCS, DEAD, ZCC>(ofs)) return rc;
    const size_t lds = flood_lds_bytes<BG, T, kFloodNP, kFloodCS>();
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(kFloodNP * kFloodCS), lds, st, llr, ck, status, iters, 0, 0,
                       0, 0, (int64_t)0, (int64_t)0, L, (T)alpha, (T)beta, pc, work, cbs);
    return check_hip(hipGetLastError(), "ldpc_flood_kernel(mixed) launch");
}

template <int BG, typename T>
int flood_blocks_per_cu_t() {
    const size_t lds = flood_lds_bytes<BG, T, kFloodNP, kFloodCS>();
    if (set_lds_once<flood_kernel<BG, T, false, kFloodNP, kFloodCS>()>(lds)) return -1;
    int n = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ldpc_flood_kernel<BG, T, false, kFloodNP, kFloodCS>,
                                                     kFloodNP * kFloodCS, lds) != hipSuccess)
        return -1;
    return n;
}

}  // namespace
}  // namespace ldpc5g_impl
