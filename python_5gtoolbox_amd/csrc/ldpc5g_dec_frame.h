// ldpc5g_dec_frame.h — float64 flooding min-sum decoder for lifting size Zc = 384 with per-row
// thread frames (py5gphy/ldpc/nr_ldpc_decode.py:51-143, _min_sum_process :178-227).  Bit-identical
// to the reference and to ldpc_flood_kernel (ldpc5g_dec_flood.h), whose two-phase data flow it
// keeps: phase A forms every row's new compressed state from LQ_old, phase B sums the messages
// into LQ in row-ascending order per column (Lr.sum(axis=0), :126).
//
// What changes is who sums what.  ldpc_flood_kernel adds each row's messages into the LDS image of
// LQ with one barrier per group of column-disjoint rows, and columns 0 and 1 — 30 and 28 of BG1's 46
// rows — make that 32 groups.  Here the thread that runs check node z' of row i is chosen per row
// (its "frame"): a row with column 0 runs on half 0 with thread s = (z' + V(i,0)) mod Zc, a row
// with column 1 but not 0 on half 1 with s = (z' + V(i,1)) mod Zc.  Then thread s of half 0 makes
// the message of EVERY column-0 edge into column-0 entry s, and adds them in registers, in row
// order, with no barrier; half 1 does column 1 the same way.  Rows with both columns keep their
// state in LDS, where each half reads it in its own frame; when LDS is full (BG1: 3 rows), the
// owner hands the other column's message over through the LDS image of columns 0 / 1, which is
// dead during phase B.  The barrier groups only order columns >= 2: BG1 46 rows -> 18 groups
// (32 before), BG2 42 -> 23 (28).
#pragma once
#include "ldpc5g_dec_flood.h"

namespace ldpc5g_impl {
namespace {

constexpr int kFrZ = kFrameZc;
constexpr int kFrThreads = 2 * kFrZ;
constexpr int kFrColB = kFrZ * 8;          // one LQ column (float64) or hand-off slot
constexpr int kFrRowB = kFrZ * (16 + 4);   // one LDS state row: (mA, mB) pairs + sign words
constexpr int kFrFlagB = 64;

// Compile-time plan of the rows: LDS / VGPR state, owner half, frame, hand-offs, barrier groups.
template <int BG>
struct FramePlan {
    int kc[2][64] = {};   // edge (index in the row) of column c, -1: none
    bool lds[64] = {};    // state in LDS (either half can read it)
    int lslot[64] = {};
    int nls = 0;
    int owner[64] = {};   // half that runs phase A (and the final pass) of row i
    int fr[64] = {};      // frame column (0 / 1; -1: natural, thread s runs check node s)
    int off[64] = {};     // V(i, fr) mod Zc: thread s runs check node (s - off) mod Zc
    int slot[64] = {};    // VGPR state slot in the owner half
    int nslot = 0;
    int pw[64] = {}, ph[64] = {};   // VGPR sign word (rows of degree <= 12 share one: 16-bit fields)
    int npw = 0;
    int ho[64] = {};      // hand-off slot of a VGPR row with both columns 0 and 1, -1: none
    int nho = 0, nspare = 0;
    int first_row[32] = {};   // lowest row of column j >= 2 (writes 0 + r)
    int xpos[64] = {}, xlist[2][64] = {}, nx[2] = {};   // extension rows per owner half
    int ng = 0;
    int gstart[65] = {};  // barrier groups: consecutive rows whose columns >= 2 are disjoint
    int grp[64] = {};
    int eh[64][20] = {};  // LDS rows: the half that adds edge k (column >= 2) in phase B
    int st_b = 0, pk_b = 0, fl_b = 0, tbl_b = 0, sp_b = 0, bytes = 0;   // LDS layout
    bool ok = true;

    static constexpr int deg(int i) { return BGT<BG>::RS[i + 1] - BGT<BG>::RS[i]; }
    static constexpr int ncore2(int i) {   // core edges of columns >= 2
        int n = 0;
        for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i + 1]; ++e) n += BGT<BG>::COL[e] >= 2 && BGT<BG>::COL[e] < BGT<BG>::KC;
        return n;
    }
    constexpr bool both(int i) const { return kc[0][i] >= 0 && kc[1][i] >= 0; }
    constexpr int hb(int b) const { return b < 2 ? b * kFrColB : sp_b + (b - 2) * kFrColB; }

    constexpr FramePlan() {
        using P = BGT<BG>;
        const int MB = P::MB;
        for (int i = 0; i < MB; ++i) {
            kc[0][i] = kc[1][i] = -1;
            ho[i] = -1;
            for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                if (P::COL[e] < 2) kc[P::COL[e]][i] = e - P::RS[i];
        }
        gstart[0] = 0, ng = 1;
        for (int i = 1, g0 = 0; i < MB; ++i) {
            bool dis = true;
            for (int a = g0; a < i && dis; ++a)
                for (int e = P::RS[a]; e < P::RS[a + 1]; ++e)
                    for (int f = P::RS[i]; f < P::RS[i + 1]; ++f)
                        if (P::COL[e] == P::COL[f] && P::COL[e] >= 2 && P::COL[e] < P::KC) dis = false;
            if (!dis) gstart[ng++] = i, g0 = i;
        }
        gstart[ng] = MB;
        for (int g = 0; g < ng; ++g)
            for (int i = gstart[g]; i < gstart[g + 1]; ++i) grp[i] = g;
        // LDS rows: degree > 12 (split across the halves in phase B), then rows with both columns
        // (no hand-off), then the longest rows while a half would hold more than 18 VGPR rows
        const int fixed = P::KC * kFrColB + kFrFlagB + 2 * kFrZ * 4;
        for (nspare = 0; nspare < 8; ++nspare) {
            const int cap = (160 * 1024 - fixed - nspare * kFrColB) / kFrRowB;
            for (int i = 0; i < MB; ++i) lds[i] = false;
            nls = 0;
            for (int pass = 0; pass < 3; ++pass)
                for (;;) {
                    if (nls >= cap || (pass == 2 && MB - nls <= 36)) break;
                    int best = -1;
                    for (int i = 0; i < MB; ++i) {
                        const bool want = pass == 0 ? deg(i) > 12 : pass == 1 ? both(i) : true;
                        if (!lds[i] && want && (best < 0 || deg(i) > deg(best))) best = i;
                    }
                    if (best < 0) break;
                    lds[best] = true, ++nls;
                }
            nho = 0;
            for (int i = 0; i < MB; ++i) nho += !lds[i] && both(i);
            if (nho - 2 <= nspare) break;
        }
        if (nspare > 0 && nho - 2 < nspare) nspare = nho > 2 ? nho - 2 : 0;
        for (int i = 0, n = 0; i < MB; ++i)
            if (lds[i]) lslot[i] = n++;
        // owners: a row with only column c runs on half c in frame c; rows with both (hand-off) or
        // neither go where fewer VGPR rows are (then to the lighter half of their group)
        int nv[2] = {}, ea[2] = {}, gl[2][64] = {};
        for (int i = 0; i < MB; ++i) {
            if (lds[i]) {
                const int n = ncore2(i);
                gl[0][grp[i]] += (n + 1) / 2, gl[1][grp[i]] += n / 2;
                continue;
            }
            if ((kc[0][i] >= 0) == (kc[1][i] >= 0)) continue;
            const int hh = kc[0][i] >= 0 ? 0 : 1;
            owner[i] = hh, fr[i] = hh, ++nv[hh], ea[hh] += deg(i), gl[hh][grp[i]] += ncore2(i);
        }
        for (int i = 0, b = 0; i < MB; ++i) {
            if (lds[i] || (kc[0][i] >= 0) != (kc[1][i] >= 0)) continue;
            const int hh = nv[0] != nv[1] ? (nv[0] < nv[1] ? 0 : 1) : (gl[0][grp[i]] <= gl[1][grp[i]] ? 0 : 1);
            owner[i] = hh, fr[i] = both(i) ? hh : -1, ++nv[hh], ea[hh] += deg(i), gl[hh][grp[i]] += ncore2(i);
            if (both(i)) {
                ho[i] = b++;
                ok = ok && grp[i] >= 1;   // written before group 0's barrier, read after it
            }
        }
        for (;;) {   // LDS rows' phase A: by decreasing degree onto the half with fewer edges
            int best = -1;
            for (int i = 0; i < MB; ++i)
                if (lds[i] && fr[i] != -2 && (best < 0 || deg(i) > deg(best))) best = i;
            if (best < 0) break;
            const int hh = ea[0] <= ea[1] ? 0 : 1;
            owner[best] = hh, fr[best] = -2, ea[hh] += deg(best);
        }
        for (int i = 0; i < MB; ++i) {
            if (fr[i] == -2) fr[i] = -1;
            off[i] = fr[i] < 0 ? 0 : zc_shift<BG, kFrZ>(P::RS[i] + kc[fr[i]][i]);
        }
        int ns[2] = {};
        for (int i = 0; i < MB; ++i) slot[i] = lds[i] ? -1 : ns[owner[i]]++;
        nslot = ns[0] > ns[1] ? ns[0] : ns[1];
        for (int hh = 0; hh < 2; ++hh) {
            int n = 0, open = -1;
            for (int i = 0; i < MB; ++i) {
                if (lds[i] || owner[i] != hh) continue;
                if (deg(i) > 12) pw[i] = n++, ph[i] = 0;
                else if (open >= 0) pw[i] = open, ph[i] = 2, open = -1;
                else open = n, pw[i] = n++, ph[i] = 1;
            }
            npw = npw > n ? npw : n;
        }
        for (int i = 4; i < MB; ++i) xpos[i] = nx[owner[i]], xlist[owner[i]][nx[owner[i]]++] = i;
        for (int j = 0; j < P::KC; ++j) {
            first_row[j] = -1;
            for (int i = 0; i < MB && first_row[j] < 0; ++i)
                for (int e = P::RS[i]; e < P::RS[i + 1]; ++e)
                    if (P::COL[e] == j) first_row[j] = i;
        }
        for (int g = 0; g < ng; ++g) {
            // LDS rows' adds go to the half with fewer adds in the group so far (VGPR rows fixed)
            int ld[2] = {};
            for (int i = gstart[g]; i < gstart[g + 1]; ++i)
                if (!lds[i]) ld[owner[i]] += ncore2(i);
            for (int i = gstart[g]; i < gstart[g + 1]; ++i)
                for (int k = 0; lds[i] && k < deg(i); ++k) {
                    const int j = P::COL[P::RS[i] + k];
                    if (j < 2 || j >= P::KC) continue;
                    const int hh = ld[0] <= ld[1] ? 0 : 1;
                    eh[i][k] = hh, ++ld[hh];
                }
        }
        // every row holds column 0 or 1 in the 5G base graphs, or is a VGPR row (natural frame)
        st_b = P::KC * kFrColB;
        pk_b = st_b + nls * kFrZ * 16;
        fl_b = pk_b + nls * kFrZ * 4;
        tbl_b = fl_b + kFrFlagB;
        sp_b = tbl_b + 2 * kFrZ * 4;
        bytes = sp_b + nspare * kFrColB;
        ok = ok && bytes <= 160 * 1024 && nho <= 2 + nspare && nslot <= 18;
    }
};
template <int BG>
constexpr FramePlan<BG> kFrPlan{};
static_assert(kFrPlan<1>.ok && kFrPlan<2>.ok, "frame plan");

// The core-edge stream of each half: the core edges (columns < KC) of the half's rows in row
// order, edge order within a row (a row's extension edge, its last, skipped).  Phase A reads the
// stream's wrap-table offsets and LQ entries a fixed number of positions ahead, across rows.
template <int BG>
struct FrStream {
    int start[64] = {};   // position of row i's edge 0 in its owner's stream
    int n[2] = {};
    int row[2][256] = {}, k[2][256] = {};
    bool ok = true;
    constexpr FrStream() {
        using P = BGT<BG>;
        for (int i = 0; i < P::MB; ++i) {
            const int hh = kFrPlan<BG>.owner[i];
            start[i] = n[hh];
            for (int e = P::RS[i]; e < P::RS[i + 1]; ++e) {
                if (P::COL[e] < P::KC) {
                    ok = ok && n[hh] < 256 && e - P::RS[i] == n[hh] - start[i];   // core edges first
                    if (n[hh] < 256) row[hh][n[hh]] = i, k[hh][n[hh]] = e - P::RS[i];
                    ++n[hh];
                } else {
                    ok = ok && e == P::RS[i + 1] - 1 && i >= 4;   // the extension edge last
                }
            }
        }
    }
};
template <int BG>
constexpr FrStream<BG> kFrStr{};
static_assert(kFrStr<1>.ok && kFrStr<2>.ok, "frame core-edge stream");
#ifndef LDPC5G_FR_DA
#define LDPC5G_FR_DA 1   // stream positions the LQ reads run ahead
#endif
#ifndef LDPC5G_FR_DT
#define LDPC5G_FR_DT 3   // stream positions the wrap-table reads run ahead
#endif
constexpr int kFrDA = LDPC5G_FR_DA, kFrDT = LDPC5G_FR_DT;
static_assert(kFrDA >= 1 && kFrDT > kFrDA, "stream read distances");

// V(i, k) mod Zc of edge k of row i; the same relative to the row's frame (thread s runs check node
// s - off, so edge k's column entry is s + fr_cof); frame of LDS row i for half H's phase B
template <int BG>
constexpr int fr_sft(int i, int k) { return zc_shift<BG, kFrZ>(BGT<BG>::RS[i] + k); }
template <int BG>
constexpr int fr_cof(int i, int k) { return (fr_sft<BG>(i, k) - kFrPlan<BG>.off[i] + kFrZ) % kFrZ; }
template <int BG>
constexpr int fr_pf(int i, int H) { return kFrPlan<BG>.kc[H][i] >= 0 ? fr_sft<BG>(i, kFrPlan<BG>.kc[H][i]) : 0; }

// does half H add edge k of row i (a column >= 2) in phase B: LDS rows alternate edges between the
// halves, a VGPR row's owner adds all of them
template <int BG>
constexpr bool fr_item(int H, int i, int k) {
    const int j = BGT<BG>::COL[BGT<BG>::RS[i] + k];
    if (j < 2 || j >= BGT<BG>::KC) return false;
    return kFrPlan<BG>.lds[i] ? kFrPlan<BG>.eh[i][k] == H : kFrPlan<BG>.owner[i] == H;
}
// ((e mod Zc) * 8) for 0 <= c < Zc: byte offset of entry (s + c) mod Zc from the thread's own s*8
// and s*8 - Zc*8 (the smaller as unsigned is the valid one)
__device__ __forceinline__ uint32_t fr_rot(uint32_t sb, uint32_t sbw, int c) {
    if (c == 0) return sb;
    return min(sb + (uint32_t)c * 8u, sbw + (uint32_t)c * 8u);
}

// rows >= 4 of group g as bits (i - 4) of an extension-row mask; 0 when the group holds one of the
// core rows 0..3 (never dead, so such a group always adds)
template <int BG>
constexpr uint64_t fr_group_xmask(int g) {
    uint64_t m = 0;
    for (int i = kFrPlan<BG>.gstart[g]; i < kFrPlan<BG>.gstart[g + 1]; ++i) {
        if (i < 4) return 0;
        m |= 1ull << (i - 4);
    }
    return m;
}

// DEAD = true: the LDPC5G_RATE_MATCHED variant (ldpc5g_dec_flood.h): an extension row whose LLR is
// +0.0 in every entry (never transmitted) gets the short phase A of ldpc_flood_kernel's rowA_dead
// and adds nothing in phase B (its core messages are +-0: S + (+-0) = S, since no column sum or
// register sum is ever -0.0, and no dead row is a column's first row); a group of dead rows needs
// no barrier.  Bit-identical to the full update.
// The kernel's work.  KDEAD: the prologue also finds the live extension rows (bit i - 4 of live_x:
// some entry of row i's LLR column is not +0.0), and a codeblock with a dead row iterates with the
// dead-row shortcuts, one without runs the plain iterations (the shortcuts' checks cost ~15 %).
template <int BG, bool OFS, bool KDEAD>
__device__ __forceinline__ void frame_body(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
    const DecWork* __restrict__ work, const CbRef* __restrict__ cbs) {
    using T = double;
    using P = BGT<BG>;
    constexpr int Z = kFrZ, MB = P::MB, KB = P::KB, KC = P::KC;
    constexpr int KH = KC / 2;   // own columns: half h has column h and KH - 1 of columns >= 2
    static_assert(KC % 2 == 0, "column split");
    constexpr int NS = kFrPlan<BG>.nslot > 0 ? kFrPlan<BG>.nslot : 1;
    constexpr int NPW = kFrPlan<BG>.npw > 0 ? kFrPlan<BG>.npw : 1;
    extern __shared__ __align__(16) unsigned char smem[];
    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem != 0u)
        __builtin_trap();   // the byte-offset LDS addressing below assumes a zero base
    using lds_T = __attribute__((address_space(3))) T;
    using lds_V2 = __attribute__((address_space(3))) V2<T>;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    auto at = [&](uint32_t byte) -> lds_T& { return *(lds_T*)(uintptr_t)byte; };

    const int t = threadIdx.x;
    const int h = __builtin_amdgcn_readfirstlane(t / Z);
    const int s = t - h * Z;   // own entry of every column; check node (s - off[i]) of row i
    const T* lrow;
    int8_t* crow;
    int out;
    if (work) {
        const CbRef r = cbs[work[blockIdx.x].first];
        lrow = llr + r.llr_off, crow = ck + r.ck_off, out = r.out;
    } else {
        out = (int)blockIdx.x;
        lrow = llr + (int64_t)out * ldl, crow = ck + (int64_t)out * ldc;
    }
    const T* lrow_x = lrow + (KB - pc) * Z;   // extension column of row i (>= 4): lrow_x[i * Zc + z]
    // LLR e of a row base: the bases are workgroup-uniform (SGPRs), so with a 32-bit byte offset
    // each load is one saddr access — a signed element index made it a 64-bit VALU address
    auto ldg = [&](const T* base, int e) -> T {
        using gT = const __attribute__((address_space(1))) T;
        using gB = const __attribute__((address_space(1))) unsigned char;
        return *(gT*)((gB*)(uintptr_t)base + (uint32_t)e * (uint32_t)sizeof(T));
    };
    // own column jj of half h: column h, then columns 2..KH (half 0) / KH+1..KC-1 (half 1)
    auto jcol = [&](int jj) -> int { return jj == 0 ? h : jj + 1 + h * (KH - 1); };
    int* flagA = (int*)(smem + kFrPlan<BG>.fl_b);
    int* anyf = flagA + 1;
    int epoch = 0;
    auto block_any = [&](bool p) -> bool {
        ++epoch;
        if (p) *anyf = epoch;
        lds_barrier();
        return *anyf == epoch;
    };
    auto per_half = [&](auto&& f) {
        sfor<0, 2>([&](auto hc) {
            if (h == decltype(hc)::value) f(hc);
        });
    };

    // row state: (mA, mB), the signs of r_k (edge 0 in bit d-1) and the argmin edge
    T sA[NS], sB[NS];
    uint32_t sP[NPW];
#pragma unroll
    for (int x = 0; x < NS; ++x) sA[x] = T(0), sB[x] = T(0);
#pragma unroll
    for (int x = 0; x < NPW; ++x) sP[x] = 0u;
    // LDS rows: entry (state index) e of LDS row i
    auto lds_get = [&](auto ic, uint32_t e8, T& a, T& b, uint32_t& u, uint32_t& idx) {
        constexpr int i = decltype(ic)::value, d = kFrPlan<BG>.deg(i);
        const V2<T> v = *(lds_V2*)(uintptr_t)(uint32_t)(kFrPlan<BG>.st_b + kFrPlan<BG>.lslot[i] * Z * 16 + 2 * e8);
        a = v.x, b = v.y;
        const uint32_t p = *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.pk_b + kFrPlan<BG>.lslot[i] * Z * 4 + (e8 >> 1));
        u = p << (32 - d), idx = p >> 24;
        asm volatile("" : "+v"(idx));   // compare idx itself with inline constants k
    };
    auto get_state = [&](auto ic, T& a, T& b, uint32_t& u, uint32_t& idx) {
        constexpr int i = decltype(ic)::value, d = kFrPlan<BG>.deg(i);
        if constexpr (kFrPlan<BG>.lds[i]) {
            lds_get(ic, (uint32_t)s * 8u, a, b, u, idx);
        } else {
            constexpr int x = kFrPlan<BG>.slot[i], w = kFrPlan<BG>.pw[i], f = kFrPlan<BG>.ph[i];
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
        if constexpr (kFrPlan<BG>.lds[i]) {
            V2<T> v;
            v.x = a, v.y = b;
            *(lds_V2*)(uintptr_t)(uint32_t)(kFrPlan<BG>.st_b + kFrPlan<BG>.lslot[i] * Z * 16 + s * 16) = v;
            *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.pk_b + kFrPlan<BG>.lslot[i] * Z * 4 + s * 4) = negs | (idx << 24);
        } else {
            constexpr int x = kFrPlan<BG>.slot[i], w = kFrPlan<BG>.pw[i], f = kFrPlan<BG>.ph[i];
            sA[x] = a, sB[x] = b;
            if constexpr (f == 0) sP[w] = negs | (idx << 24);
            else if constexpr (f == 1) sP[w] = (sP[w] & 0xffff0000u) | negs | (idx << 12);
            else sP[w] = (sP[w] & 0xffffu) | (negs << 16) | (idx << 28);
        }
    };

    // ---- load: LQ = LLRin (:94), punctured columns 0 (:43); LDS state 0; wrap table; flags.
    // KDEAD: each thread also loads its entry of its half's extension rows (in the row's frame:
    // together all Zc entries of every row); a wave's ballots give one word (bit p: xlist row p
    // live) at the flags' offset 16 + 4 * wave, ORed per half after the prologue's barrier.
    static_assert(kFrThreads / 64 * 4 + 16 <= kFrFlagB, "per-wave liveness words in the flags");
    {
        T v0[KH];
#pragma unroll
        for (int jj = 0; jj < KH; ++jj) {
            const int j = jcol(jj);
            v0[jj] = ldg(lrow, (j < pc ? 0 : j - pc) * Z + s);
        }
        uint32_t wm = 0;
        if constexpr (KDEAD) {
            per_half([&](auto hc) {
                constexpr int hh = decltype(hc)::value, NX = kFrPlan<BG>.nx[hh];
                static_assert(NX <= 32, "one liveness word per wave");
                T xv[NX];
                sfor<0, NX>([&](auto xc) {
                    constexpr int i = kFrPlan<BG>.xlist[hh][decltype(xc)::value];
                    constexpr int c = (Z - kFrPlan<BG>.off[i]) % Z;
                    const int x = c == 0 ? s : (int)min((uint32_t)(s + c), (uint32_t)(s + c - Z));
                    xv[decltype(xc)::value] = ldg(lrow_x, i * Z + x);
                });
                sfor<0, NX>([&](auto xc) {
                    constexpr int p = decltype(xc)::value;
                    wm |= (uint32_t)(__builtin_amdgcn_ballot_w64(FT<T>::bits(xv[p]) != 0) != 0) << p;
                });
            });
        }
#pragma unroll
        for (int jj = 0; jj < KH; ++jj) {
            const int j = jcol(jj);
            at((uint32_t)(j * kFrColB + s * 8)) = j < pc ? T(0) : v0[jj];
        }
        if (KDEAD && (t & 63) == 0) *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.fl_b + 16 + (t >> 6) * 4) = wm;
    }
    for (int w = t; w < kFrPlan<BG>.nls * Z; w += kFrThreads) {
        V2<T> v;
        v.x = T(0), v.y = T(0);
        *(lds_V2*)(uintptr_t)(uint32_t)(kFrPlan<BG>.st_b + w * 16) = v;
        *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.pk_b + w * 4) = 0u;
    }
    // wrap table: entry e < 2*Zc holds (e mod Zc) * 8
    *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.tbl_b + t * 4) = (uint32_t)s * 8u;
    if (t == 0) *flagA = 0, *anyf = 0;
    lds_barrier();
    uint64_t live_x = ~0ull;
    if constexpr (KDEAD) {
        constexpr int NW = kFrThreads / 64, HW = Z / 64;
        uint32_t m[2] = {0u, 0u};
#pragma unroll
        for (int w = 0; w < NW; ++w)
            m[w / HW] |= *(lds_u32*)(uintptr_t)(uint32_t)(kFrPlan<BG>.fl_b + 16 + w * 4);
        live_x = 0;
        sfor<0, 2>([&](auto hc) {
            constexpr int hh = decltype(hc)::value;
            const uint32_t mh = __builtin_amdgcn_readfirstlane(m[hh]);
            sfor<0, kFrPlan<BG>.nx[hh]>([&](auto xc) {
                constexpr int p = decltype(xc)::value;
                live_x |= (uint64_t)((mh >> p) & 1u) << (kFrPlan<BG>.xlist[hh][p] - 4);
            });
        });
    }

    const uint32_t sb0 = (uint32_t)s * 8u, sbw0 = sb0 - (uint32_t)(Z * 8);
    const uint32_t tz0 = (uint32_t)(kFrPlan<BG>.tbl_b + s * 4);
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)
    asm volatile("" : "+v"(mv));
    bool active = true;
    uint64_t hdx_keep = 0;   // extension decisions of a codeblock decided by the syndrome test
    int it = 0;
    if constexpr (KDEAD) {
        constexpr uint64_t all = (1ull << (MB - 4)) - 1;
        if (live_x != all) {
            constexpr bool DEAD = true;
#include "ldpc5g_dec_frame_iter.h"
        } else {
            constexpr bool DEAD = false;
#include "ldpc5g_dec_frame_iter.h"
        }
    } else {
        constexpr bool DEAD = false;
#include "ldpc5g_dec_frame_iter.h"
    }

    // ---- iterations exhausted: ck = (LQ <= 0), status = syndrome == 0 (:133-143)
    int sv = s;
    asm volatile("" : "+v"(sv));   // keep the output addresses out of the loop
    uint32_t sb = sb0, sbw = sbw0;
    asm volatile("" : "+v"(sb));
    asm volatile("" : "+v"(sbw));
    auto xposf = [&](int i) -> int {
        const int c = (Z - kFrPlan<BG>.off[i]) % Z;
        if (c == 0) return sv;
        return (int)min((uint32_t)(sv + c), (uint32_t)(sv + c - Z));
    };
    uint32_t oc = 0;          // own core columns (bit jj): LQ <= 0, or LQ_old < 0 if decided
    uint64_t ox = hdx_keep;   // own extension columns (check node of the row's frame)
    if (active) {
        ox = 0;
        per_half([&](auto hc) {
            constexpr int hh = decltype(hc)::value, NX = kFrPlan<BG>.nx[hh], XB = 8;
            sfor<0, (NX + XB - 1) / XB>([&](auto bc) {
                constexpr int x0 = decltype(bc)::value * XB, x1 = x0 + XB < NX ? x0 + XB : NX;
                T vx[XB];
                sfor<x0, x1>([&](auto xc) {
                    constexpr int i = kFrPlan<BG>.xlist[hh][decltype(xc)::value];
                    vx[decltype(xc)::value - x0] = ldg(lrow_x, i * Z + xposf(i));
                });
                __builtin_amdgcn_sched_barrier(0);
                sfor<x0, x1>([&](auto xc) {
                    constexpr int i = kFrPlan<BG>.xlist[hh][decltype(xc)::value];
                    constexpr int dl = kFrPlan<BG>.deg(i) - 1;   // ext column = last edge
                    T a, b;
                    uint32_t u, idx;
                    get_state(std::integral_constant<int, i>{}, a, b, u, idx);
                    const T r = xsign_v(pick(idx == (uint32_t)dl, b, a), u << dl, mv);
                    ox |= (uint64_t)(vx[decltype(xc)::value - x0] + r <= T(0)) << (i - 4);
                });
            });
        });
        bool fail = false;
        per_half([&](auto hc) {
            constexpr int hh = decltype(hc)::value;
            constexpr uint64_t rows = [] {
                uint64_t m = 0;
                for (int i = 0; i < P::MB; ++i)
                    if (kFrPlan<BG>.owner[i] == hh) m |= 1ull << i;
                return m;
            }();
            fail = syndrome_fails<BG, rows, false, T>(
                [&](auto ic, auto kc) -> T {
                    constexpr int i = decltype(ic)::value, k = decltype(kc)::value;
                    constexpr int c = (fr_sft<BG>(i, k) - kFrPlan<BG>.off[i] + Z) % Z;
                    return at((uint32_t)(P::COL[P::RS[i] + k] * kFrColB) + fr_rot(sb, sbw, c));
                },
                [&](auto ic) -> bool { return (ox >> (decltype(ic)::value - 4)) & 1u; });
        });
        if (fail) *flagA = 1;
    }
#pragma unroll
    for (int jj = 0; jj < KH; ++jj) {
        const T v = at((uint32_t)(jcol(jj) * kFrColB) + sb);
        oc |= (uint32_t)(active ? v <= T(0) : v < T(0)) << jj;
    }
    lds_barrier();   // every LQ / state read is done: LDS below the flags is free from here
    if (active && t == 0) {
        status[out] = *flagA == 0;
        iters[out] = L;
    }
    // ---- ck through LDS (ck_store_staged, ldpc5g_dec_body.h)
    constexpr int NFZ = P::NB * Z;
    static_assert(NFZ <= kFrPlan<BG>.fl_b, "ck staging below the flags");
#pragma unroll
    for (int jj = 0; jj < KH; ++jj) ck_stage_byte((uint32_t)(jcol(jj) * Z + sv), (oc >> jj) & 1u);
    per_half([&](auto hc) {
        sfor<4, MB>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (kFrPlan<BG>.owner[i] == decltype(hc)::value)
                ck_stage_byte((uint32_t)((KB + i) * Z + xposf(i)), (uint32_t)(ox >> (i - 4)) & 1u);
        });
    });
    const bool slow = block_any(!ck_row_aligned(NFZ, crow));   // orders the staging too
    ck_store_staged(NFZ, 1, [&](int) -> int8_t* { return crow; }, slow, t, kFrThreads);
}

// DEAD: rate-matched input (dead extension rows found per codeblock in frame_body's prologue)
template <int BG, bool OFS, bool DEAD>
__global__ __launch_bounds__(kFrThreads) __attribute__((amdgpu_waves_per_eu(3))) void ldpc_frame_kernel(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
    const DecWork* __restrict__ work, const CbRef* __restrict__ cbs) {
    frame_body<BG, OFS, DEAD>(llr, ck, status, iters, ldl, ldc, L, alpha, beta, pc, work, cbs);
}

template <int BG, bool DEAD>
int launch_frame_t(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg, int64_t ldl,
                   int64_t ldc, int L, double alpha, double beta, int pc, const DecWork* work,
                   const CbRef* cbs, hipStream_t st) {
    const bool ofs = beta != 0.0;
    constexpr size_t lds = (size_t)kFrPlan<BG>.bytes;
    if (int rc = ofs ? set_lds_once<ldpc_frame_kernel<BG, true, DEAD>>(lds)
                     : set_lds_once<ldpc_frame_kernel<BG, false, DEAD>>(lds))
        return rc;
    auto kern = ofs ? ldpc_frame_kernel<BG, true, DEAD> : ldpc_frame_kernel<BG, false, DEAD>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(kFrThreads), lds, st, llr, ck, status, iters, ldl, ldc, L, alpha,
                       beta, pc, work, cbs);
    return check_hip(hipGetLastError(), "ldpc_frame_kernel launch");
}

}  // namespace
}  // namespace ldpc5g_impl
