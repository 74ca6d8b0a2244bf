// ldpc5g_dec_body.h — layered min-sum decoder kernel (the perf schedule of py5gphy/ldpc/
// nr_ldpc_decode.py:51-143's min-sum) and the helpers the flooding decoder
// (ldpc5g_dec_flood.h) shares.  Instantiated by ldpc5g_dec_l.hip, which is built without the SLP
// vectorizer (build.py NO_SLP).  Reference mapping in ldpc5g_common.h / DESIGN.md §4.
#pragma once
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {
// ================================================================================== DECODER
template <typename T>
struct FT;
template <>
struct FT<float> {
    __device__ static __forceinline__ uint32_t sbits(float x) { return __float_as_uint(x); }
    __device__ static __forceinline__ uint32_t bits(float x) { return __float_as_uint(x); }
    // x with its sign bit XORed by bit 31 of `b`
    __device__ static __forceinline__ float xsign(float x, uint32_t b) {
        return __uint_as_float(__float_as_uint(x) ^ (b & 0x80000000u));
    }
    __device__ static __forceinline__ float inf() { return __uint_as_float(0x7f800000u); }
    __device__ static __forceinline__ float med3(float a, float b, float c) {
        return __builtin_amdgcn_fmed3f(a, b, c);
    }
};
template <>
struct FT<double> {
    __device__ static __forceinline__ uint32_t sbits(double x) { return (uint32_t)__double2hiint(x); }
    __device__ static __forceinline__ uint64_t bits(double x) { return (uint64_t)__double_as_longlong(x); }
    __device__ static __forceinline__ double xsign(double x, uint32_t b) {
        return __longlong_as_double(__double_as_longlong(x) ^ ((long long)(b & 0x80000000u) << 32));
    }
    __device__ static __forceinline__ double inf() { return __longlong_as_double(0x7ff0000000000000ll); }
    __device__ static __forceinline__ double med3(double a, double b, double c) {
        return fmax(fmin(a, b), fmin(fmax(a, b), c));
    }
};

template <typename T>
using V2 = T __attribute__((ext_vector_type(2)));

// Layered state: mA/mB carry the row sign (product of all q signs), pk bits d-1-k hold the sign
// of q_k (packed with v_alignbit, edge 0 highest), bits 24..28 the argmin edge.  Then
// r_k = (k == idx ? mB : mA) with its sign flipped by sign(q_k).
template <typename T>
__device__ __forceinline__ T decomp_l(T mAs, T mBs, uint32_t pk, uint32_t idx, int d, int k) {
    return FT<T>::xsign((idx == (uint32_t)k) ? mBs : mAs, pk << (32 - d + k));
}

// Consecutive base rows with disjoint core columns form one barrier group: processing them
// together is identical to processing them one after another (layered) and keeps the
// row-ascending accumulation order of every column (flooding).  BG1: 46 rows -> 32 groups,
// BG2: 42 -> 28.
template <int BG>
struct RowGroups {
    int n = 0;
    int start[64] = {};
    constexpr RowGroups() {
        using P = BGT<BG>;
        int g0 = 0;
        start[0] = 0;
        n = 1;
        for (int i = 1; i < P::MB; ++i) {
            bool dis = true;
            for (int a = g0; a < i && dis; ++a)
                for (int e = P::RS[a]; e < P::RS[a + 1]; ++e)
                    for (int f = P::RS[i]; f < P::RS[i + 1]; ++f)
                        if (P::COL[e] == P::COL[f] && P::COL[e] < P::KC) dis = false;
            if (!dis) {
                start[n++] = i;
                g0 = i;
            }
        }
        start[n] = P::MB;
    }
};
template <int BG>
constexpr RowGroups<BG> kGroups{};

// Packed shift words (2 edges per word) spanned by the edges of row group g.
template <int BG>
constexpr int group_w0(int g) { return BGT<BG>::RS[kGroups<BG>.start[g]] >> 1; }
template <int BG>
constexpr int group_nw(int g) {
    return ((BGT<BG>::RS[kGroups<BG>.start[g + 1]] - 1) >> 1) - group_w0<BG>(g) + 1;
}
template <int BG>
constexpr int max_group_nw() {
    int m = 0;
    for (int g = 0; g < kGroups<BG>.n; ++g) m = m > group_nw<BG>(g) ? m : group_nw<BG>(g);
    return m;
}
template <int BG>
__device__ __forceinline__ uint32_t shift_word(int zi, int w) {
    if constexpr (BG == 1) return kBG1ShiftMod[zi][w];
    else return kBG2ShiftMod[zi][w];
}


// Kernels for one lifting size (template argument ZCC > 0; used for Zc = 384, the size of every
// large codeblock): the shifts V(i,j) mod Zc are compile-time constants, so wrap-table reads take
// them as immediate offsets and no shift word is loaded from memory or unpacked on the scalar unit.
template <int ZC>
constexpr int zc_set() {
    for (int i = 0; i < LDPC5G_NUM_ZC; ++i)
        if (kLdpcZcList[i] == ZC) return kLdpcZcSet[i];
    return 0;
}
template <int BG, int ZC>
constexpr int zc_shift(int e) {
    if constexpr (BG == 1) return kBG1Shift[zc_set<ZC>()][e] % ZC;
    else return kBG2Shift[zc_set<ZC>()][e] % ZC;
}

// Layered: the (mA, mB) magnitudes of the first kLdsRows rows live in LDS rather than VGPRs, so
// the kernel fits the 168-VGPR budget of 3 waves/SIMD without scratch spills (spilling kernels
// are held to fewer resident waves).  2 x (40 KB APP + 33 KB state + 3 KB flags) <= 160 KB.
template <int BG>
constexpr int lds_rows() { return BG == 1 ? 11 : 18; }
// Layered rows with more edges than this recompute their rotated LDS addresses in pass 2.
// (Variants measured and dropped are listed in DESIGN.md §4.2; tools/ab/make_variants.py rebuilds
// them as separate libraries for side-by-side timing.)
constexpr int kRecompDeg = 12;
// LDS column stride (entries) = workgroup size: 768 for layered (the flooding kernel: 384 slots)
template <bool LAYERED>
constexpr int dec_cs() { return LAYERED ? kDecThreadsL : kDecThreads; }
constexpr int kMaxG = kDecThreadsL / 2;   // = 768 / min Zc (2): per-CB-slot flag entries

// APP of the core columns, (mA, mB) of the first lds_rows rows, flags, wrap table
template <int BG, typename T, bool LAYERED>
constexpr size_t dec_lds_bytes_t() {
    constexpr size_t CS = dec_cs<LAYERED>();
    return (size_t)BGT<BG>::KC * CS * sizeof(T) + (size_t)2 * lds_rows<BG>() * CS * sizeof(T) +
           (2 * kMaxG + 4) * sizeof(int) + (size_t)2 * CS * sizeof(uint32_t);
}

// Layered state words: rows 0..3 one word each (negs | idx << 24); rows >= 4 (degree <= 12) two
// 16-bit fields (negs | idx << 12) per word.
template <int BG>
constexpr bool ext_rows_fit16() {
    for (int i = 4; i < BGT<BG>::MB; ++i)
        if (BGT<BG>::RS[i + 1] - BGT<BG>::RS[i] > 12) return false;
    return true;
}
template <int BG>
constexpr int max_group_ext_rows() {
    int m = 0;
    for (int g = 0; g < kGroups<BG>.n; ++g) {
        int c = 0;
        for (int i = kGroups<BG>.start[g]; i < kGroups<BG>.start[g + 1]; ++i) c += i >= 4;
        m = m > c ? m : c;
    }
    return m;
}

// Rows of group g as bits (i - 4) of an extension-row mask, or 0 when the group holds one of the
// core rows 0..3 (those have no extension column and are never dead).
template <int BG>
constexpr uint64_t group_xmask(int g) {
    uint64_t m = 0;
    for (int i = kGroups<BG>.start[g]; i < kGroups<BG>.start[g + 1]; ++i) {
        if (i < 4) return 0;
        m |= 1ull << (i - 4);
    }
    return m;
}

// Workgroup barrier that orders LDS only.  Threads of the decoder never exchange data through
// global memory, and __syncthreads()'s global release would make every barrier wait (vmcnt(0))
// for the ext-LLR loads prefetched across it.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---- syndrome passes (final status, layered stop rule): the rows of ROWS in batches of <= 32 core
// edges, every rotated APP read of a batch issued before any is compared.  Written edge by edge, the
// compiler waited for each read before the next (s_waitcnt per edge: ~15 us per workgroup, 40 % of
// an iteration, for a pass with 1/3 of an iteration's instructions).
template <int BG>
constexpr int core_deg(int i) {
    int c = 0;
    for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i + 1]; ++e) c += BGT<BG>::COL[e] < BGT<BG>::KC;
    return c;
}
template <int BG, uint64_t ROWS>
struct SynPlan {
    int n = 0;
    int r0[64] = {}, r1[64] = {};
    constexpr SynPlan() {
        int e = 0;
        bool open = false;
        for (int i = 0; i < BGT<BG>::MB; ++i) {
            if (!((ROWS >> i) & 1u)) continue;
            const int c = core_deg<BG>(i);
            if (open && e + c > 32) r1[n++] = i, open = false;
            if (!open) r0[n] = i, e = 0, open = true;
            e += c;
        }
        if (open) r1[n++] = BGT<BG>::MB;
    }
};
template <int BG, uint64_t ROWS>
constexpr SynPlan<BG, ROWS> kSynPlan{};
// slot of core edge k of row i among the core edges of ROWS rows in [r0, i) + row i's first k
template <int BG, uint64_t ROWS>
constexpr int syn_slot(int r0, int i, int k) {
    int n = 0;
    for (int r = r0; r < i; ++r)
        if ((ROWS >> r) & 1u) n += core_deg<BG>(r);
    for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i] + k; ++e) n += BGT<BG>::COL[e] < BGT<BG>::KC;
    return n;
}
// true when some row of ROWS fails: parity over its core edges of (core(ic, kc) < 0) [STRICT] or
// (<= 0), XOR ext(ic) (the decision of the row's extension edge; rows >= 4 only; called without side
// effects).  VPAR: the parity is the sign bit of the XOR of the values' (high) words, all VALU (the
// compare + lane-mask XOR per edge ran on the CU's one scalar unit for all 12 waves), exact unless
// a value is +-0 — a min |v| per row detects that, and then (rare; one wave-uniform branch for the
// whole pass) the compare pass decides those lanes.  !VPAR: the compare pass (also the layered
// stop rule inside the iteration loop, where the VALU form's registers spilled).
template <int BG, uint64_t ROWS, bool STRICT, typename T, bool VPAR = false, typename Core, typename Ext>
__device__ __forceinline__ bool syndrome_fails(Core&& core, Ext&& ext) {
    using P = BGT<BG>;
    uint32_t fails = 0;
    bool zany = false;
    sfor<0, kSynPlan<BG, ROWS>.n>([&](auto bc) {
        constexpr int r0 = kSynPlan<BG, ROWS>.r0[decltype(bc)::value];
        constexpr int r1 = kSynPlan<BG, ROWS>.r1[decltype(bc)::value];
        constexpr int NE = syn_slot<BG, ROWS>(r0, r1, 0);
        T a[NE > 0 ? NE : 1];
        sfor<r0, r1>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr ((ROWS >> i) & 1u)
                sfor<0, P::RS[i + 1] - P::RS[i]>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    if constexpr (P::COL[P::RS[i] + k] < P::KC) a[syn_slot<BG, ROWS>(r0, i, k)] = core(ic, kc);
                });
        });
        __builtin_amdgcn_sched_barrier(0);
        T zm = FT<T>::inf();
        sfor<r0, r1>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr ((ROWS >> i) & 1u) {
                constexpr int n0 = syn_slot<BG, ROWS>(r0, i, 0), n1 = syn_slot<BG, ROWS>(r0, i + 1, 0);
                if constexpr (VPAR) {
                    uint32_t sx = 0;
                    sfor<n0, n1>([&](auto nc) {
                        constexpr int n = decltype(nc)::value;
                        if constexpr ((n - n0) % 2 == 1)
                            sx = __builtin_amdgcn_bitop3_b32(sx, FT<T>::sbits(a[n - 1]), FT<T>::sbits(a[n]), 0x96);
                        else if constexpr (n == n1 - 1)
                            sx ^= FT<T>::sbits(a[n]);
                        zm = fmin(zm, fabs(a[n]));
                    });
                    uint32_t par = sx >> 31;
                    if constexpr (i >= 4) par ^= (uint32_t)ext(ic);
                    fails |= par;
                } else {
                    bool pb = false;
                    if constexpr (i >= 4) pb = ext(ic);
                    sfor<n0, n1>([&](auto nc) {
                        const T v = a[decltype(nc)::value];
                        pb ^= STRICT ? v < T(0) : v <= T(0);
                    });
                    fails |= (uint32_t)pb;
                }
            }
        });
        if constexpr (VPAR) zany |= zm == T(0);
    });
    if constexpr (VPAR) {
        if (__builtin_amdgcn_ballot_w64(zany) != 0) {   // some lane saw a +-0: compare pass
            const bool slow = syndrome_fails<BG, ROWS, STRICT, T, false>(core, ext);
            if (zany) fails = slow;
        }
    }
    return fails != 0;
}
template <int BG>
constexpr uint64_t all_rows() { return BGT<BG>::MB >= 64 ? ~0ull : (1ull << BGT<BG>::MB) - 1; }

// ---- ck through LDS (both decoders).  The decisions of a workgroup's slots are staged in LDS in
// output order (byte j*Zc + z of slot s at s*SS, SS = Nf*Zc rounded up to 16) once the decoding is
// over, then written as 16-B pieces of whole rows: every 128-B line of ck is written once and in
// full (direct byte stores wrote 32-64 B per codeblock, column and wave).  A slot whose row is not
// 16-B aligned (Zc % 4 != 0, or an odd ck offset) takes a byte loop, still one row per slot.
__device__ __forceinline__ int ck_stage_stride(int NFZ) { return (NFZ + 15) & ~15; }
__device__ __forceinline__ void ck_stage_byte(uint32_t off, uint32_t bit) {
    *(__attribute__((address_space(3))) uint8_t*)(uintptr_t)off = (uint8_t)bit;
}
__device__ __forceinline__ bool ck_row_aligned(int NFZ, const int8_t* p) {
    return (NFZ & 15) == 0 && ((uintptr_t)p & 15) == 0;
}
// after the staging writes and a barrier; `slow`: some slot's row is unaligned (workgroup-uniform)
template <typename SlotDst>
__device__ __forceinline__ void ck_store_staged(int NFZ, int nslots, SlotDst&& slot_dst, bool slow,
                                                int t, int nthr) {
    using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
    using lds_u4 = __attribute__((address_space(3))) u32x4;
    using lds_u8 = __attribute__((address_space(3))) uint8_t;
    const int SS = ck_stage_stride(NFZ);
    const int nch = NFZ >> 4;
    for (int c = t; c < nslots * nch; c += nthr) {
        const int s = c / nch, k = c - s * nch;
        int8_t* dst = slot_dst(s);
        if (ck_row_aligned(NFZ, dst)) *(u32x4*)(dst + 16 * k) = *(lds_u4*)(uintptr_t)(uint32_t)(s * SS + 16 * k);
    }
    if (slow) {
        for (int c = t; c < nslots * NFZ; c += nthr) {
            const int s = c / NFZ, b = c - s * NFZ;
            int8_t* dst = slot_dst(s);
            if (!ck_row_aligned(NFZ, dst)) dst[b] = (int8_t)*(lds_u8*)(uintptr_t)(uint32_t)(s * SS + b);
        }
    }
}

// OFS = false: the caller guarantees beta == 0 (plain / normalized min-sum), so the offset and
// its clamp at 0 are compiled out (min >= +0 already; the result is identical).
// DEAD = true: the variant for rate-recovered inputs (LDPC5G_RATE_MATCHED), which detects and
// skips dead extension rows; DEAD = false compiles none of that (the headline kernel).
template <int BG, typename T, bool LAYERED, bool OFS = true, bool DEAD = false, int ZCC = 0>
__device__ __forceinline__ void dec_body(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int B, int Zc_u, int zi_u, int G_u, int64_t ldl, int64_t ldc,
    int L, T alpha, T beta, int pc, const DecWork* __restrict__ work,
    const CbRef* __restrict__ cbs) {
    // pc = number of leading punctured block columns absent from the LLR rows (2, or 0 when the
    // caller passes full-length rows as decode_ldpc(LLRin, H, ...) does, nr_ldpc_decode.py:51)
    static_assert(LAYERED, "the flooding schedule is ldpc5g_dec_flood.h");
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, TS = sizeof(T);
    constexpr int CS = dec_cs<LAYERED>();   // LDS column stride = workgroup size
    static_assert(ext_rows_fit16<BG>(), "packed layered state needs degree <= 12");
    constexpr int ST_B = KC * CS * TS;   // byte offsets in LDS: APP, then the LDS row state
    constexpr int NLR = lds_rows<BG>();
    constexpr int FLAG_B = ST_B + 2 * NLR * CS * TS;
    constexpr int TBL_B = FLAG_B + (2 * kMaxG + 4) * 4;   // wrap table, 2*CS entries
    static_assert(FLAG_B >= CS * P::NB + 15 * kMaxG, "ck staging (G * SS bytes) below the flags");
    extern __shared__ __align__(16) unsigned char smem[];

    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem != 0u)
        __builtin_trap();   // the byte-offset LDS addressing below assumes a zero base
    int Zc = Zc_u, zi = zi_u, G = G_u;
    const int t = threadIdx.x;
    if (work) {
        DecWork w = work[blockIdx.x];
        Zc = w.Zc, zi = w.zi, G = w.G;
    }
    constexpr bool kZ = ZCC > 0;   // compile-time lifting size (zc_shift): G = CS / ZCC slots
    static_assert(!kZ || CS % ZCC == 0, "Zc-specialised layered kernel");
    if constexpr (kZ) Zc = ZCC, G = CS / ZCC;
    // thread t = z*G + cl owns row z of codeblock slot cl; LDS column entries are interleaved the
    // same way (entry (z, cl) at byte (z*G + cl)*TS), so a cyclic shift never crosses CB slots
    const int z = t / G;
    const int cbl = t - z * G;
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
            // slots past the end of the batch keep lrow = llr (row 0 of CB 0): the ext-LLR
            // prefetch below is issued by every thread and must stay inside the caller's buffer
            const int cb = blockIdx.x * G + cbl;
            valid = cb < B;
            if (valid) {
                lrow = llr + (int64_t)cb * ldl;
                crow = ck + (int64_t)cb * ldc;
                out = cb;
            }
        }
    }
    const int cl = valid ? cbl : 0;
    // The row loop's ext-LLR loads as saddr accesses: a workgroup-uniform base (SGPRs: the first
    // codeblock of the workgroup, whose row has the lowest offset — ldpc5g_capi.hip build_plan sorts
    // a work item's codeblocks) plus a 32-bit per-lane byte offset (< 4 GiB: checked by the
    // launchers / the plan), instead of a per-lane 64-bit VALU address per load
    const T* lbase;
    uint32_t lofs = 0;
    if (work) {
        const int64_t off0 = cbs[work[blockIdx.x].first].llr_off;
        lbase = llr + off0;
        if (valid) lofs = (uint32_t)((lrow - lbase) * TS);
    } else {
        lbase = llr + (int64_t)blockIdx.x * G * ldl;
        if (valid) lofs = (uint32_t)((int64_t)cl * ldl * TS);
    }
    const int tzb = valid ? t * TS : 0;   // byte offset of this thread's own column entry
    const uint32_t GT = (uint32_t)(G * TS), ZGT = (uint32_t)(Zc * G * TS);
    const uint32_t tzbw = (uint32_t)tzb - ZGT;   // own entry one wrap back (negative -> huge)
    // global row index used in the iteration loop: threads outside any CB (z >= Zc or cb >= B)
    // use row 0 of CB 0, so loads issued without a branch stay in bounds
    const int zg = valid ? z : 0;
    int zv = zg, ziv = zi;   // made opaque per iteration (see the iteration loop)
    int* flagA = (int*)(smem + FLAG_B);
    int* flagB = flagA + kMaxG;
    // block-wide "any": the slot holds the epoch of the last call in which some thread voted yes.
    // No reset is needed; consecutive calls are separated by other barriers.  (__syncthreads_or
    // would pull in 256 B of static LDS, moving the dynamic base off 0 and costing a v_add per
    // edge address.)
    int* anyf = flagB + kMaxG;
    int epoch = 0;
    auto block_any = [&](bool p) -> bool {
        ++epoch;
        if (p) *anyf = epoch;
        lds_barrier();
        return *anyf == epoch;
    };
    // LDS is addressed by plain byte offsets: this kernel has no static LDS, so the dynamic block
    // starts at LDS address 0 (checked at entry) and no symbol base is added to every address.
    using lds_T = __attribute__((address_space(3))) T;
    auto at = [&](int byte) -> lds_T& { return *(lds_T*)(uintptr_t)(uint32_t)byte; };
    auto own = [&](int j) -> lds_T& { return at(j * CS * TS + tzb); };
    // channel LLR of the degree-1 extension column of row i = 4 + i4 (own column z)
    auto llrx = [&](int i4) -> T { return lrow[(KB + 4 + i4 - pc) * Zc + zv]; };

    // per-thread state of rows (i, z), i = 0..MB-1
    constexpr int NSP = 4 + (MB - 3) / 2;
    T sA[MB], sB[MB];
    uint32_t sP[NSP];
#pragma unroll
    for (int i = 0; i < MB; ++i) sA[i] = T(0), sB[i] = T(0);
    // (mA, mB) of row i: VGPRs, or LDS for the first NLR rows of the layered kernel
    auto getA = [&](auto ic) -> T {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NLR) return at(ST_B + (2 * i) * CS * TS + tzb);
        else return sA[i];
    };
    auto getB = [&](auto ic) -> T {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NLR) return at(ST_B + (2 * i + 1) * CS * TS + tzb);
        else return sB[i];
    };
    auto putAB = [&](auto ic, T a, T b) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < NLR) {
            at(ST_B + (2 * i) * CS * TS + tzb) = a;
            at(ST_B + (2 * i + 1) * CS * TS + tzb) = b;
        } else {
            sA[i] = a;
            sB[i] = b;
        }
    };
#pragma unroll
    for (int i = 0; i < NSP; ++i) sP[i] = 0u;
    // layered: row i's sign bits / argmin as one word (negs | idx << 24), whatever the storage
    auto get_row = [&](auto ic) -> uint32_t {
        constexpr int i = decltype(ic)::value;
        constexpr int d = P::RS[i + 1] - P::RS[i];
        if constexpr (i < 4) {
            return sP[i];
        } else {
            constexpr int w = 4 + (i - 4) / 2;
            const uint32_t f = ((i - 4) & 1) ? (sP[w] >> 16) : (sP[w] & 0xffffu);
            return (f & ((1u << d) - 1u)) | ((f >> 12) << 24);
        }
    };
    auto put_row = [&](auto ic, uint32_t negs, uint32_t idx) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < 4) {
            sP[i] = negs | (idx << 24);
        } else {
            constexpr int w = 4 + (i - 4) / 2;
            const uint32_t f = negs | (idx << 12);
            sP[w] = ((i - 4) & 1) ? ((sP[w] & 0xffffu) | (f << 16)) : ((sP[w] & 0xffff0000u) | f);
        }
    };

    uint32_t hdc_prev = 0;   // hard decisions of own core columns, last iteration end
    uint64_t hdx_prev = 0;   // ... of own extension columns
    uint64_t nzx = 0;        // extension columns whose LLR is not +0.0 (bit pattern) at this z
    if (valid) {
        // all Nf - pc loads are issued before any is used: one HBM round trip per workgroup
        // (a conditional load per punctured column made 26 + 6 dependent round trips, ~40 us)
        // (the extension LLRs only for DEAD, for the live-row mask: otherwise their initial hard
        // decisions are taken in iteration 0 from the loads the row loop issues anyway)
        T vc[KC], vx[MB - 4];
#pragma unroll
        for (int j = 0; j < KC; ++j) vc[j] = lrow[(j < pc ? 0 : j - pc) * Zc + z];
        if constexpr (DEAD)
#pragma unroll
            for (int i4 = 0; i4 < MB - 4; ++i4) vx[i4] = lrow[(KB + 4 + i4 - pc) * Zc + z];
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            const T v = j < pc ? T(0) : vc[j];   // punctured columns: LLR 0 (:43)
            own(j) = v;
            hdc_prev |= (uint32_t)(v < T(0)) << j;
        }
        if constexpr (DEAD)
#pragma unroll
            for (int i4 = 0; i4 < MB - 4; ++i4) {
                const T v = vx[i4];
                hdx_prev |= (uint64_t)(v < T(0)) << i4;
                nzx |= (uint64_t)(FT<T>::bits(v) != 0) << i4;
            }
    }
    for (int w = 0; w < 2 * NLR; ++w) at(ST_B + w * CS * TS + tzb) = T(0);
    if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
    uint32_t* livew = (uint32_t*)(anyf + 2);   // workgroup OR of nzx (2 words)
    if (t == 0) *anyf = 0;
    if constexpr (DEAD)
        if (t == 0) livew[0] = 0u, livew[1] = 0u;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    {   // T[e] = byte offset of entry e mod (Zc*G), e in [0, 2*Zc*G)
        const int ZG = Zc * G;
        if (t < ZG) {
            *(lds_u32*)(uintptr_t)(uint32_t)(TBL_B + t * 4) = (uint32_t)(t * 4);
            *(lds_u32*)(uintptr_t)(uint32_t)(TBL_B + (t + ZG) * 4) = (uint32_t)(t * 4);
        }
    }
    const uint32_t tzbT0 = (uint32_t)(TBL_B + (valid ? t : 0) * 4);
    // kZ: the table base is re-made opaque each iteration, so the compile-time shift offsets stay
    // immediates and LICM does not hoist ~300 constant addresses into VGPRs
    uint32_t tzbT = tzbT0;
    bool active = valid;
    lds_barrier();
    // Dead extension rows: a row whose degree-1 column has LLR +0.0 for every codeblock slot of the
    // workgroup (punctured by rate matching: high code rates leave most parity columns untransmitted)
    // sends exactly +-0 to every core column (its min |q| is the zero of the extension edge), so the
    // core APPs never change through it; only its extension decision r_ext = sign * alpha *
    // max(min|q_core| - beta, 0) does.  Such rows run dead_row (pass 1 without the old-message
    // rebuild, no APP writes) and consecutive dead groups share one barrier: bit-identical results.
    // gdm: bit g set when every row of group g is dead (a workgroup-uniform SGPR)
    uint32_t gdm = 0;
    if constexpr (DEAD) {
        if (nzx & 0xffffffffu) atomicOr(&livew[0], (uint32_t)nzx);
        if (nzx >> 32) atomicOr(&livew[1], (uint32_t)(nzx >> 32));
        lds_barrier();
        const uint64_t live_x = ((uint64_t)__builtin_amdgcn_readfirstlane(livew[1]) << 32) |
                                (uint64_t)__builtin_amdgcn_readfirstlane(livew[0]);
        sfor<0, kGroups<BG>.n>([&](auto gc) {
            constexpr uint64_t m = group_xmask<BG>(decltype(gc)::value);
            if constexpr (m != 0)
                if ((live_x & m) == 0) gdm |= 1u << decltype(gc)::value;
        });
        gdm = __builtin_amdgcn_readfirstlane(gdm);
    }
    auto gdead = [&](auto gc) -> bool {
        constexpr int g = decltype(gc)::value;
        if constexpr (!DEAD || group_xmask<BG>(g) == 0) return false;
        else return (gdm >> g) & 1u;
    };

    // byte offset (without the column base) of column entry (z + s) mod Zc of this thread
    // ((z + s) mod Zc, cl): the unwrapped candidate is tzb + s*GT; when z + s >= Zc the wrapped
    // one tzbw + s*GT is a valid (smaller) offset, otherwise it is negative, i.e. a huge unsigned.
    auto rot = [&](int s) -> int {
        const uint32_t S = (uint32_t)s * GT;
        return (int)min((uint32_t)tzb + S, tzbw + S);
    };

    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)
    asm volatile("" : "+v"(mv));
    int it = 0;
    for (; it < L; ++it) {
        // zv / ziv are re-materialised opaque each iteration: otherwise LICM hoists the ~300
        // loop-invariant column addresses (z + V) mod Zc out of the loop into VGPRs/SGPRs.
        zv = zg;
        ziv = zi;
        asm volatile("" : "+v"(zv));
        asm volatile("" : "+s"(ziv));
        if constexpr (kZ) {
            tzbT = tzbT0;
            asm volatile("" : "+v"(tzbT));
        }
        bool fail = false;
        uint64_t hdx = 0;   // ext hard decisions at the end of the pass
        // ---- layered row i: q = APP - r_old, APP = q + r_new.
        //      Op choice follows the gfx950 VALU rates measured by tools/microbench/valu_rates.hip: f32
        //      add/sub and all-VGPR bitwise ops (and, xor, bitop3, u32 add) issue at twice the
        //      rate of min/max/med3, compares and any op with an SGPR or literal operand.  So the
        //      sign mask lives in a VGPR (mv) and the sign bits are walked with u + u.
        auto layered_row = [&](auto ic, auto& gshift, T xl) {
            constexpr int i = decltype(ic)::value;
            constexpr int e0 = P::RS[i];
            constexpr int d = P::RS[i + 1] - e0;
            const T mAs = getA(ic), mBs = getB(ic);
            const uint32_t pk = get_row(ic);
            // opaque: otherwise the shift folds into an SDWA byte-select compare, which cannot take
            // the edge index as an inline constant, and every edge pays a v_mov for it
            uint32_t idxo = pk >> 24;
            asm volatile("" : "+v"(idxo));
            uint32_t u = pk << (32 - d);   // bit 31 = sign of q_k for the edge k being visited
            T q[d];
            int rb[d];
            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                if constexpr (j < KC) {
                    const T sel = (idxo == (uint32_t)k) ? mBs : mAs;
                    const T rold = __uint_as_float(__builtin_amdgcn_bitop3_b32(u, __float_as_uint(sel), mv, 0x6c));
                    // rotated entry (z + s) mod Zc: the wrap table maps the unwrapped offset
                    rb[k] = (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)gshift(e0 + k) * GT);
                    q[k] = at(j * CS * TS + rb[k]) - rold;
                } else {
                    q[k] = xl;   // degree-1 column: q is the channel LLR itself
                    if constexpr (!DEAD)   // initial hard decision of the ext column (see prologue)
                        if (it == 0) hdx_prev |= (uint64_t)(xl < T(0)) << (i - 4);
                }
                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1, all-VGPR form
                const T aq = fabs(q[k]);
                min2 = FT<T>::med3(min1, min2, aq);
                min1 = fmin(min1, aq);
                if constexpr (k % 2 == 1)   // three-input XOR
                    sx = __builtin_amdgcn_bitop3_b32(sx, FT<T>::sbits(q[k - 1]), FT<T>::sbits(q[k]), 0x96);
                else if constexpr (k == d - 1)
                    sx ^= FT<T>::sbits(q[k]);
            });
            T x1 = min1, x2 = min2;
            if constexpr (OFS) {
                x1 = min1 - beta, x2 = min2 - beta;
                x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
            }
            const T nAs = FT<T>::xsign(alpha * x1, sx);
            const T nBs = FT<T>::xsign(alpha * x2, sx);
            uint32_t negs = 0, idxn = 0;
            // High-degree rows (BG1 rows 0-3, d = 19): keeping all d rotated addresses live from
            // pass 1 to pass 2 beside the d messages overflows the 168-VGPR budget (scratch spills
            // reloaded inside the iteration loop); their addresses are looked up again from an
            // opaque copy of the table base instead (1 VALU + 1 LDS read per edge, no CSE).
            constexpr bool RECOMP = d > kRecompDeg;
            uint32_t tzbT2 = tzbT;
            if constexpr (RECOMP) asm volatile("" : "+v"(tzbT2));
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                const uint32_t qb = FT<T>::sbits(q[k]);
                const bool isMin = fabs(q[k]) == min1;   // ties: nB == nA, either is right
                idxn = isMin ? (uint32_t)k : idxn;
                const T sel = isMin ? nBs : nAs;
                const T r = __uint_as_float(__builtin_amdgcn_bitop3_b32(qb, __float_as_uint(sel), mv, 0x6c));
                negs = __builtin_amdgcn_alignbit(negs, qb, 31);
                const T app = q[k] + r;
                if constexpr (j < KC) {
                    if constexpr (RECOMP) {
                        const uint32_t S = (uint32_t)gshift(e0 + k) * GT;
                        at(j * CS * TS + (int)*(lds_u32*)(uintptr_t)(tzbT2 + S)) = app;
                    } else {
                        at(j * CS * TS + rb[k]) = app;
                    }
                } else {
                    hdx |= (uint64_t)(app < T(0)) << (i - 4);
                }
            });
            putAB(ic, nAs, nBs);
            put_row(ic, negs, idxn);
        };
        // dead extension row (q_ext = +0, so min1 = 0 and every core r is +-0): q_k = APP_k - (+-0)
        // = APP_k up to the sign of a zero; only the extension message changes:
        // r_ext = sign(prod q_k) * alpha * max(min |q_k| - beta, 0) (min2 of the row), APP_ext =
        // 0 + r_ext.  State as the full update leaves it: mA = +-0, mB = r_ext, argmin = the
        // extension edge (last), its sign bit 0.
        auto dead_row = [&](auto ic, auto& gshift) {
            constexpr int i = decltype(ic)::value;
            constexpr int e0 = P::RS[i];
            constexpr int d = P::RS[i + 1] - e0;
            T mn = FT<T>::inf();
            uint32_t sx = 0;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                if constexpr (j < KC) {
                    const int rbk = (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)gshift(e0 + k) * GT);
                    const T a = at(j * CS * TS + rbk);
                    mn = fmin(mn, fabs(a));
                    sx ^= FT<T>::sbits(a);
                }
            });
            T x2 = mn;
            if constexpr (OFS) {
                x2 = mn - beta;
                x2 = x2 > T(0) ? x2 : T(0);
            }
            const T nBs = FT<T>::xsign(alpha * x2, sx);
            hdx |= (uint64_t)(nBs < T(0)) << (i - 4);
            putAB(ic, T(0), nBs);
            put_row(ic, 0u, (uint32_t)(d - 1));
        };
        // the next row group's packed shift words are loaded (scalar, wave-uniform) before the
        // barrier that precedes the group, so their latency hides behind it
        constexpr int NPW = max_group_nw<BG>();
        constexpr int NXR = max_group_ext_rows<BG>() > 0 ? max_group_ext_rows<BG>() : 1;
        uint32_t nsw[NPW];
        T xlb[2][NXR] = {};   // layered: ext-column LLRs of rows >= 4, double-buffered by group parity
        auto prefetch = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (kZ) return;
            sfor<0, group_nw<BG>(g)>([&](auto wc) {
                constexpr int w = decltype(wc)::value;
                nsw[w] = shift_word<BG>(ziv, group_w0<BG>(g) + w);
            });
        };
        // layered: the ext-column LLRs of group g are loaded from global memory at the start of
        // group g - 1, so a whole group's work hides the L2 / Infinity-Cache latency
        auto prefetch_xl = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            constexpr int r0 = kGroups<BG>.start[g] > 4 ? kGroups<BG>.start[g] : 4;
            sfor<r0, (kGroups<BG>.start[g + 1] > r0 ? kGroups<BG>.start[g + 1] : r0)>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                // unconditional (see zg); row base uniform, lane part 32-bit: one saddr load
                using gT = const __attribute__((address_space(1))) T;
                using gB = const __attribute__((address_space(1))) unsigned char;
                gB* rowb = (gB*)(uintptr_t)lbase + (uint32_t)((KB + i - pc) * Zc * TS);
                xlb[g & 1][i - r0] = *(gT*)(rowb + (lofs + (uint32_t)zv * (uint32_t)TS));
            });
        };
        prefetch(std::integral_constant<int, 0>{});
        prefetch_xl(std::integral_constant<int, 0>{});   // row 0 has no ext column: no load
        sfor<0, kGroups<BG>.n>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            uint32_t csw[NPW];
#pragma unroll
            for (int x = 0; x < NPW; ++x) csw[x] = nsw[x];
            if constexpr (g + 1 < kGroups<BG>.n) {
                if (!gdead(std::integral_constant<int, g + 1>{}))   // dead groups load nothing
                    prefetch_xl(std::integral_constant<int, g + 1>{});
            }
            auto gshift = [&](int e) -> int {   // e compile-time after unrolling
                if constexpr (kZ) return zc_shift<BG, ZCC>(e);
                const uint32_t w = csw[(e >> 1) - group_w0<BG>(g)];
                return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
            };
            const bool dead = gdead(gc);
            if (active) {
                if constexpr (DEAD && group_xmask<BG>(g) != 0) {
                    if (dead)
                        sfor<kGroups<BG>.start[g], kGroups<BG>.start[g + 1]>([&](auto ic) { dead_row(ic, gshift); });
                }
                if (!dead) {
                    sfor<kGroups<BG>.start[g], kGroups<BG>.start[g + 1]>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        constexpr int r0 = kGroups<BG>.start[g] > 4 ? kGroups<BG>.start[g] : 4;
                        layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));
                    });
                }
            }
            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});
            // dead rows only read the APPs: two dead groups in a row need no barrier between them
            if constexpr (g + 1 < kGroups<BG>.n) {
                if (!(dead && gdead(std::integral_constant<int, g + 1>{}))) lds_barrier();
            } else {
                lds_barrier();
            }
        });

        const int clq = valid ? t - zv * G : 0;
        {
            // ---- layered stopping rule: no hard decision changed over the iteration, then an
            //      exact syndrome check of those decisions (oracle.decode_layered)
            uint32_t hdc = 0;
            if (active)
                for (int j = 0; j < KC; ++j) hdc |= (uint32_t)(own(j) < T(0)) << j;
            if (active && (hdc != hdc_prev || hdx != hdx_prev)) flagA[clq] = 1;
            // a stopped slot keeps the decisions of its stopping iteration (staged at the end)
            if (active) hdc_prev = hdc, hdx_prev = hdx;
            lds_barrier();
            const bool cand = active && flagA[clq] == 0;
            if (block_any(cand)) {
                if (cand) {
                    const bool sf = syndrome_fails<BG, all_rows<BG>(), true, T, false>(
                        [&](auto ic, auto kc) -> T {
                            constexpr int e = P::RS[decltype(ic)::value] + decltype(kc)::value;
                            if constexpr (kZ)   // the wrap table: immediate offsets, no VALU
                                return at(P::COL[e] * CS * TS +
                                          (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)zc_shift<BG, ZCC>(e) * GT));
                            else
                                return at(P::COL[e] * CS * TS + rot(shift_of<BG>(ziv, e)));
                        },
                        [&](auto ic) -> bool { return (hdx >> (decltype(ic)::value - 4)) & 1u; });
                    if (sf) flagB[clq] = 1;
                }
                lds_barrier();
                if (cand && flagB[clq] == 0) {
                    if (z == 0) {
                        int tq = t;
                        asm volatile("" : "+v"(tq));
                        const int cq = tq - zv * G;
                        const int oq = work ? cbs[work[blockIdx.x].first + cq].out : (int)blockIdx.x * G + cq;
                        status[oq] = 1, iters[oq] = it + 1;
                    }
                    active = false;
                }
            }
        }
        lds_barrier();
        if (z == 0 && valid) flagA[clq] = 0, flagB[clq] = 0;
        if (!block_any(active)) break;
    }

    // r of edge k of row i from the stored state (layout depends on the schedule)
    auto rfinal = [&](auto ic, int d, int k) -> T {
        const uint32_t pk = get_row(ic);
        return decomp_l(getA(ic), getB(ic), pk, pk >> 24, d, k);
    };
    // ---- iterations exhausted: ck = (APP <= 0), status = syndrome == 0 (:133-143)
    // rotated address for the final syndrome pass, multiplied on the VALU (v_mul_u32_u24 with an
    // opaque VGPR stride): the scalar unit is shared by the workgroup's 12 waves
    uint32_t GTv = GT;
    asm volatile("" : "+v"(GTv));
    auto rot_v = [&](int sft) -> int {
        const uint32_t S = __umul24((uint32_t)sft, GTv);
        return (int)min((uint32_t)tzb + S, tzbw + S);
    };
    zv = z;
    asm volatile("" : "+v"(zv));   // keep the output addresses out of the loop (no hoist/spill)
    int t2 = t;
    asm volatile("" : "+v"(t2));
    const int cl2 = t2 - zv * G;   // zv = z here (no division)
    int out2 = 0;
    const T* lrow2 = llr;
    if (valid) {
        if (work) {
            const CbRef r2 = cbs[work[blockIdx.x].first + cl2];
            out2 = r2.out, lrow2 = llr + r2.llr_off;
        } else {
            out2 = (int)blockIdx.x * G + cl2, lrow2 = llr + (int64_t)out2 * ldl;
        }
    }
    auto llrx2 = [&](int i4) -> T { return lrow2[(KB + 4 + i4 - pc) * Zc + zv]; };
    if (active) {
        // extension decisions first, their LLRs requested in batches of 14 before any is used (one
        // load per row made the scheduler serialise them; all 42 at once spill), so the row state
        // is dead before the syndrome pass
        uint64_t ox = 0;
        constexpr int XB = 14, NX = MB - 4;
        sfor<0, (NX + XB - 1) / XB>([&](auto bc) {
            constexpr int x0 = decltype(bc)::value * XB, x1 = x0 + XB < NX ? x0 + XB : NX;
            T vx[XB];
            sfor<x0, x1>([&](auto xc) { vx[decltype(xc)::value - x0] = llrx2(decltype(xc)::value); });
            __builtin_amdgcn_sched_barrier(0);
            sfor<x0, x1>([&](auto xc) {
                constexpr int i = decltype(xc)::value + 4;
                constexpr int dl = P::RS[i + 1] - P::RS[i] - 1;   // ext column = last edge
                ox |= (uint64_t)(vx[i - 4 - x0] + rfinal(std::integral_constant<int, i>{}, dl + 1, dl) <= T(0)) << (i - 4);
            });
        });
        const bool fail = syndrome_fails<BG, all_rows<BG>(), false, T>(
            [&](auto ic, auto kc) -> T {
                constexpr int e = P::RS[decltype(ic)::value] + decltype(kc)::value;
                return at(P::COL[e] * CS * TS + rot_v(shift_of<BG>(zi, e)));
            },
            [&](auto ic) -> bool { return (ox >> (decltype(ic)::value - 4)) & 1u; });
        if (fail) flagA[cl2] = 1;
        uint32_t oc = 0;
        for (int j = 0; j < KC; ++j) oc |= (uint32_t)(own(j) <= T(0)) << j;
        hdc_prev = oc, hdx_prev = ox;
    }
    lds_barrier();   // every APP / state read is done: LDS below FLAG_B is free from here
    if (active && z == 0) {
        status[out2] = flagA[cl2] == 0;
        iters[out2] = L;
    }
    // ---- ck through LDS (ck_store_staged): LDS below FLAG_B is free, and G * SS <= 768 * Nf + 15 * G
    //      fits it for every Zc
    {
        const int NFZ = P::NB * Zc;
        if (valid) {
            const uint32_t sb = (uint32_t)(cl2 * ck_stage_stride(NFZ) + zv);
            for (int j = 0; j < KC; ++j) ck_stage_byte(sb + (uint32_t)(j * Zc), (hdc_prev >> j) & 1u);
            for (int i4 = 0; i4 < MB - 4; ++i4)
                ck_stage_byte(sb + (uint32_t)((KB + 4 + i4) * Zc), (uint32_t)(hdx_prev >> i4) & 1u);
        }
        int8_t* crow2 = ck;
        if (valid) crow2 = work ? ck + cbs[work[blockIdx.x].first + cl2].ck_off : ck + (int64_t)out2 * ldc;
        const bool slow = block_any(valid && !ck_row_aligned(NFZ, crow2));   // orders the staging too
        const int nslots = work ? G : min(G, B - (int)blockIdx.x * G);
        ck_store_staged(NFZ, nslots, [&](int sl) -> int8_t* {
            if (work) return ck + cbs[work[blockIdx.x].first + sl].ck_off;
            return ck + (int64_t)((int)blockIdx.x * G + sl) * ldc;
        }, slow, t, (int)blockDim.x);
    }
}

#define LDPC5G_DEC_PARAMS                                                                        \
    const T *__restrict__ llr, int8_t *__restrict__ ck, uint8_t *__restrict__ status,             \
        int32_t *__restrict__ iters, int B, int Zc_u, int zi_u, int G_u, int64_t ldl, int64_t ldc, \
        int L, T alpha, T beta, int pc, const DecWork *__restrict__ work,                          \
        const CbRef *__restrict__ cbs
#define LDPC5G_DEC_ARGS \
    llr, ck, status, iters, B, Zc_u, zi_u, G_u, ldl, ldc, L, alpha, beta, pc, work, cbs

// layered float32: 768 threads = 12 waves = 3 per SIMD (<= 168 VGPRs), G = floor(768/Zc) CBs
template <int BG, typename T, bool LAYERED, bool OFS, bool DEAD = false, int ZCC = 0>
__global__ __launch_bounds__(kDecThreadsL) __attribute__((amdgpu_waves_per_eu(3))) void
ldpc_dec_kernel_l(LDPC5G_DEC_PARAMS) {
    dec_body<BG, T, LAYERED, OFS, DEAD, ZCC>(LDPC5G_DEC_ARGS);
}
template <int BG, typename T, bool LAYERED, bool OFS = true, bool DEAD = false, int ZCC = 0>
constexpr auto dec_kernel() {
    static_assert(LAYERED, "the flooding kernels are in ldpc5g_dec_flood.h");
    return ldpc_dec_kernel_l<BG, T, LAYERED, OFS, DEAD, ZCC>;
}

template <int BG, typename T, bool LAYERED>
size_t dec_lds_bytes() {
    static_assert(dec_lds_bytes_t<BG, T, LAYERED>() <= 160 * 1024, "LDS budget of one CU");
    return dec_lds_bytes_t<BG, T, LAYERED>();
}

// the kernel for one (OFS, ZCC) pair
template <int BG, typename T, bool LAYERED, bool DEAD, int ZCC>
int launch_dec_zc(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                  int G, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    auto kern = beta != 0.0 ? dec_kernel<BG, T, LAYERED, true, DEAD, ZCC>() : dec_kernel<BG, T, LAYERED, false, DEAD, ZCC>();
    const size_t lds = dec_lds_bytes<BG, T, LAYERED>();
    const int threads = ((G * Zc + 63) / 64) * 64;
    const int grid = (B + G - 1) / G;
    if (int rc = beta != 0.0 ? set_lds_once<dec_kernel<BG, T, LAYERED, true, DEAD, ZCC>()>(lds)
                             : set_lds_once<dec_kernel<BG, T, LAYERED, false, DEAD, ZCC>()>(lds))
        return rc;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, st, llr, ck, status, iters, B, Zc, zi,
                       G, ldl, ldc, L, (T)alpha, (T)beta, pc, (const DecWork*)nullptr,
                       (const CbRef*)nullptr);
    return check_hip(hipGetLastError(), "ldpc_dec_kernel launch");
}

template <int BG, typename T, bool LAYERED, bool DEAD = false>
int launch_dec_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                 int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    // small batches (the per-codeblock drop-ins): no more slots than codeblocks, so one BG2 Zc=8
    // codeblock runs as a single wave and its ~30 row-group barriers per iteration are cheap
    const int G = std::min(dec_G(Zc, LAYERED), B);
    if ((int64_t)G * ldl * (int64_t)sizeof(T) >= ((int64_t)1 << 32))   // 32-bit lane offsets (dec_body)
        return fail(LDPC5G_ESIZE, "ldl=%lld: a workgroup's %d LLR rows span >= 4 GiB", (long long)ldl, G);
    constexpr int ZL = 384;   // BG1's largest lifting size has its own kernel (zc_shift)
    if constexpr (BG == 1)
        if (Zc == ZL && G == dec_cs<LAYERED>() / ZL)
            return launch_dec_zc<BG, T, LAYERED, DEAD, ZL>(llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L,
                                                           alpha, beta, pc, st);
    return launch_dec_zc<BG, T, LAYERED, DEAD, 0>(llr, ck, status, iters, B, Zc, zi, G, ldl, ldc, L, alpha,
                                                  beta, pc, st);
}

// ZCC > 0: every work item is a Zc = ZCC item with a full G (ldpc5g_capi.hip build_plan puts them last)
template <int BG, typename T, bool LAYERED, bool DEAD = false, int ZCC = 0>
int launch_dec_mixed_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                       const DecWork* work, const CbRef* cbs, int L, double alpha, double beta,
                       int pc, hipStream_t st) {
    auto kern = beta != 0.0 ? dec_kernel<BG, T, LAYERED, true, DEAD, ZCC>() : dec_kernel<BG, T, LAYERED, false, DEAD, ZCC>();
    const size_t lds = dec_lds_bytes<BG, T, LAYERED>();
    if (int rc = beta != 0.0 ? set_lds_once<dec_kernel<BG, T, LAYERED, true, DEAD, ZCC>()>(lds)
                             : set_lds_once<dec_kernel<BG, T, LAYERED, false, DEAD, ZCC>()>(lds))
        return rc;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(dec_cs<LAYERED>()), lds, st, llr, ck, status, iters, 0, 0,
                       0, 0, (int64_t)0, (int64_t)0, L, (T)alpha, (T)beta, pc, work, cbs);
    return check_hip(hipGetLastError(), "ldpc_dec_kernel(mixed) launch");
}

template <int BG, typename T, bool LAYERED>
int blocks_per_cu_t() {
    auto kern = dec_kernel<BG, T, LAYERED>();
    const size_t lds = dec_lds_bytes<BG, T, LAYERED>();
    if (set_lds_once<dec_kernel<BG, T, LAYERED>()>(lds)) return -1;
    int n = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, dec_cs<LAYERED>(), lds) != hipSuccess) return -1;
    return n;
}

}  // namespace
}  // namespace ldpc5g_impl
