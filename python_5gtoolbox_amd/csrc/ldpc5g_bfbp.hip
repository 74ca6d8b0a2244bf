// ldpc5g_bfbp.hip — hard-decision bit flipping (BF) and float64 sum-product (BP) decoders.
//
//   BF : py5gphy/ldpc/ldpc_decoder_bit_flipping.py:5-73 (reached via nr_decode_ldpc(algo='BF'))
//        ck = hard decisions of LLR (LLR == 0 -> 0); per iteration: syndrome S; return if 0;
//        En[c] = sum over the checks of column c of (2S-1); flip every bit with En == max(En);
//        after L iterations return (ck, False) — no final syndrome (:45-73).
//   BP : py5gphy/ldpc/nr_ldpc_decode.py:51-143 with _BP_process :145-176, flooding, float64:
//        Lr = 2 atanh(prod tanh(Lq/2) / tanh(Lq_k/2)), clipped to +-2*19.07 when |.| >= 1;
//        one zero among the row's Lq: only that edge gets prod(tanh of the others) (the
//        reference assigns the product itself there, no atanh — reproduced); >= 2 zeros: 0.
//        Per-edge messages do not compress, so they live in a caller-provided float64 scratch
//        [B][E][Zc] (coalesced over z); APP and the row-ascending accumulator are in LDS as in
//        the min-sum flooding kernel.
// Thread mapping as the min-sum decoder: one thread per check row z, G = 384/Zc codeblocks
// per workgroup.  BP walks the rows with a runtime loop (scalar table reads, tanh / atanh inlined
// once) and parks tanh(Lq/2) in the message scratch between its two passes: no per-thread arrays.
#include <stdint.h>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {

// Column adjacency of a base graph: for column j, the (row, edge) pairs in ascending row order.
template <int BG>
struct ColLists {
    int start[80] = {};
    int row[330] = {};
    int edge[330] = {};
    constexpr ColLists() {
        using P = BGT<BG>;
        int cnt[80] = {};
        for (int e = 0; e < P::E; ++e) ++cnt[P::COL[e]];
        start[0] = 0;
        for (int j = 0; j < P::NB; ++j) start[j + 1] = start[j] + cnt[j];
        int fill[80] = {};
        for (int i = 0; i < P::MB; ++i)
            for (int e = P::RS[i]; e < P::RS[i + 1]; ++e) {
                const int j = P::COL[e];
                row[start[j] + fill[j]] = i;
                edge[start[j] + fill[j]] = e;
                ++fill[j];
            }
    }
};
template <int BG>
constexpr ColLists<BG> kCols{};

constexpr int kBfThreads = 384;

// ------------------------------------------------------------------------------------- BF
template <int BG, typename T>
__global__ __launch_bounds__(kBfThreads) void ldpc_bf_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int B, int Zc, int zi, int G, int64_t ldl, int64_t ldc, int L,
    int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, NB = P::NB;
    extern __shared__ __align__(16) unsigned char smem[];
    int8_t* hd = (int8_t*)smem;                 // [NB][kCS] hard decisions
    int8_t* S = hd + NB * kCS;                  // [MB][kCS] syndrome bits
    int* red = (int*)(S + MB * kCS);            // [2][kCS] per-CB flags / max
    const int t = threadIdx.x;
    const int cbl = t / Zc, z = t - cbl * Zc;
    const int cb = blockIdx.x * G + cbl;
    const bool valid = cbl < G && cb < B;
    const int cl = valid ? cbl : 0;
    const int tz = cl * Zc + z;
    const T* lrow = llr + (int64_t)(valid ? cb : 0) * ldl;
    int8_t* crow = ck + (int64_t)(valid ? cb : 0) * ldc;
    int* anyS = red;
    int* mx = red + kCS;
    auto rotp = [&](int s) { int m = z + s; return cl * Zc + (m >= Zc ? m - Zc : m); };   // (z+s)%Zc
    auto rotm = [&](int s) { int m = z - s; return cl * Zc + (m < 0 ? m + Zc : m); };     // (z-s)%Zc

    if (valid)
        for (int j = 0; j < NB; ++j) {
            const T v = j < pc ? T(0) : lrow[(j - pc) * Zc + z];
            hd[j * kCS + tz] = (int8_t)(v < T(0));   // LLR > 0 -> 0, < 0 -> 1, 0 stays 0 (:41-43)
        }
    if (valid && z == 0) anyS[cl] = 0, mx[cl] = -(1 << 30);
    bool active = valid;
    __syncthreads();
    int it = 0;
    for (; it < L; ++it) {
        // ---- S = H ck mod 2 (:47)
        bool any = false;
        if (active)
            sfor<0, MB>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                int par = 0;
                sfor<P::RS[i], P::RS[i + 1]>([&](auto ec) {
                    constexpr int e = decltype(ec)::value;
                    par ^= hd[P::COL[e] * kCS + rotp(shift_of<BG>(zi, e))];
                });
                S[i * kCS + tz] = (int8_t)par;
                any |= par != 0;
            });
        if (active && any) anyS[cl] = 1;
        __syncthreads();
        if (active && anyS[cl] == 0) {   // (:54-56)
            for (int j = 0; j < NB; ++j) crow[j * Zc + z] = hd[j * kCS + tz];
            if (z == 0) status[cb] = 1, iters[cb] = it;
            active = false;
        }
        // ---- En = (2S - 1) H per column; flip all bits at the maximum (:61-70).  The column sums
        //      are formed twice (for the maximum, then for the flips) rather than kept in a
        //      per-thread array of NB ints, which lived in scratch
        auto en_of = [&](auto jc) -> int {
            constexpr int j = decltype(jc)::value;
            int acc = 0;
            sfor<kCols<BG>.start[j], kCols<BG>.start[j + 1]>([&](auto xc) {
                constexpr int x = decltype(xc)::value;
                constexpr int i = kCols<BG>.row[x], e = kCols<BG>.edge[x];
                // row i*Zc+m connects column j*Zc+(m+V)%Zc, so column z meets row m=(z-V)%Zc
                acc += 2 * S[i * kCS + rotm(shift_of<BG>(zi, e))] - 1;
            });
            return acc;
        };
        int m = -(1 << 30);
        if (active) sfor<0, NB>([&](auto jc) { const int v = en_of(jc); m = v > m ? v : m; });
        if (active) atomicMax(&mx[cl], m);
        __syncthreads();
        if (active) {
            const int M = mx[cl];
            sfor<0, NB>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if (en_of(jc) == M) hd[j * kCS + tz] ^= 1;
            });
        }
        __syncthreads();
        if (valid && z == 0) anyS[cl] = 0, mx[cl] = -(1 << 30);
        if (!__syncthreads_or(active)) break;
    }
    if (active) {   // iterations exhausted: (ck, False) (:72-73)
        for (int j = 0; j < NB; ++j) crow[j * Zc + z] = hd[j * kCS + tz];
        if (z == 0) status[cb] = 0, iters[cb] = L;
    }
}

// ------------------------------------------------------------------------------------- BP
// Float64 sum-product flooding (nr_ldpc_decode.py:51-143, _BP_process :145-176).  Per-edge
// messages do not compress, so they live in the caller's scratch (layout below); LQ_old and the
// row-ascending sums Lr.sum(axis=0) of the core columns live in LDS (2 x 80 KB at Zc = 384, one
// workgroup per CU).  Every slot (z, codeblock) has TWO lanes, adjacent in the wave: the even and
// the odd edges of every row.  Rows run in order (a runtime loop; the row body is unrolled over
// the lane's <= 10 edges, tanh / atanh inlined once per edge slot); a barrier only where a new
// group of column-disjoint rows starts (BG1: 32 per iteration), so the LDS sums keep the
// reference's row order; the lane pair combines its partial products, zero counts and syndrome
// parity with one DPP lane swap (no LDS).  The next row's messages are loaded before the current
// row's arithmetic.  r05: 19.8 -> 10.7 ms per 1024 BG1 Zc=384 codeblocks (L=8).
constexpr int kBpThreads = 768;   // two lanes per slot (even / odd edges of every row)
// scheduling barrier every LDPC5G_BP_SB edges of a row (0: none): it bounds the registers the
// interleaved tanh / atanh chains of neighbouring edges take (r05: 1 / 2 / 0 measured 8.60 / 8.60
// / 8.65 ms per 1024 BG1 Zc=384 codeblocks)
#ifndef LDPC5G_BP_SB
#define LDPC5G_BP_SB 1
#endif
constexpr int kBpSb = LDPC5G_BP_SB;
__device__ __forceinline__ void bp_sched_point(int kk) {
    if (kBpSb > 0 && kk % (kBpSb > 0 ? kBpSb : 1) == (kBpSb > 0 ? kBpSb : 1) - 1) __builtin_amdgcn_sched_barrier(0);
}
constexpr double kBpClip = 2.0 * 19.07;   // (:159,161)
constexpr int kBpMaxDeg = 19;

template <int BG>
constexpr int bp_max_deg() {
    int m = 0;
    for (int i = 0; i < BGT<BG>::MB; ++i) m = m > BGT<BG>::RS[i + 1] - BGT<BG>::RS[i] ? m : BGT<BG>::RS[i + 1] - BGT<BG>::RS[i];
    return m;
}
static_assert(bp_max_deg<1>() <= kBpMaxDeg && bp_max_deg<2>() <= kBpMaxDeg, "BP row degree");

// degrees that occur in base graph BG (the row body is instantiated for each)
template <int BG>
constexpr bool bp_has_deg(int d) {
    for (int i = 0; i < BGT<BG>::MB; ++i)
        if (BGT<BG>::RS[i + 1] - BGT<BG>::RS[i] == d) return true;
    return false;
}

// ---- float64 tanh(q/2) and 2*atanh(y) for the BP kernel.  The reference uses numpy's np.tanh /
// np.arctanh, whose own results differ by 1-3 ulp between hosts (SVML vs glibc), so the
// BP bar is a stated tolerance; these are accurate to a few ulp and cheap: polynomial coefficients
// are f64 values in SGPR pairs made opaque at the start of each pass (otherwise the compiler hoists
// every coefficient of both functions out of the iteration loop into VGPRs and spills them inside
// the Horner chains).
// LDPC5G_BP_FASTDIV: the two divisions with bounded operands (tanh's e / (e + 2), e + 2 in [2, 2.4e17],
// and log's f / (2 + f), 2 + f in [1.4, 2.5]) by v_rcp_f64 + two Newton steps + one residual
// correction (<= 1 ulp, not correctly rounded: inside §2's stated BP tolerance) instead of the
// IEEE sequence (div_scale x 2, rcp, 4 fma, mul, div_fmas, div_fixup); and 2 atanh(P / t) as
// log1p(2|P| / (|t| - |P|)) — one division where y = P / t and u = 2|y| / (1 - |y|) took two
#ifndef LDPC5G_BP_FASTDIV
#define LDPC5G_BP_FASTDIV 1
#endif
__device__ __forceinline__ double bp_div_bounded(double a, double b) {
    if constexpr (!LDPC5G_BP_FASTDIV) return a / b;
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
}
__device__ __forceinline__ double sk(double c) {
    asm volatile("" : "+s"(c));
    return c;
}
struct BpTanhK {   // expm1 on [0, 40]: x = k ln2 + r, |r| <= ln2/2, Taylor to r^13
    double c[12];   // 1/n!, n = 2..13
    double inv_ln2, ln2_hi, ln2_lo, xmax;
    __device__ __forceinline__ void load() {
        const double f[12] = {0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333,
                              0.001388888888888889, 0.0001984126984126984, 2.48015873015873e-05,
                              2.7557319223985893e-06, 2.755731922398589e-07, 2.505210838544172e-08,
                              2.08767569878681e-09, 1.6059043836821613e-10};
#pragma unroll
        for (int n = 0; n < 12; ++n) c[n] = sk(f[n]);
        inv_ln2 = sk(1.4426950408889634), ln2_hi = sk(0.6931471787393093), ln2_lo = sk(1.8206359985041462e-09);
        xmax = sk(40.0);
    }
};
// tanh(q/2) = expm1(|q|) / (expm1(|q|) + 2) with q's sign; |q| clamped at 40 (tanh(20) rounds to 1)
__device__ __forceinline__ double bp_tanh_half(double q, const BpTanhK& K) {
    const double x = fmin(fabs(q), K.xmax);
    const double k = __builtin_rint(x * K.inv_ln2);
    double r = fma(-k, K.ln2_hi, x);
    r = fma(-k, K.ln2_lo, r);
    double h = K.c[11];
#pragma unroll
    for (int n = 10; n >= 0; --n) h = fma(h, r, K.c[n]);
    const double p = fma(r * r, h, r);   // expm1(r)
    const int ki = (int)k;
    const double e = __builtin_amdgcn_ldexp(p, ki) + (__builtin_amdgcn_ldexp(1.0, ki) - 1.0);   // expm1(x)
    return copysign(bp_div_bounded(e, e + 2.0), q);
}
struct BpAtanhK {   // log1p(u) = log(w) + c: w = m 2^e, m in [sqrt 1/2, sqrt 2), s = f/(2+f)
    double c[10];   // 2/(2n+1), n = 1..10
    double sqrt_half, ln2_hi, ln2_lo;
    __device__ __forceinline__ void load() {
#pragma unroll
        for (int n = 0; n < 10; ++n) c[n] = sk(2.0 / (2 * n + 3));
        sqrt_half = sk(0.7071067811865476), ln2_hi = sk(0.6931471787393093), ln2_lo = sk(1.8206359985041462e-09);
    }
};
// log1p(u), u >= 0
__device__ __forceinline__ double bp_log1p(double u, const BpAtanhK& K) {
    const double w = 1.0 + u;
    const double cw = (u - (w - 1.0)) * __builtin_amdgcn_rcp(w);   // rounding of 1 + u (tiny)
    double m = __builtin_amdgcn_frexp_mant(w);
    int ex = __builtin_amdgcn_frexp_exp(w);
    const bool lo = m < K.sqrt_half;
    m = lo ? 2.0 * m : m;
    ex = lo ? ex - 1 : ex;
    const double f = m - 1.0;
    const double s = bp_div_bounded(f, 2.0 + f);
    const double s2 = s * s;
    double h = K.c[9];
#pragma unroll
    for (int n = 8; n >= 0; --n) h = fma(h, s2, K.c[n]);
    const double lf = fma(s * s2, h, 2.0 * s);   // log(m) = 2 atanh(s)
    const double de = (double)ex;
    return fma(de, K.ln2_hi, lf + fma(de, K.ln2_lo, cw));
}
// 2 atanh(y) = log1p(2|y| / (1 - |y|)) with y's sign, |y| < 1
__device__ __forceinline__ double bp_two_atanh(double y, const BpAtanhK& K) {
    const double a = fabs(y);
    return copysign(bp_log1p((2.0 * a) / (1.0 - a), K), y);
}
// the message 2 atanh(P / t) of an edge (P: the row's tanh product, t: the edge's own), clipped to
// +-2 * 19.07 where |P / t| >= 1 (:157-162)
__device__ __forceinline__ double bp_msg(double P, double t, const BpAtanhK& K) {
    if constexpr (!LDPC5G_BP_FASTDIV) {
        const double tmp2 = P / t;
        return tmp2 >= 1.0 ? kBpClip : (tmp2 <= -1.0 ? -kBpClip : bp_two_atanh(tmp2, K));
    }
    const double aP = fabs(P), at = fabs(t);
    const uint32_t neg = (uint32_t)(__double2hiint(P) ^ __double2hiint(t)) & 0x80000000u;
    const double mag = aP >= at ? kBpClip : bp_log1p((2.0 * aP) / (at - aP), K);
    return __hiloint2double(__double2hiint(mag) ^ (int)neg, __double2loint(mag));
}

// Consecutive base rows with disjoint core columns (the grouping of ldpc5g_dec_body.h RowGroups):
// their sums into a column never meet, so a group needs no barrier inside it.
template <int BG>
struct BpGroups {
    int n = 0;
    int start[64] = {};
    constexpr BpGroups() {
        using P = BGT<BG>;
        int g0 = 0;
        n = 1;
        for (int i = 1; i < P::MB; ++i) {
            bool dis = true;
            for (int a = g0; a < i && dis; ++a)
                for (int e = P::RS[a]; e < P::RS[a + 1]; ++e)
                    for (int f = P::RS[i]; f < P::RS[i + 1]; ++f)
                        if (P::COL[e] == P::COL[f] && P::COL[e] < P::KC) dis = false;
            if (!dis) start[n++] = i, g0 = i;
        }
        start[n] = P::MB;
    }
};
template <int BG>
constexpr BpGroups<BG> kBpGroups{};

// Message scratch layout: the edges of row i are taken in pairs (k = 2kk, 2kk + 1; a row of odd
// degree pads its last pair), pair slot P(i, kk) = PS[i] + kk, and a pair's two messages of slot z
// are adjacent: msg[cb][P][z][2] -- the two lanes of a slot (even / odd edges) touch consecutive
// 8-B words, so a wave's message loads and stores are 512 contiguous bytes.
// Every field is 32-bit and read at a wave-uniform index, so the row loop's table reads are scalar
// loads (the generic int8 / int16 base-graph tables compile to vector loads there, and their
// s_waitcnt vmcnt(0) would also wait for the message prefetch in flight).
template <int BG>
struct BpPairs {
    int ps[64] = {};      // first pair slot of row i
    int np = 0;           // pair slots per codeblock
    int first[64] = {};   // row i starts a group of column-disjoint rows (RowGroups)
    int rs[64] = {};      // first edge of row i
    int col[BGT<BG>::E] = {};   // column of edge e
    constexpr BpPairs() {
        using P = BGT<BG>;
        for (int i = 0; i < P::MB; ++i) ps[i] = np, np += (P::RS[i + 1] - P::RS[i] + 1) / 2;
        for (int g = 0; g < kBpGroups<BG>.n; ++g) first[kBpGroups<BG>.start[g]] = 1;
        for (int i = 0; i <= P::MB; ++i) rs[i] = P::RS[i];
        for (int e = 0; e < P::E; ++e) col[e] = P::COL[e];
    }
};
template <int BG>
constexpr BpPairs<BG> kBpPairs{};
__constant__ BpPairs<1> kBpPairsD1 = kBpPairs<1>;   // device copies (runtime row index)
__constant__ BpPairs<2> kBpPairsD2 = kBpPairs<2>;
template <int BG>
__device__ __forceinline__ const BpPairs<BG>& bp_pairs_d() {
    if constexpr (BG == 1) return kBpPairsD1;
    else return kBpPairsD2;
}

// the pair partner's value (lanes 2s <-> 2s+1): DPP quad_perm [1,0,3,2], no LDS
__device__ __forceinline__ uint32_t pair_swap(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ double pair_swap(double x) {
    const uint32_t lo = pair_swap((uint32_t)__double2loint(x)), hi = pair_swap((uint32_t)__double2hiint(x));
    return __hiloint2double((int)hi, (int)lo);
}

template <int BG>
__global__ __launch_bounds__(kBpThreads) void ldpc_bp_kernel(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, double* __restrict__ msg, int B, int Zc, int zi, int G,
    int64_t ldl, int64_t ldc, int L, int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, DM = bp_max_deg<BG>(), KK = (DM + 1) / 2;
    constexpr int NPAIR = kBpPairs<BG>.np;
    extern __shared__ __align__(16) unsigned char smem[];
    double* app = (double*)smem;              // [KC][kCS] LQ of the core columns (LQ_old in a pass)
    double* acc = app + KC * kCS;             // [KC][kCS] Lr.sum(axis=0), rows ascending
    int* flag = (int*)(acc + KC * kCS);       // [kCS] per codeblock slot
    const int t = threadIdx.x;
    const int par_lane = t & 1;               // edges k = 2kk + par_lane of every row
    const int s = t >> 1;                     // slot (CB-major: cl * Zc + z)
    const int cbl = s / Zc, z = s - cbl * Zc;
    const int cb = blockIdx.x * G + cbl;
    const bool valid = cbl < G && cb < B && s < kCS;
    const int cl = valid ? cbl : 0;
    const int zv = valid ? z : 0;
    const int tz = cl * Zc + zv;
    const double* lrow = llr + (int64_t)(valid ? cb : 0) * ldl;
    int8_t* crow = ck + (int64_t)(valid ? cb : 0) * ldc;
    double* mrow = msg + (int64_t)(valid ? cb : 0) * NPAIR * Zc * 2;   // [P][z][2]
    // The message accesses of the row loop: this workgroup's scratch from a uniform base (SGPRs,
    // opaque per row like the z index) plus 32-bit per-lane byte offsets, so each load / store is
    // one saddr access with one VALU add, not a 64-bit VALU address (sign extension + lshl_add_u64)
    const double* msg_wg = msg + (int64_t)blockIdx.x * G * NPAIR * Zc * 2;
    const uint32_t mlaneB = (uint32_t)((cl * NPAIR * Zc * 2 + par_lane) * 8);
    auto opaque_s = [&]() {
        uint64_t v = (uint64_t)(uintptr_t)msg_wg;
        asm volatile("" : "+s"(v));
        return (__attribute__((address_space(1))) unsigned char*)(uintptr_t)v;
    };
    // pair slot q, entry zo of this lane's codeblock
    auto msg_at = [&](__attribute__((address_space(1))) unsigned char* mb, int q, int zo)
        -> __attribute__((address_space(1))) double& {
        return *(__attribute__((address_space(1))) double*)(mb + (mlaneB + (uint32_t)(q * Zc + zo) * 16u));
    };
    // z / base pointers opaque per row or pass: otherwise LICM hoists the loop-invariant per-edge
    // addresses out of the iteration loop into registers (hundreds of scratch spills)
    auto opaque_z = [&]() {
        int zo = zv;
        asm volatile("" : "+v"(zo));
        return zo;
    };
    // returned as a global (address space 1) pointer: through a generic pointer the accesses are
    // flat_load / flat_store, which also count against lgkmcnt, so every LDS wait of the row
    // would wait for the next row's message prefetch as well
    auto opaque_p = [&](auto* p) {
        uint64_t v = (uint64_t)(uintptr_t)p;
        asm volatile("" : "+v"(v));
        using E = std::remove_pointer_t<decltype(p)>;
        return (__attribute__((address_space(1))) E*)(uintptr_t)v;
    };
    // own core column entries for the LQ update: columns j = 2jj + par_lane
    if (valid) {
        for (int j = par_lane; j < KC; j += 2) {
            app[j * kCS + tz] = j < pc ? 0.0 : lrow[(j - pc) * Zc + z];
            acc[j * kCS + tz] = 0.0;
        }
        for (int q = 0; q < NPAIR; ++q) mrow[(q * Zc + z) * 2 + par_lane] = 0.0;   // Lr = 0 (:101)
    }
    if (valid && z == 0 && par_lane == 0) flag[cl] = 0;
    bool active = valid;
    __syncthreads();

    double pf[KK];   // r_old of the next row's own edges, loaded ahead
    double pxl = 0.0;   // and the next row's extension-column LLR (rows >= 4)
    auto load_row = [&](int i, int zo, __attribute__((address_space(1))) unsigned char* mb,
                        const __attribute__((address_space(1))) double* lr) {
        const int d = bp_pairs_d<BG>().rs[i + 1] - bp_pairs_d<BG>().rs[i], q0 = bp_pairs_d<BG>().ps[i];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
            if (2 * kk < d) pf[kk] = msg_at(mb, q0 + kk, zo);
        if (i >= 4) pxl = lr[(KB + i - pc) * Zc + zo];
    };
    int it = 0;
    for (; it < L; ++it) {
        bool fail = false;
        uint64_t hdx = 0;   // ext decisions (LQ_old < 0) of the rows whose ext edge is this lane's
        if (active) {
            load_row(0, opaque_z(), opaque_s(), opaque_p(lrow));
            for (int i = 0; i < MB; ++i) {
                // next row group: the LDS sums ordered.  An LDS-only barrier: __syncthreads() would
                // also wait (vmcnt(0)) for the next row's message loads and this row's stores
                if (bp_pairs_d<BG>().first[i] && i > 0) lds_sync();
                const int e0 = bp_pairs_d<BG>().rs[i], d = bp_pairs_d<BG>().rs[i + 1] - e0;
                const int q0 = bp_pairs_d<BG>().ps[i];
                const int zo = opaque_z();
                const auto mb = opaque_s();
                const auto lr = opaque_p(lrow);
                auto rotz = [&](int sft) { int m = zo + sft; return cl * Zc + (m >= Zc ? m - Zc : m); };
                double tq[KK];
#pragma unroll
                for (int kk = 0; kk < KK; ++kk) tq[kk] = pf[kk];   // r_old
                const double xl = pxl;
                if (i + 1 < MB) load_row(i + 1, zo, mb, lr);
                bool par = false;
                int nz = 0, zk = 255;
                double prod = 1.0, pnz = 1.0;   // product of all own t / of those with q != 0
                int jcol[KK];
                {
                    BpTanhK TK;
                    TK.load();
#pragma unroll
                    for (int kk = 0; kk < KK; ++kk) {
                        const int k = 2 * kk + par_lane;
                        jcol[kk] = -1;
                        if (2 * kk < d) {   // wave-uniform: the pair's first edge exists
                            // both lanes' table entries by wave-uniform (scalar) loads, then a lane
                            // select: a lane-indexed lookup is a vector load whose s_waitcnt vmcnt(0)
                            // would also wait for the next row's message prefetch and this row's stores
                            const int ea = e0 + 2 * kk, eb = min(ea + 1, P::E - 1);
                            const int ja = bp_pairs_d<BG>().col[ea], jb = bp_pairs_d<BG>().col[eb];
                            const int sa = shift_of<BG>(zi, ea), sb = shift_of<BG>(zi, eb);
                            const int j = par_lane ? jb : ja;
                            const int sft = par_lane ? sb : sa;
                            if (k < d) {
                                const double rold = tq[kk];
                                double a;
                                if (j < KC) {
                                    a = app[j * kCS + rotz(sft)];
                                    jcol[kk] = j * kCS + rotz(sft);
                                } else {
                                    a = xl + rold;   // degree-1 column
                                    hdx |= (uint64_t)(a < 0.0) << (i - 4);
                                }
                                par ^= a < 0.0;
                                const double q = a - rold;   // Lq (:129-131)
                                const double tk = bp_tanh_half(q, TK);   // tanh(q/2) (:152, :165)
                                tq[kk] = tk;
                                prod *= tk;
                                if (q == 0.0) {
                                    zk = nz == 0 ? k : zk;
                                    ++nz;
                                } else {
                                    pnz *= tk;
                                }
                            }
                        }
                        bp_sched_point(kk);
                    }
                }
                // the pair's totals (np.prod order aside: even-edge x odd-edge partial products)
                par ^= (pair_swap((uint32_t)par) & 1u) != 0;
                fail |= par;
                const uint32_t nzw = (uint32_t)nz | ((uint32_t)zk << 8), onzw = pair_swap(nzw);
                const int nzt = nz + (int)(onzw & 0xff);
                const int zkt = min(zk, (int)(onzw >> 8));
                const double prodt = prod * pair_swap(prod);
                const double pnzt = pnz * pair_swap(pnz);
                {
                    BpAtanhK AK;
                    AK.load();
#pragma unroll
                    for (int kk = 0; kk < KK; ++kk) {
                        const int k = 2 * kk + par_lane;
                        if (2 * kk < d) {
                            double r = 0.0;
                            if (k < d) {
                                if (nzt == 0) {
                                    r = bp_msg(prodt, tq[kk], AK);
                                } else if (nzt == 1 && k == zkt) {
                                    r = pnzt;   // prod(t[0:zk]) * prod(t[zk+1:]) (:166-172)
                                }
                                // rows of a group: disjoint columns; ds_add_f64 (no return), not a
                                // read -> add -> write chain (r05: 8.98 -> 8.90 ms)
                                if (jcol[kk] >= 0)
                                    __hip_atomic_fetch_add(&acc[jcol[kk]], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                            msg_at(mb, q0 + kk, zo) = r;
                        }
                        bp_sched_point(kk);
                    }
                }
            }
            if (fail) flag[cl] = 1;
        }
        lds_sync();   // flags, last group's sums (LDS only; messages are per lane)
        const uint32_t hx0 = pair_swap((uint32_t)hdx), hx1 = pair_swap((uint32_t)(hdx >> 32));
        hdx |= ((uint64_t)hx1 << 32) | hx0;
        if (active && flag[cl] == 0) {   // syndrome of LQ at pass start was 0 (:107-114)
            const int zo = opaque_z();
            const auto cr = opaque_p(crow);
            for (int j = par_lane; j < KC; j += 2) cr[j * Zc + zo] = (int8_t)(app[j * kCS + cl * Zc + zo] < 0.0);
            for (int i = 4 + par_lane; i < MB; i += 2) cr[(KB + i) * Zc + zo] = (int8_t)((hdx >> (i - 4)) & 1u);
            if (z == 0 && par_lane == 0) status[cb] = 1, iters[cb] = it;
            active = false;
        }
        if (active) {   // LQ = LLRin + Lr.sum(axis=0) (:126) for the own entries; sums back to 0
            const int zo = opaque_z();
            const auto lr = opaque_p(lrow);
            for (int j = par_lane; j < KC; j += 2) {
                const int x = j * kCS + cl * Zc + zo;
                const double lf = j < pc ? 0.0 : lr[(j < pc ? 0 : j - pc) * Zc + zo];
                app[x] = lf + acc[x];
                acc[x] = 0.0;
            }
        }
        __syncthreads();
        if (valid && z == 0 && par_lane == 0) flag[cl] = 0;
        if (!__syncthreads_or(active)) break;
    }
    // ---- exhausted: ck = LQ <= 0, status = syndrome == 0 (:133-143)
    const int zo = opaque_z();
    const auto mr = opaque_p(mrow);
    const auto lr = opaque_p(lrow);
    const auto cr = opaque_p(crow);
    auto rotf = [&](int sft) { int m = zo + sft; return cl * Zc + (m >= Zc ? m - Zc : m); };
    if (active) {
        bool fail = false;
        for (int i = 0; i < MB; ++i) {
            const int e0 = row_start_d<BG>(i), d = row_start_d<BG>(i + 1) - e0, q0 = bp_pairs_d<BG>().ps[i];
            bool par = false;
            for (int k = par_lane; k < d; k += 2) {
                const int e = e0 + k, j = col_d<BG>(e);
                const double a = j < KC ? app[j * kCS + rotf(shift_of<BG>(zi, e))]
                                        : lr[(KB + i - pc) * Zc + zo] + mr[((q0 + k / 2) * Zc + zo) * 2 + par_lane];
                par ^= a <= 0.0;
                if (j >= KC) cr[(KB + i) * Zc + zo] = (int8_t)(a <= 0.0);   // the ext decision
            }
            par ^= (pair_swap((uint32_t)par) & 1u) != 0;
            fail |= par;
        }
        if (fail) flag[cl] = 1;
    }
    __syncthreads();
    if (active) {
        for (int j = par_lane; j < KC; j += 2) cr[j * Zc + zo] = (int8_t)(app[j * kCS + cl * Zc + zo] <= 0.0);
        if (z == 0 && par_lane == 0) status[cb] = flag[cl] == 0, iters[cb] = L;
    }
}

template <int BG, typename T>
int launch_bf_t(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
                int64_t ldl, int64_t ldc, int L, int pc, hipStream_t st) {
    using P = BGT<BG>;
    const int G = dec_G(Zc);
    const size_t lds = (size_t)(P::NB + P::MB) * kCS + 2 * kCS * sizeof(int);
    const int threads = ((G * Zc + 63) / 64) * 64;
    hipLaunchKernelGGL((ldpc_bf_kernel<BG, T>), dim3((B + G - 1) / G), dim3(threads), lds, st, llr,
                       ck, status, iters, B, Zc, zi, G, ldl, ldc, L, pc);
    return check_hip(hipGetLastError(), "ldpc_bf_kernel launch");
}

template <int BG>
int launch_bp_t(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, double* msg,
                int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L, int pc, hipStream_t st) {
    using P = BGT<BG>;
    auto kern = ldpc_bp_kernel<BG>;
    const int G = dec_G(Zc);
    // LQ image + row-ascending sums of the core columns, flags: one workgroup per CU
    const size_t lds = (size_t)2 * P::KC * kCS * sizeof(double) + kCS * sizeof(int);
    if (int rc = set_lds_once<ldpc_bp_kernel<BG>>(lds)) return rc;
    const int threads = ((2 * G * Zc + 63) / 64) * 64;
    hipLaunchKernelGGL(kern, dim3((B + G - 1) / G), dim3(threads), lds, st, llr, ck, status, iters,
                       msg, B, Zc, zi, G, ldl, ldc, L, pc);
    return check_hip(hipGetLastError(), "ldpc_bp_kernel launch");
}

}  // namespace

int launch_bf(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status, int32_t* iters,
              int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L, int pc, hipStream_t st) {
    if (dtype == LDPC5G_F64)
        return bgn == 1 ? launch_bf_t<1, double>((const double*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, pc, st)
                        : launch_bf_t<2, double>((const double*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, pc, st);
    return bgn == 1 ? launch_bf_t<1, float>((const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, pc, st)
                    : launch_bf_t<2, float>((const float*)llr, ck, status, iters, B, Zc, zi, ldl, ldc, L, pc, st);
}

int launch_bp(int bgn, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
              double* msg, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L, int pc,
              hipStream_t st) {
    return bgn == 1 ? launch_bp_t<1>(llr, ck, status, iters, msg, B, Zc, zi, ldl, ldc, L, pc, st)
                    : launch_bp_t<2>(llr, ck, status, iters, msg, B, Zc, zi, ldl, ldc, L, pc, st);
}

int edges_of_bg(int bgn) { return bgn == 1 ? BGT<1>::E : BGT<2>::E; }

int bp_scratch_per_zc(int bgn) { return 2 * (bgn == 1 ? kBpPairs<1>.np : kBpPairs<2>.np); }

}  // namespace ldpc5g_impl
