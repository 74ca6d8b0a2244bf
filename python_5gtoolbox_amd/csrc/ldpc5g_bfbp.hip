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
// Two phases per iteration, as the min-sum flooding kernel, but per-edge messages (they do not
// compress) in the caller's scratch msg[cb][e][z] (coalesced over z):
//   phase A  every row (a runtime loop; the row body instantiated per degree, tanh / atanh inlined
//            once per edge slot of that degree) reads LQ_old (LDS) and r_old (scratch), forms
//            q = LQ_old - r_old, t = tanh(q/2) and writes r_new over r_old; the syndrome of LQ_old
//            comes from the same reads.  The next row's r_old loads are issued before the current
//            row's arithmetic, so their latency hides behind it.  No barrier between rows.
//   phase B  a column-owner gather: each core column entry sums the messages of its rows in
//            ascending row order (Lr.sum(axis=0), :126) straight from the scratch, into a register,
//            then writes LQ = LLR + sum over LQ_old in LDS.  No barrier between columns.
// One thread per slot (z, codeblock), 384-thread workgroups holding only the LQ image (80 KB), so
// two workgroups (two codeblocks of Zc = 384) share a CU and cover each other's barriers.
constexpr int kBpThreads = 384;
constexpr double kBpClip = 2.0 * 19.07;   // (:159,161)
constexpr int kBpMaxDeg = 19;
constexpr int kBpPrefetch = 10;   // r_old loads issued one row ahead (edges 0..9: every row but rows 0-3 of BG1)

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
    return copysign(e / (e + 2.0), q);
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
// 2 atanh(y) = log1p(2|y| / (1 - |y|)) with y's sign, |y| < 1
__device__ __forceinline__ double bp_two_atanh(double y, const BpAtanhK& K) {
    const double a = fabs(y);
    const double u = (2.0 * a) / (1.0 - a);
    const double w = 1.0 + u;
    const double cw = (u - (w - 1.0)) * __builtin_amdgcn_rcp(w);   // rounding of 1 + u (tiny)
    double m = __builtin_amdgcn_frexp_mant(w);
    int ex = __builtin_amdgcn_frexp_exp(w);
    const bool lo = m < K.sqrt_half;
    m = lo ? 2.0 * m : m;
    ex = lo ? ex - 1 : ex;
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double s2 = s * s;
    double h = K.c[9];
#pragma unroll
    for (int n = 8; n >= 0; --n) h = fma(h, s2, K.c[n]);
    const double lf = fma(s * s2, h, 2.0 * s);   // log(m) = 2 atanh(s)
    const double de = (double)ex;
    const double r = fma(de, K.ln2_hi, lf + fma(de, K.ln2_lo, cw));
    return copysign(r, y);
}

template <int BG>
__global__ __launch_bounds__(kBpThreads, 3) void ldpc_bp_kernel(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, double* __restrict__ msg, int B, int Zc, int zi, int G,
    int64_t ldl, int64_t ldc, int L, int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E, DM = bp_max_deg<BG>();
    extern __shared__ __align__(16) unsigned char smem[];
    double* app = (double*)smem;              // [KC][kCS] LQ of the core columns
    int* flag = (int*)(app + KC * kCS);       // [kCS] per codeblock slot
    const int t = threadIdx.x;
    const int cbl = t / Zc, z = t - cbl * Zc;
    const int cb = blockIdx.x * G + cbl;
    const bool valid = cbl < G && cb < B;
    const int cl = valid ? cbl : 0;
    const int tz = cl * Zc + z;
    const int zv = valid ? z : 0;
    const double* lrow = llr + (int64_t)(valid ? cb : 0) * ldl;
    int8_t* crow = ck + (int64_t)(valid ? cb : 0) * ldc;
    double* mrow = msg + (int64_t)(valid ? cb : 0) * E * Zc;   // Lr[e][z]
    auto rot = [&](int s) { int m = zv + s; return cl * Zc + (m >= Zc ? m - Zc : m); };   // (z+s) % Zc
    auto llrx = [&](int i) { return lrow[(KB + i - pc) * Zc + zv]; };   // ext column of row i

    if (valid) {
        for (int j = 0; j < KC; ++j) app[j * kCS + tz] = j < pc ? 0.0 : lrow[(j - pc) * Zc + z];
        for (int e = 0; e < E; ++e) mrow[e * Zc + z] = 0.0;   // Lr = 0 (:101)
    }
    if (valid && z == 0) flag[cl] = 0;
    bool active = valid;
    __syncthreads();

    // r_old of the next row's first PF edges, loaded ahead (the rest at the row: registers)
    constexpr int PF = DM < kBpPrefetch ? DM : kBpPrefetch;
    double pf[PF];
    // z made opaque per row / column pass: otherwise LICM hoists the hundreds of loop-invariant
    // per-edge addresses out of the iteration loop into registers (hundreds of scratch spills)
    auto opaque_z = [&]() {
        int zo = zv;
        asm volatile("" : "+v"(zo));
        return zo;
    };
    auto opaque_p = [&](auto* p) {   // the same for a row base pointer (no hoisted per-edge addresses)
        uint64_t v = (uint64_t)(uintptr_t)p;
        asm volatile("" : "+v"(v));
        return (decltype(p))(uintptr_t)v;
    };
    auto load_row = [&](int i, int zo, double* mr) {
        const int e0 = row_start_d<BG>(i), d = row_start_d<BG>(i + 1) - e0;
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if (k < d) pf[k] = mr[(e0 + k) * Zc + zo];
    };
    int it = 0;
    for (; it < L; ++it) {
        bool fail = false;
        uint64_t hdx = 0;
        // ---- phase A (:117-123, _BP_process :145-176)
        if (active) {
            load_row(0, opaque_z(), opaque_p(mrow));
            for (int i = 0; i < MB; ++i) {
                const int e0 = row_start_d<BG>(i), d = row_start_d<BG>(i + 1) - e0;
                const int zo = opaque_z();
                double* const mr = opaque_p(mrow);
                const double* const lr = opaque_p(lrow);
                auto rotz = [&](int s) { int m = zo + s; return cl * Zc + (m >= Zc ? m - Zc : m); };
                auto row = [&](auto dc) {
                    constexpr int D = decltype(dc)::value;
                    double tq[D];
                    bool par = false;
#pragma unroll
                    for (int k = 0; k < D; ++k) tq[k] = k < PF ? pf[k] : mr[(e0 + k) * Zc + zo];   // r_old
                    if (i + 1 < MB) load_row(i + 1, zo, mr);
                    int nz = 0, zk = 0;
                    double prod = 1.0, pb = 1.0, pa = 1.0;   // all; before / after the first zero
                    BpTanhK TK;
                    TK.load();
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        const int e = e0 + k, j = col_d<BG>(e);
                        const double rold = tq[k];
                        double a;
                        if (j < KC) {
                            a = app[j * kCS + rotz(shift_of<BG>(zi, e))];
                        } else {
                            a = lr[(KB + i - pc) * Zc + zo] + rold;   // LQ of the degree-1 column
                            hdx |= (uint64_t)(a < 0.0) << (i - 4);
                        }
                        par ^= a < 0.0;
                        const double q = a - rold;   // Lq (:129-131)
                        const double tk = bp_tanh_half(q, TK);   // tanh(q / 2) (:152, :165)
                        tq[k] = tk;
                        __builtin_amdgcn_sched_barrier(0);   // one edge's temporaries at a time
                        prod = k == 0 ? tk : prod * tk;   // np.prod: left to right
                        if (q == 0.0) {
                            if (nz == 0) zk = k;
                            ++nz;
                        } else if (nz == 0) {
                            pb = k == 0 ? tk : pb * tk;
                        } else {
                            pa = k == zk + 1 ? tk : pa * tk;
                        }
                    }
                    fail |= par;
                    const double pzero = pb * pa;   // prod(t[0:zk]) * prod(t[zk+1:])
                    BpAtanhK AK;
                    AK.load();
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        double r;
                        if (nz == 0) {
                            const double tmp2 = prod / tq[k];
                            r = tmp2 >= 1.0 ? kBpClip : (tmp2 <= -1.0 ? -kBpClip : bp_two_atanh(tmp2, AK));
                        } else {
                            r = (nz == 1 && k == zk) ? pzero : 0.0;
                        }
                        mr[(e0 + k) * Zc + zo] = r;
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                switch (d) {   // wave-uniform
#define LDPC5G_BP_DEG(D) \
    case D:              \
        if constexpr (bp_has_deg<BG>(D)) row(std::integral_constant<int, D>{}); \
        break;
                    LDPC5G_BP_DEG(3) LDPC5G_BP_DEG(4) LDPC5G_BP_DEG(5) LDPC5G_BP_DEG(6) LDPC5G_BP_DEG(7)
                    LDPC5G_BP_DEG(8) LDPC5G_BP_DEG(9) LDPC5G_BP_DEG(10) LDPC5G_BP_DEG(19)
#undef LDPC5G_BP_DEG
                    default: __builtin_trap();
                }
            }
            if (fail) flag[cl] = 1;
        }
        __syncthreads();   // messages (global) and flags: visible to the workgroup
        if (active && flag[cl] == 0) {   // syndrome of LQ at pass start was 0 (:107-114)
            const int zo = opaque_z();
            int8_t* const cr = opaque_p(crow);
            for (int j = 0; j < KC; ++j) cr[j * Zc + zo] = (int8_t)(app[j * kCS + cl * Zc + zo] < 0.0);
            for (int i = 4; i < MB; ++i) cr[(KB + i) * Zc + zo] = (int8_t)((hdx >> (i - 4)) & 1u);
            if (z == 0) status[cb] = 1, iters[cb] = it;
            active = false;
        }
        // ---- phase B: LQ = LLRin + Lr.sum(axis=0) (:126), column by column, rows ascending
        if (active)
            sfor<0, KC>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const int zo = opaque_z();
                const double* const mr = opaque_p(mrow);
                const double* const lr = opaque_p(lrow);
                auto rotmz = [&](int s) { int m = zo - s; return m < 0 ? m + Zc : m; };   // (z-s) % Zc
                constexpr int x0 = kCols<BG>.start[j], x1 = kCols<BG>.start[j + 1];
                double v[x1 - x0];
                sfor<x0, x1>([&](auto xc) {
                    constexpr int e = kCols<BG>.edge[decltype(xc)::value];
                    v[decltype(xc)::value - x0] = mr[e * Zc + rotmz(shift_of<BG>(zi, e))];
                });
                const double lf = j < pc ? 0.0 : lr[(j < pc ? 0 : j - pc) * Zc + zo];
                double acc = 0.0;
#pragma unroll
                for (int x = 0; x < x1 - x0; ++x) acc = acc + v[x];
                app[j * kCS + tz] = lf + acc;
                __builtin_amdgcn_sched_barrier(0);   // one column's loads in flight at a time
            });
        __syncthreads();
        if (valid && z == 0) flag[cl] = 0;
        if (!__syncthreads_or(active)) break;
    }
    // ---- exhausted: ck = LQ <= 0, status = syndrome == 0 (:133-143)
    const int zo = opaque_z();
    double* const mr = opaque_p(mrow);
    const double* const lr = opaque_p(lrow);
    int8_t* const cr = opaque_p(crow);
    auto rotf = [&](int s) { int m = zo + s; return cl * Zc + (m >= Zc ? m - Zc : m); };
    if (active) {
        bool fail = false;
        for (int i = 0; i < MB; ++i) {
            const int e0 = row_start_d<BG>(i), e1 = row_start_d<BG>(i + 1);
            bool par = false;
            for (int e = e0; e < e1; ++e) {
                const int j = col_d<BG>(e);
                const double a = j < KC ? app[j * kCS + rotf(shift_of<BG>(zi, e))]
                                        : lr[(KB + i - pc) * Zc + zo] + mr[e * Zc + zo];
                par ^= a <= 0.0;
            }
            fail |= par;
        }
        if (fail) flag[cl] = 1;
    }
    __syncthreads();
    if (active) {
        for (int j = 0; j < KC; ++j) cr[j * Zc + zo] = (int8_t)(app[j * kCS + cl * Zc + zo] <= 0.0);
        for (int i = 4; i < MB; ++i) {
            const int el = row_start_d<BG>(i + 1) - 1;   // the ext column is the row's last edge
            cr[(KB + i) * Zc + zo] = (int8_t)(lr[(KB + i - pc) * Zc + zo] + mr[el * Zc + zo] <= 0.0);
        }
        if (z == 0) status[cb] = flag[cl] == 0, iters[cb] = L;
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
    const size_t lds = (size_t)P::KC * kCS * sizeof(double) + kCS * sizeof(int);   // 2 workgroups / CU
    if (int rc = set_lds_once<ldpc_bp_kernel<BG>>(lds)) return rc;
    const int threads = ((G * Zc + 63) / 64) * 64;
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

}  // namespace ldpc5g_impl
