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
template <int BG>
__global__ __launch_bounds__(kBfThreads) void ldpc_bp_kernel(
    const double* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, double* __restrict__ msg, int B, int Zc, int zi, int G,
    int64_t ldl, int64_t ldc, int L, int pc) {
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, E = P::E;
    constexpr double kClip = 2.0 * 19.07;   // (:159,161)
    extern __shared__ __align__(16) unsigned char smem[];
    double* app = (double*)smem;              // [KC][kCS] LQ of the core columns
    double* acc = app + KC * kCS;             // [KC][kCS] sum of Lr, row-ascending
    int* flag = (int*)(acc + KC * kCS);       // [kCS]
    const int t = threadIdx.x;
    const int cbl = t / Zc, z = t - cbl * Zc;
    const int cb = blockIdx.x * G + cbl;
    const bool valid = cbl < G && cb < B;
    const int cl = valid ? cbl : 0;
    const int tz = cl * Zc + z;
    const double* lrow = llr + (int64_t)(valid ? cb : 0) * ldl;
    int8_t* crow = ck + (int64_t)(valid ? cb : 0) * ldc;
    double* mrow = msg + (int64_t)(valid ? cb : 0) * E * Zc;   // Lr[e][z]
    auto rot = [&](int s) { int m = z + s; return cl * Zc + (m >= Zc ? m - Zc : m); };
    auto llrx = [&](int i) { return lrow[(KB + i - pc) * Zc + z]; };   // ext column of row i

    if (valid) {
        for (int j = 0; j < KC; ++j) {
            app[j * kCS + tz] = j < pc ? 0.0 : lrow[(j - pc) * Zc + z];
            acc[j * kCS + tz] = 0.0;
        }
        for (int e = 0; e < E; ++e) mrow[e * Zc + z] = 0.0;   // Lr = 0 (:101)
    }
    if (valid && z == 0) flag[cl] = 0;
    bool active = valid;
    __syncthreads();
    int it = 0;
    for (; it < L; ++it) {
        bool fail = false;
        uint64_t hdx = 0;
        // rows in ascending order (a runtime loop over the base graph's device tables: the row and
        // edge indices are uniform, so their table reads are scalar loads, and tanh / atanh appear
        // once in the code instead of at each of the 316 edges of an unrolled graph)
        for (int i = 0; i < MB; ++i) {
            const int e0 = row_start_d<BG>(i), d = row_start_d<BG>(i + 1) - e0;
            if (active) {
                // pass 1: Lq = LQ - Lr (:129-131), tanh(Lq/2) (:152, :165) parked in the message
                // slot (the thread's own), the zero count, and the products the three cases need
                int nz = 0, zk = 0;
                bool par = false;
                double prod = 1.0, pb = 1.0, pa = 1.0;   // all; before / after the first zero
                for (int k = 0; k < d; ++k) {
                    const int e = e0 + k, j = col_d<BG>(e);
                    double* m = mrow + (int64_t)e * Zc + z;
                    const double rold = *m;
                    double a;
                    if (j < KC) {
                        a = app[j * kCS + rot(shift_of<BG>(zi, e))];
                    } else {
                        a = llrx(i) + rold;   // LQ of the degree-1 column
                        hdx |= (uint64_t)(a < 0.0) << (i - 4);
                    }
                    par ^= a < 0.0;
                    const double q = a - rold;
                    const double tq = tanh(q / 2);
                    *m = tq;
                    prod = k == 0 ? tq : prod * tq;   // np.prod: left to right
                    if (q == 0.0) {
                        if (nz == 0) zk = k;
                        ++nz;
                    } else if (nz == 0) {
                        pb = k == 0 ? tq : pb * tq;
                    } else {
                        pa = k == zk + 1 ? tq : pa * tq;
                    }
                }
                fail |= par;
                // pass 2 (:150-175): three cases on the number of zero Lq in the row
                const double pzero = pb * pa;   // prod(t[0:zk]) * prod(t[zk+1:])
                for (int k = 0; k < d; ++k) {
                    const int e = e0 + k, j = col_d<BG>(e);
                    double* m = mrow + (int64_t)e * Zc + z;
                    double r;
                    if (nz == 0) {
                        const double tmp2 = prod / *m;
                        r = tmp2 >= 1.0 ? kClip : (tmp2 <= -1.0 ? -kClip : 2.0 * atanh(tmp2));
                    } else if (nz == 1) {
                        r = (k == zk) ? pzero : 0.0;
                    } else {
                        r = 0.0;
                    }
                    *m = r;
                    if (j < KC) {
                        double& ac = acc[j * kCS + rot(shift_of<BG>(zi, e))];
                        ac = ac + r;   // row-ascending accumulation (:126)
                    }
                }
            }
            __syncthreads();
        }
        if (active && fail) flag[cl] = 1;
        __syncthreads();
        if (active && flag[cl] == 0) {   // syndrome of LQ at pass start was 0 (:107-114)
            for (int j = 0; j < KC; ++j) crow[j * Zc + z] = (int8_t)(app[j * kCS + tz] < 0.0);
            for (int i = 4; i < MB; ++i) crow[(KB + i) * Zc + z] = (int8_t)((hdx >> (i - 4)) & 1u);
            if (z == 0) status[cb] = 1, iters[cb] = it;
            active = false;
        } else if (active) {
            for (int j = 0; j < KC; ++j) {
                const double lf = j < pc ? 0.0 : lrow[(j - pc) * Zc + z];
                app[j * kCS + tz] = lf + acc[j * kCS + tz];   // LQ = LLR + sum Lr (:126)
                acc[j * kCS + tz] = 0.0;
            }
        }
        __syncthreads();
        if (valid && z == 0) flag[cl] = 0;
        if (!__syncthreads_or(active)) break;
    }
    // ---- exhausted: ck = LQ <= 0, status = syndrome == 0 (:133-143)
    if (active) {
        bool fail = false;
        for (int i = 0; i < MB; ++i) {
            const int e0 = row_start_d<BG>(i), e1 = row_start_d<BG>(i + 1);
            bool par = false;
            for (int e = e0; e < e1; ++e) {
                const int j = col_d<BG>(e);
                const double a = j < KC ? app[j * kCS + rot(shift_of<BG>(zi, e))]
                                        : llrx(i) + mrow[(int64_t)e * Zc + z];
                par ^= a <= 0.0;
            }
            fail |= par;
        }
        if (fail) flag[cl] = 1;
    }
    __syncthreads();
    if (active) {
        for (int j = 0; j < KC; ++j) crow[j * Zc + z] = (int8_t)(app[j * kCS + tz] <= 0.0);
        for (int i = 4; i < MB; ++i) {
            const int el = row_start_d<BG>(i + 1) - 1;   // the ext column is the row's last edge
            crow[(KB + i) * Zc + z] = (int8_t)(llrx(i) + mrow[(int64_t)el * Zc + z] <= 0.0);
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
    const size_t lds = (size_t)2 * P::KC * kCS * sizeof(double) + kCS * sizeof(int);
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
