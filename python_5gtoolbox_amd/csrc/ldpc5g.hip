// ldpc5g.hip — MI355X (gfx950, CDNA4) 5G NR QC-LDPC encode / min-sum decode engine.
//
// Replaces the hot path of py5gphy/ldpc (reference xu753x/python_5gtoolbox):
//   encode  : nr_ldpc_encode.py:8-50 + _gen_ldpc_parity_bit :52-115
//   decode  : nr_ldpc_decode.py:11-49 (nr_decode_ldpc), :51-143 (decode_ldpc, flooding loop),
//             :178-227 (_min_sum_process: MS / NMS / OMS / mixed check-node update)
// Design notes: DESIGN.md §4.  No MFMA: this is integer / min-select / add work.
//
// Kernel map
//   ldpc_enc_kernel<BG>            one workgroup per codeblock; bits packed 32/word in LDS, every
//                                  Zc-cyclic shift is a funnel shift (v_alignbit) of a periodic
//                                  extension of the block column; HBM-bound.
//   ldpc_dec_kernel<BG,T,LAYERED>  one thread per check row z of every base row ("row-z lane"),
//                                  G = floor(384/Zc) codeblocks per workgroup; core-column APP in
//                                  LDS, compressed check-node state (two magnitudes + argmin +
//                                  sign bits) in VGPRs, fully unrolled over the base graph so the
//                                  structure is compile-time and only V mod Zc is loaded.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "ldpc5g_tables.h"
#include "ldpc5g.h"

#define LDPC5G_VERSION "ldpc5g 0.1.0 gfx950"

namespace {

// ------------------------------------------------------------------------------ base graphs
template <int BG>
struct BGT;
template <>
struct BGT<1> {
    static constexpr int MB = LDPC5G_BG1_ROWS;   // 46 base rows
    static constexpr int NB = LDPC5G_BG1_COLS;   // 68 base columns
    static constexpr int KB = 22;                // information columns
    static constexpr int KC = 26;                // core columns (degree > 1): info + 4 parity
    static constexpr int E = LDPC5G_BG1_EDGES;   // 316
    static constexpr const int16_t* RS = kBG1RowStart;
    static constexpr const int8_t* COL = kBG1Col;
};
template <>
struct BGT<2> {
    static constexpr int MB = LDPC5G_BG2_ROWS;   // 42
    static constexpr int NB = LDPC5G_BG2_COLS;   // 52
    static constexpr int KB = 10;
    static constexpr int KC = 14;
    static constexpr int E = LDPC5G_BG2_EDGES;   // 197
    static constexpr const int16_t* RS = kBG2RowStart;
    static constexpr const int8_t* COL = kBG2Col;
};

template <int BG>
constexpr int edge_of(int i, int j) {
    for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i + 1]; ++e)
        if (BGT<BG>::COL[e] == j) return e;
    return -1;
}

// V(i,j) mod Zc of edge e for lifting size index zi (tables packed 2 edges per 32-bit word so a
// wave-uniform read is a scalar load)
template <int BG>
__device__ __forceinline__ int shift_of(int zi, int e) {
    uint32_t w;
    if constexpr (BG == 1) w = kBG1ShiftMod[zi][e >> 1];
    else w = kBG2ShiftMod[zi][e >> 1];
    return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
}
template <int BG>
__device__ __forceinline__ int row_start_d(int i) {
    if constexpr (BG == 1) return kBG1RowStartD[i];
    else return kBG2RowStartD[i];
}
template <int BG>
__device__ __forceinline__ int col_d(int e) {
    if constexpr (BG == 1) return kBG1ColD[e];
    else return kBG2ColD[e];
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int I, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, E>(f);
    }
}

// ================================================================================== ENCODER
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}

// 32 bits starting at bit `bit` of a packed LSB-first vector (needs one word of padding).
__device__ __forceinline__ uint32_t window32(const uint32_t* v, int bit) {
    return funnel(v[(bit >> 5) + 1], v[bit >> 5], (uint32_t)bit);
}

// bit b of the result = block[(start + b) mod Zc], where block is the Zc-bit vector at bit
// offset `base` of v.  (P_s x)[m] = x[(m+s) mod Zc] is one shifted identity block of H
// (ldpc_info.py:124-137), so this is a 32-row slice of a block product.
__device__ uint32_t fetch_rot32(const uint32_t* v, int base, int Zc, int start) {
    uint32_t out = 0;
    int b = 0, pos = start;
    while (b < 32) {
        int n = min(32 - b, Zc - pos);
        uint32_t w = window32(v, base + pos);
        if (n < 32) w &= (1u << n) - 1u;
        out |= w << b;
        b += n;
        pos += n;
        if (pos >= Zc) pos = 0;
    }
    return out;
}

__device__ __forceinline__ int mod_zc(int x, int Zc) {   // x in [0, 3*Zc + 64)
    while (x >= Zc) x -= Zc;
    return x;
}

// OR the low n (<=32) bits of val into the packed vector at bit offset `bit`.
__device__ __forceinline__ void or_bits(uint32_t* v, int bit, uint32_t val, int n) {
    if (n < 32) val &= (1u << n) - 1u;
    if (!val) return;
    int w = bit >> 5, s = bit & 31;
    atomicOr(&v[w], val << s);
    if (s) {
        uint32_t hi = val >> (32 - s);
        if (hi) atomicOr(&v[w + 1], hi);
    }
}

struct EncLayout {
    int K, N, W, DW, KW, PBW, words;
};
template <int BG>
__host__ __device__ inline EncLayout enc_layout(int Zc) {
    using P = BGT<BG>;
    EncLayout L;
    L.K = P::KB * Zc;
    L.N = (P::NB - 2) * Zc;
    L.W = (Zc + 31) >> 5;
    L.DW = 2 * L.W + 2;
    L.KW = (L.K + 31) >> 5;
    L.PBW = ((P::MB * Zc + 31) >> 5) + 2;
    // ib[KW+2] | X[KC*DW] | lam[4W] | pv[5W] | PB[PBW] | raw bytes (K, rounded to 16)
    L.words = (L.KW + 2) + P::KC * L.DW + 4 * L.W + 5 * L.W + L.PBW;
    L.words = (L.words + 3) & ~3;
    return L;
}
template <int BG>
inline size_t enc_lds_bytes(int Zc) {
    EncLayout L = enc_layout<BG>(Zc);
    return (size_t)L.words * 4 + (((size_t)L.K + 15) & ~(size_t)15);
}

__device__ __forceinline__ uint32_t expand4(uint32_t b4) {   // 4 bits -> 4 bytes of 0/1
    return (b4 * 0x00204081u) & 0x01010101u;
}

template <int BG>
__global__ __launch_bounds__(256) void ldpc_enc_kernel(const int8_t* __restrict__ ck,
                                                       int8_t* __restrict__ dn, int B, int Zc,
                                                       int zi, int64_t ldk, int64_t ldn) {
    using P = BGT<BG>;
    const int b = blockIdx.x;
    if (b >= B) return;
    const int t = threadIdx.x;
    const int NT = blockDim.x;
    const EncLayout Ly = enc_layout<BG>(Zc);
    const int K = Ly.K, N = Ly.N, W = Ly.W, DW = Ly.DW, KW = Ly.KW;
    const int S = K - 2 * Zc;   // systematic bytes in dn
    extern __shared__ __align__(16) uint32_t sm[];
    uint32_t* ib = sm;
    uint32_t* X = ib + KW + 2;
    uint32_t* lam = X + P::KC * DW;
    uint32_t* pv = lam + 4 * W;   // p1 p2 p3 p4 L2
    uint32_t* PB = pv + 5 * W;
    int8_t* raw = (int8_t*)(sm + Ly.words);
    // ---- 1. load info bytes, keep them raw in LDS, pack parity bits (fillers -> 0)
    const int8_t* src = ck + (int64_t)b * ldk;
    const bool al16 = (((uintptr_t)src) & 15) == 0;
    const int twoZ = 2 * Zc;
    for (int wi = t; wi < KW; wi += NT) {
        const int base = wi * 32;
        uint32_t bits = 0;
        if (al16 && base + 32 <= K) {
            int4 v[2];
            v[0] = *(const int4*)(src + base);
            v[1] = *(const int4*)(src + base + 16);
            *(int4*)(raw + base) = v[0];
            *(int4*)(raw + base + 16) = v[1];
            const uint32_t* d = (const uint32_t*)v;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
#pragma unroll
                for (int y = 0; y < 4; ++y) {
                    uint32_t by = (d[q] >> (8 * y)) & 0xffu;
                    int pos = base + 4 * q + y;
                    uint32_t bit = (by & 1u) & ~((uint32_t)(pos >= twoZ && by == 0xffu));
                    bits |= bit << (4 * q + y);
                }
            }
        } else {
            for (int y = 0; y < 32; ++y) {
                int pos = base + y;
                if (pos < K) {
                    uint32_t by = (uint8_t)src[pos];
                    raw[pos] = (int8_t)by;
                    uint32_t bit = (by & 1u) & ~((uint32_t)(pos >= twoZ && by == 0xffu));
                    bits |= bit << y;
                }
            }
        }
        ib[wi] = bits;
    }
    if (t < 2) ib[KW + t] = 0;
    for (int w = t; w < Ly.PBW; w += NT) PB[w] = 0;
    __syncthreads();

    // ---- 2. periodic extensions X_j[t] = block_j[t mod Zc] of the information columns
    for (int task = t; task < P::KB * DW; task += NT) {
        int j = task / DW, q = task - j * DW;
        X[j * DW + q] = fetch_rot32(ib, j * Zc, Zc, mod_zc(32 * q, Zc));
    }
    __syncthreads();

    // ---- 3. lambda_i = A_i c for the 4 core rows (nr_ldpc_encode.py:92-94)
    for (int task = t; task < 4 * W; task += NT) {
        int i = task / W, w = task - i * W;
        uint32_t acc = 0;
        for (int e = row_start_d<BG>(i); e < row_start_d<BG>(i + 1); ++e) {
            int j = col_d<BG>(e);
            if (j < P::KB) acc ^= window32(X + j * DW, 32 * w + shift_of<BG>(zi, e));
        }
        lam[i * W + w] = acc;
    }
    __syncthreads();

    // ---- 4. core parity by the double-diagonal recursion (BG1 :95-100, BG2 :101-106)
    constexpr int eS = (BG == 1) ? edge_of<BG>(1, 22) : edge_of<BG>(2, 10);
    constexpr int eA = edge_of<BG>(0, P::KB);
    constexpr int eC = edge_of<BG>(3, P::KB);
    constexpr int eD = (BG == 1) ? edge_of<BG>(2, 25) : edge_of<BG>(1, 11);
    static_assert(eS >= 0 && eA >= 0 && eC >= 0 && eD >= 0, "base graph core structure");
    uint32_t* p1 = pv;
    uint32_t* p2 = pv + W;
    uint32_t* p3 = pv + 2 * W;
    uint32_t* p4 = pv + 3 * W;
    uint32_t* L2 = pv + 4 * W;
    for (int w = t; w < W; w += NT) L2[w] = lam[w] ^ lam[W + w] ^ lam[2 * W + w] ^ lam[3 * W + w];
    // (window reads one word past a vector; those bits are masked, the word exists in LDS)
    __syncthreads();
    {
        const int s1 = shift_of<BG>(zi, eS);
        // p1 = roll(L2, s1): p1[z] = L2[(z - s1) mod Zc]
        for (int w = t; w < W; w += NT) p1[w] = fetch_rot32(L2, 0, Zc, mod_zc(mod_zc(32 * w, Zc) + Zc - s1, Zc));
    }
    __syncthreads();
    for (int w = t; w < W; w += NT) {
        p2[w] = lam[w] ^ fetch_rot32(p1, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eA), Zc));
        p4[w] = lam[3 * W + w] ^ fetch_rot32(p1, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eC), Zc));
    }
    __syncthreads();
    for (int w = t; w < W; w += NT) {
        if constexpr (BG == 1) p3[w] = lam[2 * W + w] ^ fetch_rot32(p4, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eD), Zc));
        else p3[w] = lam[1 * W + w] ^ fetch_rot32(p2, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eD), Zc));
    }
    __syncthreads();

    // ---- 5. extensions of the 4 core parity columns; core parity bits into PB
    for (int task = t; task < 4 * DW; task += NT) {
        int k = task / DW, q = task - k * DW;
        X[(P::KB + k) * DW + q] = fetch_rot32(pv + k * W, 0, Zc, mod_zc(32 * q, Zc));
    }
    for (int task = t; task < 4 * W; task += NT) {
        int k = task / W, w = task - k * W;
        or_bits(PB, k * Zc + 32 * w, pv[k * W + w], min(32, Zc - 32 * w));
    }
    __syncthreads();

    // ---- 6. extension parity rows 4..MB-1: pe = C [c; p] (nr_ldpc_encode.py:111-112)
    for (int task = t; task < (P::MB - 4) * W; task += NT) {
        int i = 4 + task / W, w = task % W;
        uint32_t acc = 0;
        for (int e = row_start_d<BG>(i); e < row_start_d<BG>(i + 1); ++e) {
            int j = col_d<BG>(e);
            if (j < P::KC) acc ^= window32(X + j * DW, 32 * w + shift_of<BG>(zi, e));
        }
        or_bits(PB, i * Zc + 32 * w, acc, min(32, Zc - 32 * w));
    }
    __syncthreads();

    // ---- 7. dn = [ck[2Zc:K], parity bits] as int8 (16 bytes per lane when aligned)
    int8_t* dst = dn + (int64_t)b * ldn;
    const bool dal16 = (((uintptr_t)dst) & 15) == 0;
    const bool raw4 = (twoZ & 3) == 0;
    const int nch = (N + 15) >> 4;
    for (int c = t; c < nch; c += NT) {
        const int q0 = c * 16;
        if (dal16 && q0 + 16 <= N) {
            uint32_t o[4];
            if (q0 >= S) {   // all parity
                uint32_t bits = window32(PB, q0 - S);
#pragma unroll
                for (int y = 0; y < 4; ++y) o[y] = expand4((bits >> (4 * y)) & 15u);
            } else if (q0 + 16 <= S && raw4) {   // all systematic
                const uint32_t* r = (const uint32_t*)(raw + twoZ + q0);
#pragma unroll
                for (int y = 0; y < 4; ++y) o[y] = r[y];
            } else {
#pragma unroll
                for (int y = 0; y < 4; ++y) {
                    uint32_t v = 0;
#pragma unroll
                    for (int x = 0; x < 4; ++x) {
                        int q = q0 + 4 * y + x;
                        uint32_t by = q < S ? (uint8_t)raw[twoZ + q] : ((PB[(q - S) >> 5] >> ((q - S) & 31)) & 1u);
                        v |= by << (8 * x);
                    }
                    o[y] = v;
                }
            }
            *(uint4*)(dst + q0) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            for (int q = q0; q < min(q0 + 16, N); ++q) {
                dst[q] = q < S ? raw[twoZ + q] : (int8_t)((PB[(q - S) >> 5] >> ((q - S) & 31)) & 1u);
            }
        }
    }
}

// Fast encoder: Zc % 16 == 0 and 16-B aligned rows (every BG1/BG2 Zc >= 16 that is a multiple
// of 16, including the Zc=384 hot path).  Same arithmetic as ldpc_enc_kernel; the differences are
// where bytes go: systematic bytes are stored straight from the load registers, every parity
// row-word (32 bits of one base row) is expanded and stored straight to dn as 32 (or 16) bytes,
// and the p1..p4 recursion runs inside wave 0 with wave-level syncs (no parity bit array, no LDS
// atomics, 4 workgroup barriers instead of 9).
struct EncFastLayout {
    int K, N, W, DW, KW, words;
};
template <int BG>
__host__ __device__ inline EncFastLayout enc_fast_layout(int Zc) {
    using P = BGT<BG>;
    EncFastLayout L;
    L.K = P::KB * Zc;
    L.N = (P::NB - 2) * Zc;
    L.W = (Zc + 31) >> 5;
    L.DW = 2 * L.W + 2;
    L.KW = (L.K + 31) >> 5;
    // ib[KW+2] | X[KC*DW] | lam[4W] | pv[5W + 2]
    L.words = (L.KW + 2) + P::KC * L.DW + 4 * L.W + 5 * L.W + 2;
    return L;
}
template <int BG>
inline size_t enc_fast_lds_bytes(int Zc) {
    return (size_t)enc_fast_layout<BG>(Zc).words * 4;
}

// 32 parity bits -> 32 int8 bytes (nbits = 32 or 16) at a 16-B aligned address
__device__ __forceinline__ void store_bits(int8_t* dst, uint32_t bits, int nbits) {
    uint4 a = make_uint4(expand4(bits & 15u), expand4((bits >> 4) & 15u), expand4((bits >> 8) & 15u),
                         expand4((bits >> 12) & 15u));
    *(uint4*)dst = a;
    if (nbits > 16) {
        uint4 b = make_uint4(expand4((bits >> 16) & 15u), expand4((bits >> 20) & 15u),
                             expand4((bits >> 24) & 15u), expand4(bits >> 28));
        *(uint4*)(dst + 16) = b;
    }
}

template <int BG>
__global__ __launch_bounds__(256) void ldpc_enc_fast_kernel(const int8_t* __restrict__ ck,
                                                            int8_t* __restrict__ dn, int B, int Zc,
                                                            int zi, int64_t ldk, int64_t ldn) {
    using P = BGT<BG>;
    const int b = blockIdx.x;
    if (b >= B) return;
    const int t = threadIdx.x;
    const int NT = blockDim.x;
    const EncFastLayout Ly = enc_fast_layout<BG>(Zc);
    const int K = Ly.K, W = Ly.W, DW = Ly.DW, KW = Ly.KW;
    const int twoZ = 2 * Zc;
    const int S = K - twoZ;
    extern __shared__ __align__(16) uint32_t sm[];
    uint32_t* ib = sm;
    uint32_t* X = ib + KW + 2;
    uint32_t* lam = X + P::KC * DW;
    uint32_t* pv = lam + 4 * W;   // p1 p2 p3 p4 L2
    const int8_t* src = ck + (int64_t)b * ldk;
    int8_t* dst = dn + (int64_t)b * ldn;

    // ---- 1. info bytes: pack parity bits; the systematic part is stored straight to dn
    for (int wi = t; wi < KW; wi += NT) {
        const int base = wi * 32;   // K = Kb*Zc is a multiple of 32 when Zc % 16 == 0
        uint32_t bits = 0;
        if (base + 32 <= K) {
            int4 v[2];
            v[0] = *(const int4*)(src + base);
            v[1] = *(const int4*)(src + base + 16);
            if (base >= twoZ) {   // 2Zc and K are multiples of 32 here
                *(int4*)(dst + base - twoZ) = v[0];
                *(int4*)(dst + base - twoZ + 16) = v[1];
            }
            const uint32_t* d = (const uint32_t*)v;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t x = d[q];
                // per byte: LSB, minus fillers (0xff) at positions >= 2Zc
                uint32_t lsb = x & 0x01010101u;
                const uint32_t ff = (x & (x >> 1) & (x >> 2) & (x >> 3) & (x >> 4) & (x >> 5) &
                                     (x >> 6) & (x >> 7)) & 0x01010101u;   // byte == 0xff
                if (base + 4 * q >= twoZ) lsb &= ~ff;
                bits |= ((lsb | (lsb >> 7) | (lsb >> 14) | (lsb >> 21)) & 15u) << (4 * q);
            }
        } else {   // (unreachable for Kb*Zc % 32 == 0; kept for safety)
            int4 v0 = *(const int4*)(src + base);
            if (base >= twoZ) *(int4*)(dst + base - twoZ) = v0;
            const uint32_t* d = (const uint32_t*)&v0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t x = d[q];
                uint32_t lsb = x & 0x01010101u;
                const uint32_t ff = (x & (x >> 1) & (x >> 2) & (x >> 3) & (x >> 4) & (x >> 5) &
                                     (x >> 6) & (x >> 7)) & 0x01010101u;
                if (base + 4 * q >= twoZ) lsb &= ~ff;
                bits |= ((lsb | (lsb >> 7) | (lsb >> 14) | (lsb >> 21)) & 15u) << (4 * q);
            }
        }
        ib[wi] = bits;
    }
    if (t < 2) ib[KW + t] = 0;
    __syncthreads();

    // ---- 2. periodic extensions of the information columns
    for (int task = t; task < P::KB * DW; task += NT) {
        int j = task / DW, q = task - j * DW;
        X[j * DW + q] = fetch_rot32(ib, j * Zc, Zc, mod_zc(32 * q, Zc));
    }
    __syncthreads();

    // ---- 3+4. lambda and the double-diagonal recursion, all inside wave 0
    constexpr int eS = (BG == 1) ? edge_of<BG>(1, 22) : edge_of<BG>(2, 10);
    constexpr int eA = edge_of<BG>(0, P::KB);
    constexpr int eC = edge_of<BG>(3, P::KB);
    constexpr int eD = (BG == 1) ? edge_of<BG>(2, 25) : edge_of<BG>(1, 11);
    uint32_t* p1 = pv;
    uint32_t* p2 = pv + W;
    uint32_t* p3 = pv + 2 * W;
    uint32_t* p4 = pv + 3 * W;
    uint32_t* L2 = pv + 4 * W;
    if (t < 64) {
        for (int task = t; task < 4 * W; task += 64) {
            int i = task / W, w = task - i * W;
            uint32_t acc = 0;
            for (int e = row_start_d<BG>(i); e < row_start_d<BG>(i + 1); ++e) {
                int j = col_d<BG>(e);
                if (j < P::KB) acc ^= window32(X + j * DW, 32 * w + shift_of<BG>(zi, e));
            }
            lam[i * W + w] = acc;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
        for (int w = t; w < W; w += 64) L2[w] = lam[w] ^ lam[W + w] ^ lam[2 * W + w] ^ lam[3 * W + w];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int s1 = shift_of<BG>(zi, eS);
        for (int w = t; w < W; w += 64)
            p1[w] = fetch_rot32(L2, 0, Zc, mod_zc(mod_zc(32 * w, Zc) + Zc - s1, Zc));
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        for (int w = t; w < W; w += 64) {
            p2[w] = lam[w] ^ fetch_rot32(p1, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eA), Zc));
            p4[w] = lam[3 * W + w] ^ fetch_rot32(p1, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eC), Zc));
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        for (int w = t; w < W; w += 64) {
            if constexpr (BG == 1) p3[w] = lam[2 * W + w] ^ fetch_rot32(p4, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eD), Zc));
            else p3[w] = lam[1 * W + w] ^ fetch_rot32(p2, 0, Zc, mod_zc(32 * w + shift_of<BG>(zi, eD), Zc));
        }
    }
    __syncthreads();

    // ---- 5. extensions of the 4 core parity columns; core parity bytes straight to dn
    for (int task = t; task < 4 * DW; task += NT) {
        int k = task / DW, q = task - k * DW;
        X[(P::KB + k) * DW + q] = fetch_rot32(pv + k * W, 0, Zc, mod_zc(32 * q, Zc));
    }
    for (int task = t; task < 4 * W; task += NT) {
        int k = task / W, w = task - k * W;
        store_bits(dst + S + k * Zc + 32 * w, pv[k * W + w], min(32, Zc - 32 * w));
    }
    __syncthreads();

    // ---- 6. extension parity rows, each row-word stored straight to dn
    for (int task = t; task < (P::MB - 4) * W; task += NT) {
        int i = 4 + task / W, w = task % W;
        uint32_t acc = 0;
        for (int e = row_start_d<BG>(i); e < row_start_d<BG>(i + 1); ++e) {
            int j = col_d<BG>(e);
            if (j < P::KC) acc ^= window32(X + j * DW, 32 * w + shift_of<BG>(zi, e));
        }
        store_bits(dst + S + i * Zc + 32 * w, acc, min(32, Zc - 32 * w));
    }
}

// ================================================================================== DECODER
template <typename T>
struct FT;
template <>
struct FT<float> {
    __device__ static __forceinline__ uint32_t sbits(float x) { return __float_as_uint(x); }
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
    __device__ static __forceinline__ double xsign(double x, uint32_t b) {
        return __longlong_as_double(__double_as_longlong(x) ^ ((long long)(b & 0x80000000u) << 32));
    }
    __device__ static __forceinline__ double inf() { return __longlong_as_double(0x7ff0000000000000ll); }
    __device__ static __forceinline__ double med3(double a, double b, double c) {
        return fmax(fmin(a, b), fmin(fmax(a, b), c));
    }
};

// Compressed check-node state of one row: r_k = (k == idx ? mB : mA), sign = bit k of pk.
// pk: bits 0..deg-1 = sign of r_k, bits 24..28 = idx (an edge holding min |q|).
template <typename T>
__device__ __forceinline__ T decomp(T mA, T mB, uint32_t pk, uint32_t idx, int k) {
    return FT<T>::xsign((idx == (uint32_t)k) ? mB : mA, pk << (31 - k));
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

struct DecWork {     // one workgroup of the mixed-Zc path
    int32_t zi, Zc, G, first;
};
struct CbRef {       // one codeblock of the mixed-Zc path
    int64_t llr_off, ck_off;
    int32_t out, pad;
};

constexpr int kDecThreads = 384;   // = max Zc: one thread per check row z of a base row
constexpr int kCS = kDecThreads;   // LDS column stride (entries): G*Zc <= 384 always

template <typename T, bool LAYERED>
constexpr size_t dec_lds_bytes_t(int MB, int KC) {
    return (size_t)KC * kCS * sizeof(T) * (LAYERED ? 1 : 2) +
           (sizeof(T) == 4 ? (size_t)(MB - 4) * kCS * sizeof(T) : 0) + 2 * kCS * sizeof(int);
}

template <int BG, typename T, bool LAYERED>
__global__ __launch_bounds__(kDecThreads) void ldpc_dec_kernel(
    const T* __restrict__ llr, int8_t* __restrict__ ck, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, int B, int Zc_u, int zi_u, int G_u, int64_t ldl, int64_t ldc,
    int L, T alpha, T beta, int pc, const DecWork* __restrict__ work,
    const CbRef* __restrict__ cbs) {
    // pc = number of leading punctured block columns absent from the LLR rows (2, or 0 when the
    // caller passes full-length rows as decode_ldpc(LLRin, H, ...) does, nr_ldpc_decode.py:51)
    using P = BGT<BG>;
    constexpr int MB = P::MB, KB = P::KB, KC = P::KC, TS = sizeof(T);
    constexpr bool XL_LDS = TS == 4;
    constexpr int ACC_B = KC * kCS * TS;                        // byte offsets in LDS
    constexpr int XL_B = KC * kCS * TS * (LAYERED ? 1 : 2);
    constexpr int FLAG_B = XL_B + (XL_LDS ? (MB - 4) * kCS * TS : 0);
    extern __shared__ __align__(16) unsigned char smem[];

    int Zc = Zc_u, zi = zi_u, G = G_u;
    const int t = threadIdx.x;
    if (work) {
        DecWork w = work[blockIdx.x];
        Zc = w.Zc, zi = w.zi, G = w.G;
    }
    const int cbl = t / Zc;
    const int z = t - cbl * Zc;
    bool valid = cbl < G;
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
            int cb = blockIdx.x * G + cbl;
            valid = cb < B;
            lrow = llr + (int64_t)cb * ldl;
            crow = ck + (int64_t)cb * ldc;
            out = cb;
        }
    }
    const int cl = valid ? cbl : 0;
    const int tzb = (cl * Zc + z) * TS;   // byte offset of this thread's own column entry
    const int ZcT = Zc * TS;
    int zv = z, ziv = zi;   // made opaque per iteration (see the iteration loop)
    int* flagA = (int*)(smem + FLAG_B);
    int* flagB = flagA + kCS;
    auto at = [&](int byte) -> T& { return *(T*)(smem + byte); };
    auto own = [&](int j) -> T& { return at(j * kCS * TS + tzb); };
    // channel LLR of the degree-1 extension column of row i = 4 + i4 (own column z)
    auto llrx = [&](int i4) -> T {
        if constexpr (XL_LDS) return at(XL_B + i4 * kCS * TS + tzb);
        else return lrow[(KB + 4 + i4 - pc) * Zc + zv];
    };

    // per-thread state of rows (i, z), i = 0..MB-1
    T sA[MB], sB[MB];
    uint32_t sP[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) sA[i] = T(0), sB[i] = T(0), sP[i] = 0u;

    uint32_t hdc_prev = 0;   // layered: hard decisions of own core columns, last iteration end
    uint64_t hdx_prev = 0;   // layered: ... of own extension columns
    if (valid) {
        for (int j = 0; j < KC; ++j) {
            const T v = j < pc ? T(0) : lrow[(j - pc) * Zc + z];   // punctured columns: LLR 0 (:43)
            own(j) = v;
            if (!LAYERED) at(ACC_B + j * kCS * TS + tzb) = T(0);
            hdc_prev |= (uint32_t)(v < T(0)) << j;
        }
        for (int i4 = 0; i4 < MB - 4; ++i4) {
            const T v = lrow[(KB + 4 + i4 - pc) * Zc + z];
            if constexpr (XL_LDS) at(XL_B + i4 * kCS * TS + tzb) = v;
            hdx_prev |= (uint64_t)(v < T(0)) << i4;
        }
    }
    if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
    bool active = valid;
    __syncthreads();

    // byte offset (without the column base) of column entry (z + s) mod Zc of this thread
    auto rot = [&](int s) -> int { return tzb + s * TS - (zv >= Zc - s ? ZcT : 0); };

    int it = 0;
    for (; it < L; ++it) {
        // zv / ziv are re-materialised opaque each iteration: otherwise LICM hoists the ~300
        // loop-invariant column addresses (z + V) mod Zc out of the loop into VGPRs/SGPRs.
        zv = z;
        ziv = zi;
        asm volatile("" : "+v"(zv));
        asm volatile("" : "+s"(ziv));
        bool fail = false;
        uint64_t hdx = 0;   // flooding: ext hard decisions at pass start; layered: at pass end
        // the next row group's packed shift words are loaded (scalar, wave-uniform) before the
        // barrier that precedes the group, so their latency hides behind it
        constexpr int NPW = max_group_nw<BG>();
        uint32_t nsw[NPW];
        auto prefetch = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            sfor<0, group_nw<BG>(g)>([&](auto wc) {
                constexpr int w = decltype(wc)::value;
                nsw[w] = shift_word<BG>(ziv, group_w0<BG>(g) + w);
            });
        };
        prefetch(std::integral_constant<int, 0>{});
        sfor<0, kGroups<BG>.n>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            uint32_t csw[NPW];
#pragma unroll
            for (int x = 0; x < NPW; ++x) csw[x] = nsw[x];
            auto gshift = [&](int e) -> int {   // e compile-time after unrolling
                const uint32_t w = csw[(e >> 1) - group_w0<BG>(g)];
                return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
            };
            if (active) {
                sfor<kGroups<BG>.start[g], kGroups<BG>.start[g + 1]>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    constexpr int e0 = P::RS[i];
                    constexpr int d = P::RS[i + 1] - e0;
                    const T mA = sA[i], mB = sB[i];
                    const uint32_t pk = sP[i];
                    const uint32_t idxo = pk >> 24;
                    T q[d];
                    int rb[d];
                    T min1 = FT<T>::inf(), min2 = FT<T>::inf();
                    uint32_t sx = 0, idx = 0, negs = 0;
                    bool par = false;
                    // ---- pass 1: variable-to-check messages q, two-min, sign product
                    sfor<0, d>([&](auto kc) {
                        constexpr int k = decltype(kc)::value;
                        constexpr int j = P::COL[e0 + k];
                        const T rold = decomp(mA, mB, pk, idxo, k);
                        T qq;
                        if constexpr (j < KC) {
                            rb[k] = rot(gshift(e0 + k));
                            const T a = at(j * kCS * TS + rb[k]);
                            qq = a - rold;
                            if constexpr (!LAYERED) par ^= a < T(0);
                        } else if constexpr (LAYERED) {
                            qq = llrx(i - 4);   // degree-1 column: q is the channel LLR itself
                        } else {
                            const T a = llrx(i - 4) + rold;   // LQ of a degree-1 column
                            qq = a - rold;
                            const bool h = a < T(0);
                            par ^= h;
                            hdx |= (uint64_t)h << (i - 4);
                        }
                        q[k] = qq;
                        const T aq = fabs(qq);
                        if constexpr (!LAYERED) {
                            idx = aq < min1 ? (uint32_t)k : idx;
                            negs |= (FT<T>::sbits(qq) >> 31) << k;
                        }
                        min2 = FT<T>::med3(min1, min2, aq);
                        min1 = fmin(min1, aq);
                        sx ^= FT<T>::sbits(qq);
                    });
                    fail |= par;
                    const T x1 = min1 - beta, x2 = min2 - beta;
                    const T nA = alpha * (x1 > T(0) ? x1 : T(0));   // (:201-202)
                    const T nB = alpha * (x2 > T(0) ? x2 : T(0));
                    // ---- pass 2: check-to-variable messages r = sign * (k == argmin ? nB : nA)
                    uint32_t signs = 0, idxn = 0;
                    sfor<0, d>([&](auto kc) {
                        constexpr int k = decltype(kc)::value;
                        constexpr int j = P::COL[e0 + k];
                        T r;
                        if constexpr (LAYERED) {
                            const T aq = fabs(q[k]);
                            const bool isMin = aq == min1;   // ties: nB == nA, either is right
                            idxn = isMin ? (uint32_t)k : idxn;
                            const uint32_t sb = FT<T>::sbits(q[k]) ^ sx;
                            r = FT<T>::xsign(isMin ? nB : nA, sb);
                            signs |= (sb >> 31) << k;
                            if constexpr (j < KC) {
                                at(j * kCS * TS + rb[k]) = q[k] + r;
                            } else {
                                hdx |= (uint64_t)(llrx(i - 4) + r < T(0)) << (i - 4);
                            }
                        } else {
                            const uint32_t sb = (negs >> k ^ sx >> 31) << 31;
                            r = FT<T>::xsign(idx == (uint32_t)k ? nB : nA, sb);
                            if constexpr (j < KC) {
                                T& a = at(ACC_B + j * kCS * TS + rb[k]);
                                a = a + r;   // row-ascending accumulation (:126)
                            }
                        }
                    });
                    sA[i] = nA;
                    sB[i] = nB;
                    if constexpr (LAYERED) sP[i] = signs | (idxn << 24);
                    else sP[i] = (negs ^ ((sx >> 31) ? ((1u << d) - 1u) : 0u)) | (idx << 24);
                });
            }
            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});
            __syncthreads();
        });

        if constexpr (!LAYERED) {
            // ---- reference order: the syndrome of LQ at the start of the pass decides (:107-114)
            if (active && fail) flagA[cl] = 1;
            __syncthreads();
            const bool conv = active && flagA[cl] == 0;
            if (conv) {
                for (int j = 0; j < KC; ++j) crow[j * Zc + zv] = (int8_t)(own(j) < T(0));
                for (int i4 = 0; i4 < MB - 4; ++i4)
                    crow[(KB + 4 + i4) * Zc + zv] = (int8_t)((hdx >> i4) & 1u);
                if (z == 0) status[out] = 1, iters[out] = it;
                active = false;
            } else if (active) {
                for (int j = 0; j < KC; ++j) {
                    T& acc = at(ACC_B + j * kCS * TS + tzb);
                    const T lf = j < pc ? T(0) : lrow[(j - pc) * Zc + zv];
                    own(j) = lf + acc;   // LQ = LLR + sum Lr (:126)
                    acc = T(0);
                }
            }
        } else {
            // ---- layered stopping rule: no hard decision changed over the iteration, then an
            //      exact syndrome check of those decisions (oracle.decode_layered)
            uint32_t hdc = 0;
            if (active)
                for (int j = 0; j < KC; ++j) hdc |= (uint32_t)(own(j) < T(0)) << j;
            if (active && (hdc != hdc_prev || hdx != hdx_prev)) flagA[cl] = 1;
            hdc_prev = hdc;
            hdx_prev = hdx;
            __syncthreads();
            const bool cand = active && flagA[cl] == 0;
            if (__syncthreads_or(cand)) {
                if (cand) {
                    bool sf = false;
                    sfor<0, MB>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        constexpr int e0 = P::RS[i];
                        constexpr int d = P::RS[i + 1] - e0;
                        bool par = false;
                        sfor<0, d>([&](auto kc) {
                            constexpr int k = decltype(kc)::value;
                            constexpr int j = P::COL[e0 + k];
                            if constexpr (j < KC)
                                par ^= at(j * kCS * TS + rot(shift_of<BG>(ziv, e0 + k))) < T(0);
                            else
                                par ^= (bool)((hdx >> (i - 4)) & 1u);
                        });
                        sf |= par;
                    });
                    if (sf) flagB[cl] = 1;
                }
                __syncthreads();
                if (cand && flagB[cl] == 0) {
                    for (int j = 0; j < KC; ++j) crow[j * Zc + zv] = (int8_t)((hdc >> j) & 1u);
                    for (int i4 = 0; i4 < MB - 4; ++i4)
                        crow[(KB + 4 + i4) * Zc + zv] = (int8_t)((hdx >> i4) & 1u);
                    if (z == 0) status[out] = 1, iters[out] = it + 1;
                    active = false;
                }
            }
        }
        __syncthreads();
        if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
        if (!__syncthreads_or(active)) break;
    }

    // ---- iterations exhausted: ck = (APP <= 0), status = syndrome == 0 (:133-143)
    zv = z;
    asm volatile("" : "+v"(zv));   // keep the output addresses out of the loop (no hoist/spill)
    if (active) {
        bool fail = false;
        sfor<0, MB>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int e0 = P::RS[i];
            constexpr int d = P::RS[i + 1] - e0;
            bool par = false;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                T a;
                if constexpr (j < KC) a = at(j * kCS * TS + rot(shift_of<BG>(zi, e0 + k)));
                else a = llrx(i - 4) + decomp(sA[i], sB[i], sP[i], sP[i] >> 24, k);
                par ^= (a <= T(0));
            });
            fail |= par;
        });
        if (fail) flagA[cl] = 1;
    }
    __syncthreads();
    if (active) {
        for (int j = 0; j < KC; ++j) crow[j * Zc + zv] = (int8_t)(own(j) <= T(0));
        sfor<4, MB>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int dl = P::RS[i + 1] - P::RS[i] - 1;   // ext column = last edge
            const T a = llrx(i - 4) + decomp(sA[i], sB[i], sP[i], sP[i] >> 24, dl);
            crow[(KB + i) * Zc + zv] = (int8_t)(a <= T(0));
        });
        if (z == 0) {
            status[out] = flagA[cl] == 0;
            iters[out] = L;
        }
    }
}

// ================================================================================== HOST
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int zc_index(int Zc) {
    for (int i = 0; i < LDPC5G_NUM_ZC; ++i)
        if (kLdpcZcList[i] == Zc) return i;
    return -1;
}

int check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(LDPC5G_EHIP, "%s: %s", what, hipGetErrorString(e));
    return LDPC5G_OK;
}

inline int dec_G(int Zc) { return Zc >= kDecThreads ? 1 : kDecThreads / Zc; }

template <int BG, typename T, bool LAYERED>
size_t dec_lds_bytes() {
    return dec_lds_bytes_t<T, LAYERED>(BGT<BG>::MB, BGT<BG>::KC);
}

template <int BG, typename T, bool LAYERED>
int launch_dec(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc, int zi,
               int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st) {
    auto kern = ldpc_dec_kernel<BG, T, LAYERED>;
    const int G = dec_G(Zc);
    const size_t lds = dec_lds_bytes<BG, T, LAYERED>();
    const int threads = ((G * Zc + 63) / 64) * 64;
    const int grid = (B + G - 1) / G;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, st, llr, ck, status, iters, B, Zc, zi,
                       G, ldl, ldc, L, (T)alpha, (T)beta, pc, (const DecWork*)nullptr,
                       (const CbRef*)nullptr);
    return check_hip(hipGetLastError(), "ldpc_dec_kernel launch");
}

template <int BG, typename T, bool LAYERED>
int launch_dec_mixed(const T* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                     const DecWork* work, const CbRef* cbs, int L, double alpha, double beta,
                     int pc, hipStream_t st) {
    auto kern = ldpc_dec_kernel<BG, T, LAYERED>;
    const size_t lds = dec_lds_bytes<BG, T, LAYERED>();
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(kDecThreads), lds, st, llr, ck, status, iters, 0, 0,
                       0, 0, (int64_t)0, (int64_t)0, L, (T)alpha, (T)beta, pc, work, cbs);
    return check_hip(hipGetLastError(), "ldpc_dec_kernel(mixed) launch");
}

// per-device scratch for the mixed path's work lists
struct MixedScratch {
    void* dev = nullptr;
    size_t cap = 0;
};
std::mutex g_mix_mu;
MixedScratch g_mix[64];

}  // namespace

// ================================================================================== C ABI
extern "C" {

const char* ldpc5g_version(void) { return LDPC5G_VERSION; }

const char* ldpc5g_last_error(void) { return g_err.c_str(); }

int ldpc5g_find_ils(int32_t Zc) {
    int i = zc_index(Zc);
    return i < 0 ? 255 : kLdpcZcSet[i];
}

int ldpc5g_encode(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc, int64_t ldk,
                  int64_t ldn, void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int K = (bgn == 1 ? 22 : 10) * Zc, N = (bgn == 1 ? 66 : 50) * Zc;
    if (B < 0 || ldk < K || ldn < N) return fail(LDPC5G_ESIZE, "bad sizes B=%d ldk=%lld ldn=%lld (K=%d N=%d)", B, (long long)ldk, (long long)ldn, K, N);
    if (B == 0) return LDPC5G_OK;
    if (!ck || !dn) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    const bool fast = (Zc % 16) == 0 && (ldk % 16) == 0 && (ldn % 16) == 0 &&
                      (((uintptr_t)ck) & 15) == 0 && (((uintptr_t)dn) & 15) == 0;
    if (fast) {
        static const int nt = [] {
            const char* e = getenv("LDPC5G_ENC_THREADS");
            int v = e ? atoi(e) : 64;
            return (v == 64 || v == 128 || v == 256) ? v : 64;
        }();
        if (bgn == 1) {
            size_t lds = enc_fast_lds_bytes<1>(Zc);
            hipLaunchKernelGGL(ldpc_enc_fast_kernel<1>, dim3(B), dim3(nt), lds, st, ck, dn, B, Zc, zi, ldk, ldn);
        } else {
            size_t lds = enc_fast_lds_bytes<2>(Zc);
            hipLaunchKernelGGL(ldpc_enc_fast_kernel<2>, dim3(B), dim3(nt), lds, st, ck, dn, B, Zc, zi, ldk, ldn);
        }
        return check_hip(hipGetLastError(), "ldpc_enc_fast_kernel launch");
    }
    if (bgn == 1) {
        size_t lds = enc_lds_bytes<1>(Zc);
        hipLaunchKernelGGL(ldpc_enc_kernel<1>, dim3(B), dim3(256), lds, st, ck, dn, B, Zc, zi, ldk, ldn);
    } else {
        size_t lds = enc_lds_bytes<2>(Zc);
        hipLaunchKernelGGL(ldpc_enc_kernel<2>, dim3(B), dim3(256), lds, st, ck, dn, B, Zc, zi, ldk, ldn);
    }
    return check_hip(hipGetLastError(), "ldpc_enc_kernel launch");
}

int ldpc5g_decode_ms(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L, double alpha,
                     double beta, int32_t schedule, int32_t flags, int64_t ldl, int64_t ldc,
                     void* stream) {
    g_err.clear();
    if (bgn != 1 && bgn != 2) return fail(LDPC5G_EBGN, "bgn must be 1 or 2 (got %d)", bgn);
    const int zi = zc_index(Zc);
    if (zi < 0) return fail(LDPC5G_EZC, "Zc=%d is not a TS 38.212 lifting size", Zc);
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    const int N = (bgn == 1 ? 66 : 50) * Zc + (2 - pc) * Zc, Nf = (bgn == 1 ? 68 : 52) * Zc;
    if (B < 0 || L < 0 || ldl < N || ldc < Nf)
        return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d ldl=%lld ldc=%lld (N=%d Nf=%d)", B, L, (long long)ldl, (long long)ldc, N, Nf);
    if (llr_dtype != LDPC5G_F64 && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "bad llr dtype %d", llr_dtype);
    if (schedule != LDPC5G_FLOODING && schedule != LDPC5G_LAYERED) return fail(LDPC5G_ESIZE, "bad schedule %d", schedule);
    if (schedule == LDPC5G_LAYERED && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "layered schedule requires float32 LLRs");
    if (B == 0) return LDPC5G_OK;
    if (!llr || !ck || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    const bool lay = schedule == LDPC5G_LAYERED;
    if (llr_dtype == LDPC5G_F64) {
        const double* p = (const double*)llr;
        return bgn == 1 ? launch_dec<1, double, false>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                        : launch_dec<2, double, false>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    }
    const float* p = (const float*)llr;
    if (bgn == 1)
        return lay ? launch_dec<1, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
                   : launch_dec<1, float, false>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
    return lay ? launch_dec<2, float, true>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st)
               : launch_dec<2, float, false>(p, ck, status, iters, B, Zc, zi, ldl, ldc, L, alpha, beta, pc, st);
}

int ldpc5g_decode_ms_mixed(const ldpc5g_cb_desc_t* desc, int32_t B, const void* llr_base,
                           int32_t llr_dtype, int8_t* ck_base, uint8_t* status, int32_t* iters,
                           int32_t L, double alpha, double beta, int32_t schedule, int32_t flags,
                           void* stream) {
    g_err.clear();
    const int pc = (flags & LDPC5G_LLR_FULL) ? 0 : 2;
    if (B < 0 || L < 0) return fail(LDPC5G_ESIZE, "bad sizes B=%d L=%d", B, L);
    if (llr_dtype != LDPC5G_F64 && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "bad llr dtype %d", llr_dtype);
    if (schedule != LDPC5G_FLOODING && schedule != LDPC5G_LAYERED) return fail(LDPC5G_ESIZE, "bad schedule %d", schedule);
    if (schedule == LDPC5G_LAYERED && llr_dtype != LDPC5G_F32) return fail(LDPC5G_ESIZE, "layered schedule requires float32 LLRs");
    if (B == 0) return LDPC5G_OK;
    if (!desc || !llr_base || !ck_base || !status || !iters) return fail(LDPC5G_ESIZE, "null buffer");
    // group codeblocks by (bgn, Zc), pack G = floor(384/Zc) per workgroup
    std::vector<std::vector<int>> bucket[2];
    bucket[0].resize(LDPC5G_NUM_ZC);
    bucket[1].resize(LDPC5G_NUM_ZC);
    for (int b = 0; b < B; ++b) {
        const ldpc5g_cb_desc_t& d = desc[b];
        if (d.bgn != 1 && d.bgn != 2) return fail(LDPC5G_EBGN, "desc[%d]: bgn must be 1 or 2 (got %d)", b, d.bgn);
        int zi = zc_index(d.Zc);
        if (zi < 0) return fail(LDPC5G_EZC, "desc[%d]: Zc=%d is not a lifting size", b, d.Zc);
        if (d.llr_off < 0 || d.ck_off < 0) return fail(LDPC5G_ESIZE, "desc[%d]: negative offset", b);
        bucket[d.bgn - 1][zi].push_back(b);
    }
    std::vector<DecWork> work[2];
    std::vector<CbRef> refs;
    for (int g = 0; g < 2; ++g)
        for (int zi = 0; zi < LDPC5G_NUM_ZC; ++zi) {
            const std::vector<int>& v = bucket[g][zi];
            const int Zc = kLdpcZcList[zi], G = dec_G(Zc);
            for (size_t s = 0; s < v.size(); s += G) {
                DecWork w;
                w.zi = zi, w.Zc = Zc, w.G = (int)std::min<size_t>(G, v.size() - s), w.first = (int)refs.size();
                for (int c = 0; c < w.G; ++c) {
                    CbRef r;
                    r.llr_off = desc[v[s + c]].llr_off, r.ck_off = desc[v[s + c]].ck_off, r.out = v[s + c], r.pad = 0;
                    refs.push_back(r);
                }
                work[g].push_back(w);
            }
        }
    const size_t wbytes = (work[0].size() + work[1].size()) * sizeof(DecWork);
    const size_t rbytes = refs.size() * sizeof(CbRef);
    const size_t need = wbytes + rbytes;
    int dev = 0;
    if (int rc = check_hip(hipGetDevice(&dev), "hipGetDevice")) return rc;
    hipStream_t st = (hipStream_t)stream;
    std::vector<unsigned char> host(need);
    memcpy(host.data(), work[0].data(), work[0].size() * sizeof(DecWork));
    memcpy(host.data() + work[0].size() * sizeof(DecWork), work[1].data(), work[1].size() * sizeof(DecWork));
    memcpy(host.data() + wbytes, refs.data(), rbytes);
    unsigned char* dbuf;
    {
        std::lock_guard<std::mutex> lk(g_mix_mu);
        MixedScratch& s = g_mix[dev & 63];
        if (s.cap < need) {
            if (s.dev) {
                (void)hipDeviceSynchronize();
                (void)hipFree(s.dev);
            }
            s.dev = nullptr;
            s.cap = 0;
            if (int rc = check_hip(hipMalloc(&s.dev, need * 2), "hipMalloc(work list)")) return rc;
            s.cap = need * 2;
        }
        dbuf = (unsigned char*)s.dev;
        // the work list is consumed by this call's kernels; a later call on another stream
        // would overwrite it, so the copy + launches are serialised on this stream and the
        // host waits for the copy before returning the buffer to the pool
        if (int rc = check_hip(hipMemcpyAsync(dbuf, host.data(), need, hipMemcpyHostToDevice, st), "hipMemcpyAsync(work list)")) return rc;
        const DecWork* w1 = (const DecWork*)dbuf;
        const DecWork* w2 = w1 + work[0].size();
        const CbRef* r = (const CbRef*)(dbuf + wbytes);
        const bool lay = schedule == LDPC5G_LAYERED;
        for (int g = 0; g < 2; ++g) {
            const int nwg = (int)work[g].size();
            if (!nwg) continue;
            const DecWork* w = g == 0 ? w1 : w2;
            int rc;
            if (llr_dtype == LDPC5G_F64) {
                const double* p = (const double*)llr_base;
                rc = g == 0 ? launch_dec_mixed<1, double, false>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st)
                            : launch_dec_mixed<2, double, false>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st);
            } else {
                const float* p = (const float*)llr_base;
                if (g == 0)
                    rc = lay ? launch_dec_mixed<1, float, true>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st)
                             : launch_dec_mixed<1, float, false>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st);
                else
                    rc = lay ? launch_dec_mixed<2, float, true>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st)
                             : launch_dec_mixed<2, float, false>(p, ck_base, status, iters, nwg, w, r, L, alpha, beta, pc, st);
            }
            if (rc) return rc;
        }
        if (int rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize(mixed)")) return rc;
    }
    return LDPC5G_OK;
}

}  // extern "C"
