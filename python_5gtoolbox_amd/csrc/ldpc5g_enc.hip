// ldpc5g_enc.hip — QC-LDPC encoder kernels (py5gphy/ldpc/nr_ldpc_encode.py:8-115)
// Part of libldpc5g.so (MI355X, gfx950); reference mapping in ldpc5g_common.h / DESIGN.md §4.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {
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
// Core-column edges of the extension rows (i >= 4), padded to MAXD slots per row: the edge list
// of phase 6, whose row index is per lane.  Slot (r, k) holds (column << 16 | edge id) or -1.
// Copied into LDS per workgroup with V mod Zc and the column's X offset folded in (empty slots
// point at a zero block), so the row loop reads its edges from LDS with no masking and no chain
// of dependent global loads.
template <int BG>
struct ExtEdges {
    static constexpr int R = BGT<BG>::MB - 4;
    int maxa = 0, maxd = 0, c0 = 0;   // section A: rows 0..3 (info columns); C from slot c0
    int32_t slot[BGT<BG>::MB * 12] = {};
    constexpr ExtEdges() {
        using P = BGT<BG>;
        for (int i = 0; i < P::MB; ++i) {
            int n = 0;
            for (int k = P::RS[i]; k < P::RS[i + 1]; ++k) n += P::COL[k] < (i < 4 ? P::KB : P::KC);
            if (i < 4) maxa = n > maxa ? n : maxa;
            else maxd = n > maxd ? n : maxd;
        }
        c0 = 4 * maxa;
        for (int i = 0; i < P::MB; ++i) {
            const int lim = i < 4 ? P::KB : P::KC, w = i < 4 ? maxa : maxd;
            const int base = i < 4 ? i * maxa : c0 + (i - 4) * maxd;
            int n = 0;
            for (int k = P::RS[i]; k < P::RS[i + 1]; ++k)
                if (P::COL[k] < lim) slot[base + n++] = (P::COL[k] << 16) | k;
            for (; n < w; ++n) slot[base + n] = -1;
        }
    }
    constexpr int size() const { return c0 + R * maxd; }
};
template <int BG>
constexpr ExtEdges<BG> kExtEdges{};
static_assert(kExtEdges<1>.size() <= BGT<1>::MB * 12 && kExtEdges<2>.size() <= BGT<2>::MB * 12, "slots");
__device__ const ExtEdges<1> kExtEdges1D = ExtEdges<1>{};   // device copies (runtime-indexed)
__device__ const ExtEdges<2> kExtEdges2D = ExtEdges<2>{};
template <int BG>
__device__ __forceinline__ int ext_slot(int c) {
    if constexpr (BG == 1) return kExtEdges1D.slot[c];
    else return kExtEdges2D.slot[c];
}

struct EncFastLayout {
    int K, N, W, DW, KW, words, tab, zoff;
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
    // ib[KW+2] | X[KC*DW] | lam[4W] | pv[5W + 2] | ext edge slots [R*MAXD] | zero block [DW]
    L.tab = (L.KW + 2) + P::KC * L.DW + 4 * L.W + 5 * L.W + 2;
    L.zoff = L.tab + kExtEdges<BG>.size() - (L.KW + 2);   // zero block, in words from X
    L.words = L.tab + kExtEdges<BG>.size() + L.DW;
    return L;
}

// Fill the LDS edge slots of phase 6: bit address (from X) of the window start of slot (r, k) for
// word 0, i.e. 32 * (column * DW) + V mod Zc, or the zero block for empty slots.
template <int BG>
__device__ __forceinline__ void enc_fill_ext_tab(uint32_t* sm, const EncFastLayout& Ly, int zi, int t, int NT) {
    uint32_t* tab = sm + Ly.tab;
    for (int c = t; c < kExtEdges<BG>.size(); c += NT) {
        const int v = ext_slot<BG>(c);
        tab[c] = v < 0 ? 32u * (uint32_t)Ly.zoff
                       : 32u * (uint32_t)((v >> 16) * Ly.DW) + (uint32_t)shift_of<BG>(zi, v & 0xffff);
    }
    for (int w = t; w < Ly.DW; w += NT) tab[kExtEdges<BG>.size() + w] = 0u;
}
template <int BG>
inline size_t enc_fast_lds_bytes(int Zc) {
    return (size_t)enc_fast_layout<BG>(Zc).words * 4;
}

// Word q of the periodic extension X[t] = block[t mod Zc] of the Zc-bit block at bit `base` of
// v: a plain word copy when Zc is a multiple of 32 (q < DW = 2W + 2), else a rotated window.
__device__ __forceinline__ uint32_t ext_word(const uint32_t* v, int base, int Zc, int W, int q) {
    if ((Zc & 31) == 0) return v[(base >> 5) + (q < W ? q : q < 2 * W ? q - W : q - 2 * W)];
    return fetch_rot32(v, base, Zc, mod_zc(32 * q, Zc));
}

// 16-B store of encoder output (non-temporal stores measured 2x slower)
template <typename V>
__device__ __forceinline__ void st16(int8_t* p, V v) {
    *(V*)p = v;
}

// Bit-matrix transpose between "byte k of word q" and "bit 4q + k" orders, by four delta swaps
// of the 5 index bits: tr84 moves bit 8k + j to bit 4j + k (k < 4, j < 8); tr84_inv undoes it.
__device__ __forceinline__ uint32_t dswap(uint32_t x, int d, uint32_t m) {
    const uint32_t t = ((x >> d) ^ x) & m;
    return x ^ t ^ (t << d);
}
__device__ __forceinline__ uint32_t tr84(uint32_t x) {
    x = dswap(x, 12, 0x0000f0f0u);
    x = dswap(x, 6, 0x00cc00ccu);
    x = dswap(x, 3, 0x0a0a0a0au);
    return dswap(x, 1, 0x22222222u);
}
__device__ __forceinline__ uint32_t tr84_inv(uint32_t x) {
    x = dswap(x, 1, 0x22222222u);
    x = dswap(x, 3, 0x0a0a0a0au);
    x = dswap(x, 6, 0x00cc00ccu);
    return dswap(x, 12, 0x0000f0f0u);
}

// 32 parity bits -> 32 int8 bytes (nbits = 32 or 16) at a 16-B aligned address: byte k of
// output word q is bit 4q + k, i.e. bit q of byte k of tr84_inv(bits)
__device__ __forceinline__ void store_bits(int8_t* dst, uint32_t bits, int nbits) {
    const uint32_t u = tr84_inv(bits);
    uint4 a = make_uint4(u & 0x01010101u, (u >> 1) & 0x01010101u, (u >> 2) & 0x01010101u,
                         (u >> 3) & 0x01010101u);
    st16(dst, a);
    if (nbits > 16) {
        uint4 b = make_uint4((u >> 4) & 0x01010101u, (u >> 5) & 0x01010101u, (u >> 6) & 0x01010101u,
                             (u >> 7) & 0x01010101u);
        st16(dst + 16, b);
    }
}

// Phase 1 of the fast encoder for one 32-byte chunk (word wi): pack the parity bits (fillers at
// k >= 2Zc -> 0, nr_ldpc_encode.py:32-37) and store the systematic bytes straight to dn.
__device__ __forceinline__ uint32_t enc_pack_chunk(const int4 (&v)[2], int base, int twoZ, int8_t* dst) {
    if (base >= twoZ) {   // 2Zc and K are multiples of 32 here
        st16(dst + base - twoZ, v[0]);
        st16(dst + base - twoZ + 16, v[1]);
    }
    const uint32_t* d = (const uint32_t*)v;
    // common case, every byte 0 or 1 (no fillers): OR the words with byte k of word q landing in
    // bit 8k + q, then one transpose to bit 4q + k
    uint32_t any = 0, u = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) any |= d[q], u |= d[q] << q;
    if (!(any & 0xfefefefeu)) return tr84(u);
    uint32_t bits = 0;
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
    return bits;
}

// Half-chunk variant (coalesced phase 1): 16 bytes = words q = 4h..4h+3 of a 32-byte chunk at
// byte `base` (= chunk start + 16h); returns their bits at 16h..16h+15 (zero elsewhere), stores
// the systematic bytes.  Same filler rule as enc_pack_chunk.
__device__ __forceinline__ uint32_t enc_pack_half(const int4& v, int base, int h, int twoZ, int8_t* dst) {
    if (base >= twoZ) st16(dst + base - twoZ, v);
    const uint32_t* d = (const uint32_t*)&v;
    uint32_t any = 0, u = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) any |= d[q], u |= d[q] << q;
    if (!(any & 0xfefefefeu)) return tr84(u << (4 * h));
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = d[q];
        uint32_t lsb = x & 0x01010101u;
        const uint32_t ff = (x & (x >> 1) & (x >> 2) & (x >> 3) & (x >> 4) & (x >> 5) &
                             (x >> 6) & (x >> 7)) & 0x01010101u;
        if (base + 4 * q >= twoZ) lsb &= ~ff;
        bits |= ((lsb | (lsb >> 7) | (lsb >> 14) | (lsb >> 21)) & 15u) << (4 * q);
    }
    return bits << (16 * h);
}

// 16 parity bits (bits 0..15 of b) -> 16 int8 bytes at a 16-B aligned address
__device__ __forceinline__ void store_bits16(int8_t* dst, uint32_t b) {
    const uint32_t u = tr84_inv(b & 0xffffu);
    st16(dst, make_uint4(u & 0x01010101u, (u >> 1) & 0x01010101u, (u >> 2) & 0x01010101u,
                         (u >> 3) & 0x01010101u));
}

// development instrumentation (tools/enc_ts_probe.py): thread 0's real-time clock (100 MHz) at
// phase boundaries, written over the first 64 bytes of the codeblock's output at the end
#ifdef LDPC5G_ENC_TS
#define ENC_TS(n) \
    if (t == 0) enc_tsv[(n)] = __builtin_amdgcn_s_memrealtime()
#else
#define ENC_TS(n)
#endif

template <bool LDSONLY>
__device__ __forceinline__ void enc_sync() {
    if constexpr (LDSONLY) lds_sync();
    else __syncthreads();
}

// Phases 2-6 of the fast encoder for one codeblock whose packed bits are in ib (LDS): parity
// straight to dst.  LDSONLY: barriers order LDS only, so the systematic and parity stores stay in
// flight across them.
template <int BG, bool LDSONLY>
__device__ __forceinline__ void enc_fast_parity(const EncFastLayout& Ly, uint32_t* sm, int8_t* dst,
                                                int Zc, int zi, int t, int NT, bool direct
#ifdef LDPC5G_ENC_TS
                                                , uint64_t* enc_tsv
#endif
                                                ) {
    using P = BGT<BG>;
    const int K = Ly.K, W = Ly.W, DW = Ly.DW, KW = Ly.KW;
    const int S = K - 2 * Zc;
    uint32_t* ib = sm;
    uint32_t* X = ib + KW + 2;
    uint32_t* lam = X + P::KC * DW;
    uint32_t* pv = lam + 4 * W;   // p1 p2 p3 p4 L2

    // ---- 2. periodic extensions of the information columns (task = j * DW + q); skipped when
    //      phase 1 already wrote them (Zc % 32 == 0, coalesced path: enc_direct_x)
    if (!direct) {
        const int dj = NT / DW, dq = NT - dj * DW;
        int j = t / DW, q = t - j * DW;
        for (int task = t; task < P::KB * DW; task += NT) {
            X[task] = ext_word(ib, j * Zc, Zc, W, q);
            j += dj, q += dq;
            if (q >= DW) q -= DW, ++j;
        }
    }
    if (!direct) enc_sync<LDSONLY>();
    ENC_TS(3);

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
        // lambda_i = A_i c: lane t = i W + w < 4W owns word w of core row i; its edges come from
        // section A of the LDS edge slots (empty slots read the zero block), so the window reads
        // are independent LDS loads in flight together
        if (t < 4 * W) {
            constexpr int MAXA = kExtEdges<BG>.maxa;
            const int i = t / W, w = t - i * W;
            const uint32_t* ta = sm + Ly.tab + i * MAXA;
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < MAXA; ++k) acc ^= window32(X, (int)ta[k] + 32 * w);
            lam[t] = acc;
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
    enc_sync<LDSONLY>();
    ENC_TS(4);

    // ---- 5. extensions of the 4 core parity columns; core parity bytes straight to dn
    for (int task = t; task < 4 * DW; task += NT) {
        int k = task / DW, q = task - k * DW;
        X[(P::KB + k) * DW + q] = ext_word(pv + k * W, 0, Zc, W, q);
    }
    for (int task = t; task < 4 * W; task += NT) {
        int k = task / W, w = task - k * W;
        store_bits(dst + S + k * Zc + 32 * w, pv[k * W + w], min(32, Zc - 32 * w));
    }
    enc_sync<LDSONLY>();
    ENC_TS(5);

    // ---- 6. extension parity rows, each row-word stored straight to dn.  The row is per lane;
    //      its MAXD edge slots come from the LDS table (enc_fill_ext_tab), empty ones reading
    //      the zero block, so all of a task's loads are independent
    constexpr int MAXD = kExtEdges<BG>.maxd;
    const uint32_t* tab = sm + Ly.tab;
    const int dq = NT / W, dw = NT - dq * W;   // (r, w) of task t + NT from that of task t
    int r = t / W, w = t - r * W;
    const int ntask = (P::MB - 4) * W;
    // Zc % 32 == 0: the extension rows are one contiguous byte range and task T is its bytes
    // [32T, 32T + 32), so a wave's 64 tasks are 2 KB in a row.  Lane l then stores 16-byte piece l
    // and piece 64 + l of that range (words l/2 and 32 + l/2, fetched with two lane permutes):
    // each store instruction writes 1 KB contiguous instead of 16 B every 32 B.
    const bool coal = (Zc & 31) == 0 && (NT & 63) == 0;
    const int lane = t & 63;
    int8_t* ext = dst + S + 4 * Zc;
    for (int task0 = t; task0 - lane < ntask; task0 += NT) {   // wave-uniform trip count
        const int task = task0;
        uint32_t acc = 0;
        if (task < ntask) {
#pragma unroll
            for (int k = 0; k < MAXD; ++k) acc ^= window32(X, (int)tab[kExtEdges<BG>.c0 + r * MAXD + k] + 32 * w);
        }
        if (coal) {
            const int wbase = task - lane;   // first task of this wave's 64
            const uint32_t a0 = (uint32_t)__shfl((int)acc, lane >> 1, 64);
            const uint32_t a1 = (uint32_t)__shfl((int)acc, 32 + (lane >> 1), 64);
            const int h = lane & 1;
            if (wbase + (lane >> 1) < ntask) store_bits16(ext + 32 * wbase + 16 * lane, a0 >> (16 * h));
            if (wbase + 32 + (lane >> 1) < ntask) store_bits16(ext + 32 * wbase + 1024 + 16 * lane, a1 >> (16 * h));
        } else if (task < ntask) {
            store_bits(dst + S + (4 + r) * Zc + 32 * w, acc, min(32, Zc - 32 * w));
        }
        r += dq, w += dw;
        if (w >= W) w -= W, ++r;
    }
}

#ifndef LDPC5G_ENC_NT
#define LDPC5G_ENC_NT 128
#endif
constexpr int kEncChunks = 3;   // 3 x 128 threads x 32 B >= K = 8448 (BG1 Zc=384): one round
constexpr int kEncPieces = 6;   // 6 x 128 threads x 16 B >= K: one round (coalesced phase 1)
template <int BG, bool LDSONLY>
__global__ __launch_bounds__(256) void ldpc_enc_fast_kernel(const int8_t* __restrict__ ck,
                                                            int8_t* __restrict__ dn, int B, int Zc,
                                                            int zi, int64_t ldk, int64_t ldn) {
    const int b = blockIdx.x;
    if (b >= B) return;
    const int t = threadIdx.x;
    const int NT = blockDim.x;
#ifdef LDPC5G_ENC_TS
    uint64_t enc_tsv[8] = {};
#endif
    ENC_TS(0);
    const EncFastLayout Ly = enc_fast_layout<BG>(Zc);
    const int twoZ = 2 * Zc;
    // Zc % 32 == 0 on the coalesced path: phase 1 writes the periodic extensions itself (no
    // phase 2 and one barrier less); w / W by a multiply-high (exact: w < 2^10, 2 <= W <= 12)
    const bool direct = (Zc & 31) == 0 && (NT & 63) == 0;
    const uint32_t wdiv = (uint32_t)(0xffffffffu / (uint32_t)Ly.W) + 1u;
    extern __shared__ __align__(16) uint32_t sm[];
    const int8_t* src = ck + (int64_t)b * ldk;
    int8_t* dst = dn + (int64_t)b * ldn;
    // ---- 1. info bytes: pack parity bits; the systematic part is stored straight to dn.  Up to
    //      kEncChunks 32-B chunks per thread are loaded before any is used (one HBM round trip,
    //      not one per chunk); the phase-6 edge table is filled meanwhile.
    if ((NT & 63) == 0) {
        // 16-byte pieces, lane-contiguous (piece p = half p & 1 of chunk p / 2): every load and
        // systematic store instruction moves 1 KB contiguous; the two halves of a chunk sit in
        // lanes l, l ^ 1 of the same wave and are joined with one lane exchange.
        const int np = 2 * Ly.KW;
        // wave-uniform trip count, at least one round (the edge-table fill is in it)
        for (int p0 = t; p0 == t || p0 - (t & 63) < np; p0 += kEncPieces * NT) {
            int4 v[kEncPieces];
#pragma unroll
            for (int c = 0; c < kEncPieces; ++c) {
                const int pc = p0 + c * NT;
                if (pc < np) v[c] = *(const int4*)(src + 16 * pc);
            }
            if (p0 == t) enc_fill_ext_tab<BG>(sm, Ly, zi, t, NT);   // every thread, first round
#pragma unroll
            for (int c = 0; c < kEncPieces; ++c) {
                const int pc = p0 + c * NT;
                if (pc - (t & 63) >= np) break;   // wave-uniform
                uint32_t part = pc < np ? enc_pack_half(v[c], 16 * pc, pc & 1, twoZ, dst) : 0u;
                part |= (uint32_t)__shfl_xor((int)part, 1, 64);
                if (pc < np && !(pc & 1)) {
                    const int w = pc >> 1;
                    if (direct) {
                        // word q of column j straight into its periodic extension X_j (word
                        // copies: X_j[q] = X_j[W + q] = block_j[q], and the two words past 2W)
                        const int j = Ly.W == 1 ? w : (int)__umulhi((uint32_t)w, wdiv), q = w - j * Ly.W;
                        uint32_t* xj = sm + Ly.KW + 2 + j * Ly.DW;
                        xj[q] = part, xj[Ly.W + q] = part;
                        if (q < 2) xj[2 * Ly.W + q] = part;
                    } else {
                        sm[w] = part;
                    }
                }
            }
        }
    } else
    for (int w0 = t; w0 < t + Ly.KW; w0 += kEncChunks * NT) {   // K = Kb*Zc: multiple of 32 here
        int4 v[kEncChunks][2];
#pragma unroll
        for (int c = 0; c < kEncChunks; ++c) {
            const int wi = w0 + c * NT;
            if (wi < Ly.KW) {
                v[c][0] = *(const int4*)(src + wi * 32);
                v[c][1] = *(const int4*)(src + wi * 32 + 16);
            }
        }
        if (w0 == t) enc_fill_ext_tab<BG>(sm, Ly, zi, t, NT);   // every thread, first round
#pragma unroll
        for (int c = 0; c < kEncChunks; ++c) {
            const int wi = w0 + c * NT;
            if (wi < Ly.KW) sm[wi] = enc_pack_chunk(v[c], wi * 32, twoZ, dst);
        }
    }
    if (t < 2) sm[Ly.KW + t] = 0;
    ENC_TS(1);
    enc_sync<LDSONLY>();
    ENC_TS(2);
#ifdef LDPC5G_ENC_TS
    enc_fast_parity<BG, LDSONLY>(Ly, sm, dst, Zc, zi, t, NT, direct, enc_tsv);
    ENC_TS(6);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ENC_TS(7);
    if (t == 0) {
        for (int q = 0; q < 8; ++q) ((uint64_t*)dst)[q] = enc_tsv[q];
        ((uint64_t*)dst)[8] = (uint64_t)__smid();
    }
#else
    enc_fast_parity<BG, LDSONLY>(Ly, sm, dst, Zc, zi, t, NT, direct);
#endif
}

}  // namespace

int launch_encode(const int8_t* ck, int8_t* dn, int B, int bgn, int Zc, int zi, int64_t ldk,
                  int64_t ldn, hipStream_t st) {
    const bool fast = (Zc % 16) == 0 && (ldk % 16) == 0 && (ldn % 16) == 0 &&
                      (((uintptr_t)ck) & 15) == 0 && (((uintptr_t)dn) & 15) == 0;
    if (fast) {
        // one 128-thread workgroup per codeblock (measured r01c/r01m: a pipelined persistent
        // variant 62 us, 256 threads +8 %, full barriers +0.5 % vs 25-40 us: the per-codeblock
        // LDS/VALU critical path, not HBM, sets the time, so most codeblocks in flight wins;
        // r05: 64-thread workgroups 4.10-4.55 TB/s and two codeblocks per workgroup with the
        // second one's loads issued before the first one's parity 4.23-4.94 TB/s, vs 4.53-5.21)
        constexpr int nt = LDPC5G_ENC_NT;
        if (bgn == 1)
            hipLaunchKernelGGL((ldpc_enc_fast_kernel<1, true>), dim3(B), dim3(nt), enc_fast_lds_bytes<1>(Zc),
                               st, ck, dn, B, Zc, zi, ldk, ldn);
        else
            hipLaunchKernelGGL((ldpc_enc_fast_kernel<2, true>), dim3(B), dim3(nt), enc_fast_lds_bytes<2>(Zc),
                               st, ck, dn, B, Zc, zi, ldk, ldn);
        return check_hip(hipGetLastError(), "ldpc_enc_fast_kernel launch");
    }
    if (bgn == 1)
        hipLaunchKernelGGL(ldpc_enc_kernel<1>, dim3(B), dim3(256), enc_lds_bytes<1>(Zc), st, ck, dn,
                           B, Zc, zi, ldk, ldn);
    else
        hipLaunchKernelGGL(ldpc_enc_kernel<2>, dim3(B), dim3(256), enc_lds_bytes<2>(Zc), st, ck, dn,
                           B, Zc, zi, ldk, ldn);
    return check_hip(hipGetLastError(), "ldpc_enc_kernel launch");
}

}  // namespace ldpc5g_impl
