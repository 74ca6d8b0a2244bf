// ldpc5g_sch.hip — the DL-SCH / UL-SCH transport-channel chain around the LDPC codec, on the
// GPU and batched over transport blocks that share one configuration (TS 38.212 §7.2 / §6.2):
//   CRC attach / check ............ py5gphy/crc/crc.py:4-88
//   codeblock segmentation ........ py5gphy/ldpc/nr_ldpc_cbsegment.py:7-33, ldpc_info.py:5-78
//   rate matching ................. py5gphy/ldpc/nr_ldpc_ratematch.py:5-97
//   rate recovery + HARQ combine .. py5gphy/ldpc/nr_ldpc_raterecover.py:6-65,
//                                   py5gphy/nr_pdsch/nr_dlsch_decode.py:62-88
//   TB reassembly + CRC checks .... py5gphy/nr_pdsch/nr_dlsch_decode.py:93-106
// The chains themselves: DLSCHEncode (nr_dlsch.py:12-74), ULSCH_Crc_CodeBlockSegment +
// ULSCH_encoding_ratematch (nr_ulsch.py:13-70), DLSCHDecode (nr_dlsch_decode.py:13-110),
// ULSCH_decoding (nr_ulsch_decode.py:13-110).
//
// All of it is byte / integer work bound by HBM or latency, not arithmetic: bits stay one per
// int8 (the reference's own representation and the encoder/decoder ABI); a lane reads 64 of them
// with 16-byte loads, packs them into a word and runs a byte-table LFSR over it, and CRCs are
// combined across lanes, codeblocks and transport blocks through the linearity
// crc(M1 || M2) = crc(M1) * x^|M2| + crc(M2)  (mod g).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {

// ===================================================================================== CRC
// Generators without the x^L term, coefficients x^(L-1) .. x^0 (crc.py:94-106).
struct CrcPoly {
    int L;
    uint32_t g;
};
constexpr CrcPoly kCrcPoly[6] = {{6, 0x21u},      {11, 0x621u},     {16, 0x1021u},
                                 {24, 0x864CFBu}, {24, 0x800063u}, {24, 0xB2B117u}};

__host__ __device__ constexpr uint32_t crc_mulx(uint32_t a, int L, uint32_t g) {
    return ((a << 1) & ((1u << L) - 1u)) ^ (((a >> (L - 1)) & 1u) ? g : 0u);
}
// a(x) * b(x) mod (x^L + g(x))
__host__ __device__ constexpr uint32_t crc_mulmod(uint32_t a, uint32_t b, int L, uint32_t g) {
    uint32_t r = 0;
    for (int i = 0; i < L; ++i) {
        if ((b >> i) & 1u) r ^= a;
        a = crc_mulx(a, L, g);
    }
    return r;
}

constexpr int kCrcNT = 256;              // threads of a CRC workgroup
constexpr int kCrcChunkWords = kCrcNT;   // 64-bit message words per workgroup chunk (16384 bits)

struct CrcTables {
    uint32_t xp2[6][40];                // x^(2^i) mod g
    uint32_t x64[6][kCrcChunkWords];    // x^(64 m) mod g
    uint32_t byte[6][256];              // v(x) x^L mod g: the register after feeding byte v, MSB first
};
constexpr CrcTables make_crc_tables() {
    CrcTables t{};
    for (int p = 0; p < 6; ++p) {
        const int L = kCrcPoly[p].L;
        const uint32_t g = kCrcPoly[p].g;
        t.xp2[p][0] = 2u;
        for (int i = 1; i < 40; ++i) t.xp2[p][i] = crc_mulmod(t.xp2[p][i - 1], t.xp2[p][i - 1], L, g);
        t.x64[p][0] = 1u;
        for (int m = 1; m < kCrcChunkWords; ++m) t.x64[p][m] = crc_mulmod(t.x64[p][m - 1], t.xp2[p][6], L, g);
        for (int v = 0; v < 256; ++v) {
            uint32_t reg = 0;
            for (int k = 7; k >= 0; --k) {
                const uint32_t fb = ((reg >> (L - 1)) ^ (uint32_t)(v >> k)) & 1u;
                reg = ((reg << 1) & ((1u << L) - 1u)) ^ (fb ? g : 0u);
            }
            t.byte[p][v] = reg;
        }
    }
    return t;
}
__constant__ CrcTables kCrcTab = make_crc_tables();

__device__ uint32_t crc_xpow(int64_t n, int p) {   // x^n mod g
    const int L = kCrcPoly[p].L;
    const uint32_t g = kCrcPoly[p].g;
    uint32_t r = 1u;
    for (int i = 0; n; ++i, n >>= 1)
        if (n & 1) r = crc_mulmod(r, kCrcTab.xp2[p][i], L, g);
    return r;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
    return v;
}

// Per-workgroup CRC state in LDS: byte tables of the (up to two) polynomials being computed,
// wave partials and the ragged last word's CRC.
struct CrcLds {
    uint32_t tab[2][256];
    uint32_t red[2][kCrcNT / 64];
    uint32_t part[2];
    uint32_t dist[2];   // x^(bits after the chunk's last full word) mod g
};
__device__ __forceinline__ void crc_lds_init(CrcLds& S, int p0, int p1) {   // kCrcNT == 256
    S.tab[0][threadIdx.x] = kCrcTab.byte[p0][threadIdx.x];
    if (p1 >= 0) S.tab[1][threadIdx.x] = kCrcTab.byte[p1][threadIdx.x];
    __syncthreads();
}

// reg * x^8 + byte * x^L  (mod g): one table step, message byte MSB (= earliest bit) first
__device__ __forceinline__ uint32_t crc_step8(uint32_t reg, uint32_t byte, int L, const uint32_t* tab) {
    if (L >= 8) return ((reg << 8) & ((1u << L) - 1u)) ^ tab[((reg >> (L - 8)) ^ byte) & 0xFFu];
    return tab[((reg << (8 - L)) ^ byte) & 0xFFu];
}
// CRC register of the nb <= 64 message bits held in w (bit k = message bit k): W(x) x^L mod g
// (the long division of crc.py:28-33)
__device__ __forceinline__ uint32_t crc_word(uint64_t w, int nb, int L, uint32_t g, const uint32_t* tab) {
    const uint64_t rv = __builtin_bitreverse64(w);   // message bit k at bit 63 - k
    uint32_t reg = 0;
    if (nb == 64) {
#pragma unroll
        for (int b = 0; b < 8; ++b) reg = crc_step8(reg, (uint32_t)(rv >> (56 - 8 * b)), L, tab);
        return reg;
    }
    int k = 0;
    for (; k + 8 <= nb; k += 8) reg = crc_step8(reg, (uint32_t)(rv >> (56 - k)), L, tab);
    for (; k < nb; ++k) {
        const uint32_t fb = ((reg >> (L - 1)) ^ (uint32_t)(w >> k)) & 1u;
        reg = ((reg << 1) & ((1u << L) - 1u)) ^ (fb ? g : 0u);
    }
    return reg;
}

// LSBs of four 0/1 bytes -> 4 bits (byte j -> bit j)
__device__ __forceinline__ uint32_t pack4(uint32_t x) { return (((x & 0x01010101u) * 0x01020408u) >> 24) & 0xFu; }

template <typename V>
__device__ __forceinline__ uint64_t load_bits64_vec(const int8_t* p, int8_t* dst) {
    constexpr int n = 64 / (int)sizeof(V);
    V x[n];
#pragma unroll
    for (int k = 0; k < n; ++k) x[k] = reinterpret_cast<const V*>(p)[k];
    uint64_t w = 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        const uint32_t* u = reinterpret_cast<const uint32_t*>(&x[k]);
#pragma unroll
        for (int j = 0; j < (int)sizeof(V) / 4; ++j)
            w |= (uint64_t)pack4(u[j]) << (4 * (k * (int)sizeof(V) / 4 + j));
    }
    if (dst) {
#pragma unroll
        for (int k = 0; k < n; ++k) reinterpret_cast<V*>(dst)[k] = x[k];
    }
    return w;
}
// nb <= 64 message bytes at p (0/1 each) -> bits of a word (byte j -> bit j); copies the bytes to
// dst when given.  `al` = common alignment of p and dst (16, 8, 4 or 1), uniform per workgroup.
__device__ __forceinline__ uint64_t load_bits64(const int8_t* p, int nb, int8_t* dst, int al) {
    if (nb == 64) {
        if (al >= 16) return load_bits64_vec<uint4>(p, dst);
        if (al >= 8) return load_bits64_vec<uint2>(p, dst);
        if (al >= 4) return load_bits64_vec<uint32_t>(p, dst);
    }
    uint64_t w = 0;
    for (int j = 0; j < nb; ++j) {
        const int8_t v = p[j];
        w |= (uint64_t)(v & 1) << j;
        if (dst) dst[j] = v;
    }
    return w;
}
__device__ __forceinline__ int ptr_align(const void* a, const void* b) {
    const uintptr_t u = (uintptr_t)a | (b ? (uintptr_t)b : 0);
    return (u & 15) == 0 ? 16 : (u & 7) == 0 ? 8 : (u & 3) == 0 ? 4 : 1;
}

// Contribution of chunk `chunk` (64-bit words [256 chunk, 256 chunk + 256), word q = message bits
// [64q, 64q + 64)) of the nbits-long message at src (one int8 0/1 per bit) to its CRC under
// polynomial ids p[0..NP): crc(chunk) * x^(bits after the chunk), in out[] of thread 0.  Each lane
// loads its word's 64 bytes with vector loads (copying them to dst if given), runs a byte-table
// LFSR over them and scales the result by x^(64 (words after it in the chunk)); the workgroup XORs
// the partials and thread 0 applies the chunk's distance to the end.  All threads must call it;
// S.tab[i] must hold the byte table of p[i].
template <int NP>
__device__ void wg_crc_mem(const int8_t* src, int8_t* dst, int64_t nbits, int64_t chunk,
                           const int (&p)[NP], CrcLds& S, uint32_t (&out)[NP]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nfull = nbits >> 6;
    const int lw = (int)(nbits & 63);
    const int64_t q0 = chunk * kCrcChunkWords, q = q0 + threadIdx.x;
    const int64_t qf = min(q0 + kCrcChunkWords - 1, nfull - 1);   // last full word in the chunk
    const int al = ptr_align(src, dst);
    // the chunk's distance to the message end (up to ~20 serial mulmods for a long message) is
    // formed by the last thread before its loads, beside the other lanes' loads, instead of by
    // thread 0 after the reduction; the barrier below publishes it
    if (threadIdx.x == kCrcNT - 1)
#pragma unroll
        for (int i = 0; i < NP; ++i)
            S.dist[i] = qf >= q0 ? crc_xpow(64 * (nfull - 1 - qf) + lw, p[i]) : 1u;
    uint32_t c[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) c[i] = 0;
    if (q < nfull || (q == nfull && lw > 0)) {
        const int nb = q < nfull ? 64 : lw;
        const uint64_t w = load_bits64(src + 64 * q, nb, dst ? dst + 64 * q : nullptr, al);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int L = kCrcPoly[p[i]].L;
            const uint32_t g = kCrcPoly[p[i]].g;
            const uint32_t r = crc_word(w, nb, L, g, S.tab[i]);
            if (q < nfull) {
                c[i] = crc_mulmod(r, kCrcTab.x64[p[i]][qf - q], L, g);
            } else {
                S.part[i] = r;   // ragged last word: nothing follows it
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        c[i] = wave_xor(c[i]);
        if (lane == 0) S.red[i][wv] = c[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            uint32_t r = 0;
            for (int w = 0; w < kCrcNT / 64; ++w) r ^= S.red[i][w];
            if (qf >= q0 && r) r = crc_mulmod(r, S.dist[i], kCrcPoly[p[i]].L, kCrcPoly[p[i]].g);
            if (lw > 0 && nfull >= q0 && nfull < q0 + kCrcChunkWords) r ^= S.part[i];
            out[i] = r;
        }
    }
    __syncthreads();
}

__host__ __device__ inline int64_t crc_chunks(int64_t nbits) {
    return ((nbits + 63) / 64 + kCrcChunkWords - 1) / kCrcChunkWords;
}

// CRC register of n <= 32 bits given MSB-first in v (bit n-1 first), continuing from reg
__device__ __forceinline__ uint32_t crc_bits_msb(uint32_t reg, uint32_t v, int n, int L, uint32_t g) {
    for (int k = n - 1; k >= 0; --k) {
        const uint32_t fb = ((reg >> (L - 1)) ^ (v >> k)) & 1u;
        reg = ((reg << 1) & ((1u << L) - 1u)) ^ (fb ? g : 0u);
    }
    return reg;
}

// rem[r] ^= crc contribution of chunk blockIdx.y of row r (rem zeroed by the launcher)
__global__ __launch_bounds__(kCrcNT) void crc_rows_kernel(const int8_t* __restrict__ bits, int64_t ld,
                                                          int64_t nbits, int p, uint32_t* rem) {
    __shared__ CrcLds S;
    crc_lds_init(S, p, -1);
    const int pp[1] = {p};
    uint32_t c[1];
    wg_crc_mem<1>(bits + (int64_t)blockIdx.x * ld, nullptr, nbits, blockIdx.y, pp, S, c);
    if (threadIdx.x == 0 && c[0]) atomicXor(&rem[blockIdx.x], c[0]);
}

// ============================================================================ SCH geometry
struct SchDev {
    int32_t A, B, tbp, Ltb, bgn, C, cbz, Lcb, K, K_apo, Zc, N, Ncb, Qm;
    int32_t E_lo, E_hi, c_switch;
    int32_t f0, F, Fin, size, start;   // fillers [f0, f0+F) of dn; Fin of them below Ncb
    int64_t G;
};

// Per-TB geometry of a multi-configuration batch (ldpc5g_sch_*_multi): every TB has its own
// configuration; its codeblock rows sit consecutively in the flat workspaces at these offsets.
struct SchGeo {
    SchDev s;
    int64_t ck_off, dn_off, dck_off;   // elements: first row in ck (K), dn / llr_dn (N), decoder ck (Nf)
    int32_t cb_off, dck_ld;            // first codeblock index (status, cb_ok); decoder ck row length
};
struct RowRef {
    int32_t t, c;   // codeblock row -> (TB, codeblock in TB)
};
// Codeblock row r: one shared configuration (gv == nullptr: t = r / C, rows strided by K / N /
// dck_ld0), or the row's TB geometry.
struct RowGeo {
    SchDev s;
    int t, c, cbi;
    int64_t ck_row, dn_row, dck_row;
};
__device__ __forceinline__ RowGeo row_geo(int r, const SchDev& s0, const SchGeo* gv, const RowRef* rm,
                                          int64_t dck_ld0) {
    RowGeo g;
    if (!gv) {
        g.s = s0;
        g.t = r / s0.C, g.c = r - g.t * s0.C, g.cbi = r;
        g.ck_row = (int64_t)r * s0.K, g.dn_row = (int64_t)r * s0.N, g.dck_row = (int64_t)r * dck_ld0;
    } else {
        const RowRef rr = rm[r];
        const SchGeo& G = gv[rr.t];
        g.s = G.s;
        g.t = rr.t, g.c = rr.c, g.cbi = G.cb_off + rr.c;
        g.ck_row = G.ck_off + (int64_t)rr.c * G.s.K, g.dn_row = G.dn_off + (int64_t)rr.c * G.s.N;
        g.dck_row = G.dck_off + (int64_t)rr.c * G.dck_ld;
    }
    return g;
}

__device__ __forceinline__ int cb_E(const SchDev& s, int c) { return c < s.c_switch ? s.E_lo : s.E_hi; }
__device__ __forceinline__ int64_t cb_goff(const SchDev& s, int c) {
    return (int64_t)c * s.E_lo + (int64_t)max(0, c - s.c_switch) * (s.E_hi - s.E_lo);
}

// ------------------------------------------------------------------------------- transmit
// TB CRC (24A / 16) of every transport block: tbcrc[t] ^= chunk contributions
__global__ __launch_bounds__(kCrcNT) void tb_crc_kernel(const int8_t* __restrict__ trblk, int64_t lda,
                                                        SchDev s0, const SchGeo* __restrict__ gv,
                                                        uint32_t* tbcrc) {
    __shared__ CrcLds S;
    const SchDev s = gv ? gv[blockIdx.x].s : s0;
    if ((int64_t)blockIdx.y >= crc_chunks(s.A)) return;   // multi: grid sized for the longest TB
    crc_lds_init(S, s.tbp, -1);
    const int pp[1] = {s.tbp};
    uint32_t c[1];
    wg_crc_mem<1>(trblk + (int64_t)blockIdx.x * lda, nullptr, s.A, blockIdx.y, pp, S, c);
    if (threadIdx.x == 0 && c[0]) atomicXor(&tbcrc[blockIdx.x], c[0]);
}

// codeblock segmentation + CRC24B (nr_ldpc_cbsegment.py:24-32): codeblock (t, c) -> ck row
// t*C + c: cbz bits of (TB || TB CRC), its CRC24B when C > 1, fillers -1 up to K.  The TB bits
// are copied by the CRC pass itself; the TB CRC bits that end the last codeblock are folded in
// by linearity, crc(M1 || M2) = crc(M1) x^|M2| + crc(M2).
__global__ __launch_bounds__(kCrcNT) void cbseg_kernel(const int8_t* __restrict__ trblk, int64_t lda,
                                                       const uint32_t* __restrict__ tbcrc, SchDev s0,
                                                       const SchGeo* __restrict__ gv,
                                                       const RowRef* __restrict__ rm,
                                                       int8_t* __restrict__ ck) {
    __shared__ CrcLds S;
    __shared__ uint32_t cbcrc;
    crc_lds_init(S, LDPC5G_CRC24B, -1);
    const RowGeo rg = row_geo(blockIdx.x, s0, gv, rm, 0);
    const SchDev& s = rg.s;
    const int t = rg.t, c = rg.c;
    const uint32_t tc = tbcrc[t];
    const int64_t base = (int64_t)c * s.cbz;
    const int nm = (int)min((int64_t)s.cbz, (int64_t)s.A - base);   // TB bits in this codeblock
    const int nt = s.cbz - nm;                                       // TB CRC bits after them
    int8_t* out = ck + rg.ck_row;
    const int pp[1] = {LDPC5G_CRC24B};
    uint32_t v[1];
    wg_crc_mem<1>(trblk + (int64_t)t * lda + base, out, nm, 0, pp, S, v);
    if (threadIdx.x == 0) {
        const uint32_t g = kCrcPoly[LDPC5G_CRC24B].g;
        const uint32_t tail = nt ? tc >> (s.Ltb - nt) : 0u;
        cbcrc = crc_mulmod(v[0], crc_xpow(nt, LDPC5G_CRC24B), 24, g) ^ crc_bits_msb(0u, tail, nt, 24, g);
    }
    __syncthreads();
    const uint32_t cb = cbcrc;
    for (int j = nm + threadIdx.x; j < s.K; j += kCrcNT) {
        int8_t b = -1;
        if (j < s.cbz) b = (int8_t)((tc >> (s.Ltb - 1 - (j - nm))) & 1u);
        else if (j < s.K_apo) b = (int8_t)((cb >> (23 - (j - s.cbz))) & 1u);
        out[j] = b;
    }
}

// rate matching (nr_ldpc_ratematch.py:64-97): bit selection from k0 skipping fillers, then the
// Qm-row interleaver, written at the codeblock's offset in g (code block concatenation).  One
// thread per interleaver column i < E/Qm: it writes the Qm consecutive output bits e = i Qm + q,
// read from the selected-bit stream at k = q E/Qm + i, so for every q a wave reads consecutive
// bytes of dn and writes 64 Qm consecutive bytes of g.
__global__ __launch_bounds__(256) void ratematch_kernel(const int8_t* __restrict__ dn, SchDev s0,
                                                        const SchGeo* __restrict__ gv,
                                                        const RowRef* __restrict__ rm,
                                                        int8_t* __restrict__ g, int64_t ldg) {
    const RowGeo rg = row_geo(blockIdx.x, s0, gv, rm, 0);
    const SchDev& s = rg.s;
    const int t = rg.t, c = rg.c;
    const int E = cb_E(s, c), EQ = E / s.Qm;
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (i >= EQ) return;
    const int8_t* src = dn + rg.dn_row;
    int8_t* dst = g + (int64_t)t * ldg + cb_goff(s, c) + (int64_t)i * s.Qm;
    const uint32_t size = (uint32_t)s.size, step = (uint32_t)(EQ % s.size);
    uint32_t idx = (uint32_t)(((int64_t)s.start + i) % s.size);   // circular-buffer index of k = i
    if (s.Qm == 8 && ((uintptr_t)dst & 7) == 0) {
        uint64_t w = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int pos = (int)idx < s.f0 ? (int)idx : (int)idx + s.Fin;
            w |= (uint64_t)(uint8_t)src[pos] << (8 * q);
            idx += step;
            if (idx >= size) idx -= size;
        }
        *reinterpret_cast<uint64_t*>(dst) = w;
        return;
    }
    for (int q = 0; q < s.Qm; ++q) {
        const int pos = (int)idx < s.f0 ? (int)idx : (int)idx + s.Fin;
        dst[q] = src[pos];
        idx += step;
        if (idx >= size) idx -= size;
    }
}

// -------------------------------------------------------------------------------- receive
constexpr int kRrNT = 512;
// interleaver rows per thread per round in the no-repetition pass (loads in flight together;
// r05 config 4: 1 / 2 / 4 -> 0.0621 / 0.0625 / 0.0646 ms)
#ifndef LDPC5G_RR_RU
#define LDPC5G_RR_RU 1
#endif
// the E LLRs of a codeblock are staged in LDS up to this size (4 x 512-thread workgroups per CU)
constexpr int kRrStageBytes = 40 * 1024;

template <typename Tin>
__device__ __forceinline__ double ld64(const Tin* p, int64_t i) { return (double)p[i]; }

// rate recovery (nr_ldpc_raterecover.py:25-64) of codeblock (t, c) + HARQ combining
// (nr_dlsch_decode.py:73-88).  Arithmetic in float64, as the reference: a position visited cnt
// times holds (0.0 + v_0 + ... + v_{cnt-1}) / cnt (the row-by-row numpy sum of tmp_buf);
// unvisited positions 0; fillers 10 * max|LLR| of the codeblock.  A float32 output is the
// float64 result rounded once.
// STAGE: the codeblock's E input LLRs are first copied into LDS in de-interleaved order
// (lds[q*EQ + r] = llr[r*Qm + q], i.e. lds[k] is the k-th bit of the interleaver's column read-out),
// in the same pass as the max|LLR| reduction: the input is read once, coalesced, and the gather
// below reads LDS at consecutive k instead of global memory at stride Qm.  A row whose E is too
// large for the stage gathers from global memory (decided per row).  Rows visited at most twice
// per position (E <= 2 size; the k-major passes below) take neither.  Outputs of the gather:
// 4 consecutive positions per thread, stored as 16-B pieces when the row is 16-B aligned.
template <typename Tin, typename Tout, bool STAGE>
__global__ __launch_bounds__(kRrNT) void raterecover_kernel(const Tin* __restrict__ llr, int64_t ldg,
                                                            SchDev s0, const SchGeo* __restrict__ gv,
                                                            const RowRef* __restrict__ rm,
                                                            const Tout* __restrict__ harq,
                                                            Tout* __restrict__ out) {
    __shared__ double red[kRrNT / 64];
    extern __shared__ __align__(16) unsigned char rr_smem[];
    Tin* lk = (Tin*)rr_smem;
    const RowGeo rg = row_geo(blockIdx.x, s0, gv, rm, 0);
    const SchDev& s = rg.s;
    const int t = rg.t, c = rg.c;
    const int E = cb_E(s, c), EQ = E / s.Qm;
    const Tin* fe = llr + (int64_t)t * ldg + cb_goff(s, c);
    const int64_t row = rg.dn_row;
    Tout* orow = out + row;
    auto combine = [&](double v, int p) -> double {   // HARQ (nr_dlsch_decode.py:73-88)
        if (harq) {
            const double h = (double)harq[row + p];
            v = (v == 0.0 || h == 0.0) ? v + h : (v + h) / 2.0;
        }
        return v;
    };
    double m = 0.0;
    // k-major rows: bit k of the column read-out (k = q*EQ + r) is LLR r*Qm + q and lands at the
    // position of rank k mod size in the circular order from k0.  A thread per r reads its Qm
    // consecutive LLRs (pairs: 8- or 16-B loads when Qm is even and the row aligned) and handles
    // them plane by plane: consecutive r -> consecutive positions, so reads and writes coalesce.
    // Rows visited at most twice per position (E <= 2 size) take this form when a first visit's
    // LLR survives a round trip through the output row exactly (float input or double output):
    // pass 1 writes every k < size — final (0.0 + x) / 1 for ranks visited once, the raw LLR for
    // ranks visited twice — and after a barrier pass 2 combines each k >= size with it as
    // (0.0 + x0 + x1) / 2, the reference's float64 sum of the two tmp_buf rows (:53-58).
    // ranks [0, E2) are visited twice.  Pass 1 parks the first visit's LLR in the output row, so
    // when the HARQ input IS the output row (in-place combining with the previous llr_dn) pass 2
    // would read that LLR instead of the previous value: such rows take the gather below, which
    // reads harq[p] and writes out[p] in one thread.
    const int E2 = E - s.size;
    const bool kmaj = E <= s.size || (sizeof(Tout) >= sizeof(Tin) && E <= 2 * s.size &&
                                      (const void*)harq != (const void*)out);
    auto pos = [&](int rank) {   // rank in [0, size) -> position in the row
        int pp = rank + s.start;   // in the filler-free index space
        if (pp >= s.size) pp -= s.size;
        return pp < s.f0 ? pp : pp + s.Fin;
    };
    auto kmajor = [&](auto&& visit) {
        const bool pairs = (s.Qm & 1) == 0 && ((uintptr_t)fe & (2 * sizeof(Tin) - 1)) == 0;
        // RU interleaver rows per thread per round, all their loads in flight before any use;
        // H = Qm / 2 pairs per row, a compile-time constant per instantiation
        auto rounds = [&](auto hc) {
            constexpr int H = decltype(hc)::value, RU = LDPC5G_RR_RU;
            using V2 = Tin __attribute__((ext_vector_type(2)));
            for (int r0 = threadIdx.x; r0 < EQ; r0 += RU * kRrNT) {
                V2 x[RU][H];
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    const int r = min(r0 + u * kRrNT, EQ - 1);   // clamped: a duplicate load, no use
                    const V2* src = (const V2*)(fe + (int64_t)r * (2 * H));
#pragma unroll
                    for (int q = 0; q < H; ++q) x[u][q] = src[q];
                }
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    const int r = r0 + u * kRrNT;
                    if (r < EQ) {
#pragma unroll
                        for (int q = 0; q < H; ++q)
                            visit(2 * q * EQ + r, (double)x[u][q][0]), visit((2 * q + 1) * EQ + r, (double)x[u][q][1]);
                    }
                }
            }
        };
        if (pairs && s.Qm == 2) {
            rounds(std::integral_constant<int, 1>{});
        } else if (pairs && s.Qm == 4) {
            rounds(std::integral_constant<int, 2>{});
        } else if (pairs && s.Qm == 6) {
            rounds(std::integral_constant<int, 3>{});
        } else if (pairs && s.Qm == 8) {
            rounds(std::integral_constant<int, 4>{});
        } else if (pairs && s.Qm == 10) {
            rounds(std::integral_constant<int, 5>{});
        } else {
            for (int r = threadIdx.x; r < EQ; r += kRrNT) {
                const Tin* src = fe + (int64_t)r * s.Qm;
                for (int q = 0; q < s.Qm; ++q) visit(q * EQ + r, (double)src[q]);
            }
        }
    };
    if (kmaj) {
        kmajor([&](int k, double x) {
            m = fmax(m, fabs(x));
            if (k < s.size) {
                const int p = pos(k);
                orow[p] = k < E2 ? (Tout)x : (Tout)combine(0.0 + x, p);
            }
        });
        if (E2 > 0) {
            __syncthreads();   // every first visit is in the row
            kmajor([&](int k, double x) {
                if (k >= s.size) {
                    const int p = pos(k - s.size);
                    const double x0 = (double)orow[p];
                    orow[p] = (Tout)combine((0.0 + x0 + x) / 2.0, p);
                }
            });
        }
    } else if (STAGE && E * (int)sizeof(Tin) <= kRrStageBytes) {   // per row: this row fits
        for (int r = threadIdx.x; r < EQ; r += kRrNT) {
            const Tin* src = fe + (int64_t)r * s.Qm;
            for (int q = 0; q < s.Qm; ++q) {
                const Tin x = src[q];
                lk[q * EQ + r] = x;
                m = fmax(m, fabs((double)x));
            }
        }
    } else {
        for (int e = threadIdx.x; e < E; e += kRrNT) m = fmax(m, fabs(ld64(fe, e)));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int w = 1; w < kRrNT / 64; ++w) m = fmax(m, red[w]);
    const double mx = m * 10.0;
    const int qE = E / s.size, rE = E - qE * s.size;   // visits of rank rr: qE + (rr < rE)
    const bool stg = STAGE && E * (int)sizeof(Tin) <= kRrStageBytes;
    if (kmaj) {
        // the positions the read-out did not reach, disjoint from those written above: the
        // unvisited ranks [E, size) (0; none when E > size), the fillers (10 * max|LLR|) and the
        // tail past Ncb (0), each a range walked directly (+ HARQ)
        for (int u = threadIdx.x; u < s.size - E; u += kRrNT) {
            const int p = pos(E + u);
            orow[p] = (Tout)combine(0.0, p);
        }
        for (int p = s.f0 + (int)threadIdx.x; p < s.f0 + s.F; p += kRrNT) orow[p] = (Tout)combine(mx, p);
        for (int p = s.Ncb + (int)threadIdx.x; p < s.N; p += kRrNT)
            if (p < s.f0 || p >= s.f0 + s.F) orow[p] = (Tout)combine(0.0, p);
        return;
    }
    // k -> (k mod EQ, k / EQ) without a divide: a multiply-high estimate and at most two corrections
    const uint32_t dq = (uint32_t)EQ, mq = 0xffffffffu / dq;
    auto divq = [&](uint32_t k, uint32_t& rem) -> uint32_t {
        uint32_t q = __umulhi(k, mq), r = k - q * dq;
        while (r >= dq) ++q, r -= dq;
        rem = r;
        return q;
    };
    auto value = [&](int p) -> double {
        double v = 0.0;
        if (p >= s.f0 && p < s.f0 + s.F) {
            v = mx;
        } else if (p < s.Ncb) {
            int rr = (p < s.f0 ? p : p - s.Fin) - s.start;
            if (rr < 0) rr += s.size;
            if (rr < E) {
                const int cnt = qE + (rr < rE ? 1 : 0);   // = (E - 1 - rr) / size + 1
                double acc = 0.0;
                for (int j = 0; j < cnt; ++j) {
                    const int k = rr + j * s.size;
                    if (STAGE && stg) {
                        acc += (double)lk[k];
                    } else {
                        uint32_t kr;
                        const uint32_t kq = divq((uint32_t)k, kr);
                        acc += ld64(fe, (int64_t)kr * s.Qm + kq);
                    }
                }
                v = cnt == 1 ? acc : acc / (double)cnt;   // x / 1.0 == x: skip the f64 divide
            }
        }
        return combine(v, p);
    };
    const bool vec = ((uintptr_t)orow & 15) == 0;
    for (int p0 = 4 * (int)threadIdx.x; p0 < s.N; p0 += 4 * kRrNT) {
        Tout v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = p0 + q < s.N ? (Tout)value(p0 + q) : Tout(0);
        if (vec && p0 + 4 <= s.N) {
            if constexpr (sizeof(Tout) == 4) {
                using f4 = float __attribute__((ext_vector_type(4)));
                *(f4*)(orow + p0) = f4{v[0], v[1], v[2], v[3]};
            } else {
                using d2 = double __attribute__((ext_vector_type(2)));
                *(d2*)(orow + p0) = d2{v[0], v[1]};
                *(d2*)(orow + p0 + 2) = d2{v[2], v[3]};
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (p0 + q < s.N) orow[p0 + q] = v[q];
        }
    }
}

// TB reassembly + checks (nr_dlsch_decode.py:93-106) for codeblock (t, c), one pass over
// ck[0:cbz]: the TB CRC share crc(seg) * x^((C-1-c) cbz), XORed into tbrem[t]; CRC24B over
// ck[0:K_apo] when C > 1 (cb_ok = remainder 0) as crc24B(ck[0:cbz]) x^24 + crc24B(ck[cbz:K_apo]);
// and the copy of ck[0:cbz] to the TB bits.
__global__ __launch_bounds__(kCrcNT) void tb_check_kernel(const int8_t* __restrict__ ck, int64_t ldc,
                                                          SchDev s0, const SchGeo* __restrict__ gv,
                                                          const RowRef* __restrict__ rm,
                                                          int8_t* __restrict__ tbblk,
                                                          int64_t ldb, uint8_t* __restrict__ cb_ok,
                                                          uint32_t* tbrem) {
    __shared__ CrcLds S;
    __shared__ uint32_t tb_dist;
    const RowGeo rg = row_geo(blockIdx.x, s0, gv, rm, ldc);
    const SchDev& s = rg.s;
    const int t = rg.t, c = rg.c;
    crc_lds_init(S, s.tbp, LDPC5G_CRC24B);
    // the TB share's distance x^((C-1-c) cbz) mod g (up to ~20 serial mulmods): the last thread
    // forms it while the others load the codeblock (its wave holds no word when cbz <= 12288 bits),
    // not thread 0 after the pass; wg_crc_mem's closing barrier publishes it
    if (threadIdx.x == kCrcNT - 1) tb_dist = crc_xpow((int64_t)(s.C - 1 - c) * s.cbz, s.tbp);
    const int8_t* row = ck + rg.dck_row;
    const int pp[2] = {s.tbp, LDPC5G_CRC24B};
    uint32_t v[2];
    wg_crc_mem<2>(row, tbblk + (int64_t)t * ldb + (int64_t)c * s.cbz, s.cbz, 0, pp, S, v);
    if (threadIdx.x == 0) {
        uint32_t cbr = 0;
        if (s.C > 1) {
            const uint32_t g = kCrcPoly[LDPC5G_CRC24B].g;
            uint32_t tail = 0;
            for (int j = 0; j < 24; ++j) tail = (tail << 1) | (uint32_t)(row[s.cbz + j] & 1);
            cbr = crc_mulmod(v[1], crc_xpow(24, LDPC5G_CRC24B), 24, g) ^ crc_bits_msb(0u, tail, 24, 24, g);
        }
        cb_ok[rg.cbi] = cbr == 0u;
        const uint32_t tbc = crc_mulmod(v[0], tb_dist, s.Ltb, kCrcPoly[s.tbp].g);
        if (tbc) atomicXor(&tbrem[t], tbc);
    }
}

__global__ void tb_ok_kernel(const uint32_t* __restrict__ tbrem, uint8_t* __restrict__ ok, int T) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) ok[t] = tbrem[t] == 0u;
}

// ============================================================================ host helpers
// cfg -> validated device geometry
int sch_dev(const ldpc5g_sch_cfg_t* c, SchDev* s) {
    if (!c) return fail(LDPC5G_ESIZE, "null cfg");
    memset(s, 0, sizeof *s);
    s->A = c->A, s->B = c->B, s->tbp = c->tb_crc_poly, s->bgn = c->bgn, s->C = c->C, s->cbz = c->cbz;
    s->Lcb = c->Lcb, s->K = c->K, s->K_apo = c->K_apo, s->Zc = c->Zc, s->N = c->N, s->Ncb = c->Ncb;
    s->Qm = c->Qm, s->E_lo = c->E_lo, s->E_hi = c->E_hi, s->c_switch = c->c_switch, s->G = c->G;
    if (s->tbp != LDPC5G_CRC24A && s->tbp != LDPC5G_CRC16) return fail(LDPC5G_ESIZE, "cfg: bad TB CRC");
    s->Ltb = kCrcPoly[s->tbp].L;
    if (c->bgn != 1 && c->bgn != 2) return fail(LDPC5G_EBGN, "cfg: bgn=%d", c->bgn);
    if (zc_index(c->Zc) < 0) return fail(LDPC5G_EZC, "cfg: Zc=%d", c->Zc);
    if (c->K != (c->bgn == 1 ? 22 : 10) * c->Zc || c->N != (c->bgn == 1 ? 66 : 50) * c->Zc)
        return fail(LDPC5G_ESIZE, "cfg: K/N inconsistent with (bgn, Zc)");
    if (c->C < 1 || (int64_t)c->cbz * c->C != c->B || c->K_apo != c->cbz + c->Lcb || c->K_apo > c->K ||
        (c->C > 1) != (c->Lcb == 24) || c->Ncb < 1 || c->Ncb > c->N || c->A < 1 || c->B <= c->A)
        return fail(LDPC5G_ESIZE, "cfg: inconsistent segmentation");
    if (c->Qm < 1 || c->E_lo < 0 || c->E_hi < c->E_lo || c->E_lo % c->Qm || c->E_hi % c->Qm ||
        c->c_switch < 0 || c->c_switch > c->C || c->k0 < 0 || c->k0 >= c->Ncb)
        return fail(LDPC5G_ESIZE, "cfg: inconsistent rate matching");
    s->f0 = c->K_apo - 2 * c->Zc;
    s->F = c->K - c->K_apo;
    if (s->f0 < 0) return fail(LDPC5G_ESIZE, "cfg: fillers before 2Zc");
    s->Fin = s->f0 < c->Ncb ? std::min(s->f0 + s->F, c->Ncb) - s->f0 : 0;
    s->size = c->Ncb - s->Fin;
    if (s->size < 1) return fail(LDPC5G_ESIZE, "cfg: empty circular buffer");
    const int k0 = c->k0;
    s->start = k0 < s->f0 ? k0 : (k0 < s->f0 + s->Fin ? s->f0 : k0 - s->Fin);
    return LDPC5G_OK;
}

int64_t sch_total_E(const SchDev& s) {
    return (int64_t)s.c_switch * s.E_lo + (int64_t)(s.C - s.c_switch) * s.E_hi;
}


template <typename Tin, typename Tout>
void raterecover_go(dim3 grid, const void* llr, int64_t ldg, const SchDev& s, const SchGeo* gv,
                    const RowRef* rm, const void* harq_in, void* llr_dn, int max_cb_E, hipStream_t st) {
    // rows whose E fits the stage use it (decided per row in the kernel): the launch's LDS is the
    // stage size capped by its largest codeblock
    const size_t lds = std::min((size_t)max_cb_E * sizeof(Tin), (size_t)kRrStageBytes);
    hipLaunchKernelGGL((raterecover_kernel<Tin, Tout, true>), grid, dim3(kRrNT), lds, st, (const Tin*)llr, ldg, s,
                       gv, rm, (const Tout*)harq_in, (Tout*)llr_dn);
}

// max_cb_E: the largest per-codeblock E of the launch (sizes the LDS stage)
int launch_raterecover(dim3 grid, const void* llr, int llr_dtype, int64_t ldg, const SchDev& s,
                       const SchGeo* gv, const RowRef* rm, const void* harq_in, void* llr_dn,
                       int dn_dtype, int max_cb_E, hipStream_t st) {
    if (llr_dtype == LDPC5G_F32 && dn_dtype == LDPC5G_F32)
        raterecover_go<float, float>(grid, llr, ldg, s, gv, rm, harq_in, llr_dn, max_cb_E, st);
    else if (llr_dtype == LDPC5G_F32)
        raterecover_go<float, double>(grid, llr, ldg, s, gv, rm, harq_in, llr_dn, max_cb_E, st);
    else if (dn_dtype == LDPC5G_F32)
        raterecover_go<double, float>(grid, llr, ldg, s, gv, rm, harq_in, llr_dn, max_cb_E, st);
    else
        raterecover_go<double, double>(grid, llr, ldg, s, gv, rm, harq_in, llr_dn, max_cb_E, st);
    return check_hip(hipGetLastError(), "raterecover launch");
}

// Host side of a multi-configuration batch: validated per-TB geometry (workspace offsets in TB
// order), the row map, and the device copy of both in a stream-ordered allocation (freed in
// stream order by release(); asynchronous and reentrant like the mixed-Zc decode).
struct SchMulti {
    std::vector<SchGeo> geo;
    std::vector<RowRef> rows;
    int64_t ck_elems = 0, dn_elems = 0, dck_elems = 0, max_E = 0;
    int max_A = 0, max_B = 0, max_EQ = 0;
    void* dev = nullptr;
    hipStream_t st = nullptr;

    int build(const ldpc5g_sch_cfg_t* cfgs, int T) {
        if (T < 0 || (T > 0 && !cfgs)) return fail(LDPC5G_ESIZE, "bad multi batch T=%d", T);
        geo.resize(T);
        for (int t = 0; t < T; ++t) {
            SchGeo& G = geo[t];
            memset(&G, 0, sizeof G);
            if (int rc = sch_dev(&cfgs[t], &G.s)) return fail(rc, "cfgs[%d]: %s", t, err_text());
            const int Nf = (G.s.bgn == 1 ? 68 : 52) * G.s.Zc;
            G.ck_off = ck_elems, G.dn_off = dn_elems, G.dck_off = dck_elems;
            G.cb_off = (int32_t)rows.size(), G.dck_ld = Nf;
            for (int c = 0; c < G.s.C; ++c) rows.push_back(RowRef{t, c});
            ck_elems += (int64_t)G.s.C * G.s.K, dn_elems += (int64_t)G.s.C * G.s.N;
            dck_elems += (int64_t)G.s.C * Nf;
            max_A = std::max(max_A, G.s.A), max_B = std::max(max_B, G.s.B);
            max_E = std::max(max_E, sch_total_E(G.s));
            max_EQ = std::max(max_EQ, G.s.E_hi / G.s.Qm);
        }
        return LDPC5G_OK;
    }
    int upload(hipStream_t s) {
        st = s;
        const size_t gb = geo.size() * sizeof(SchGeo), rb = rows.size() * sizeof(RowRef);
        std::vector<unsigned char> host(gb + rb);
        memcpy(host.data(), geo.data(), gb);
        memcpy(host.data() + gb, rows.data(), rb);
        if (int rc = check_hip(hipMallocAsync(&dev, gb + rb, st), "hipMallocAsync(sch plan)")) return rc;
        return stage_h2d(dev, host.data(), gb + rb, st);   // pinned staging slot (ldpc5g_capi.hip)
    }
    const SchGeo* dgeo() const { return (const SchGeo*)dev; }
    const RowRef* drows() const { return (const RowRef*)((const unsigned char*)dev + geo.size() * sizeof(SchGeo)); }
    int release() {
        if (!dev) return LDPC5G_OK;
        const int rc = check_hip(hipFreeAsync(dev, st), "hipFreeAsync(sch plan)");
        dev = nullptr;
        return rc;
    }
    ~SchMulti() { release(); }
};

}  // namespace
}  // namespace ldpc5g_impl

using namespace ldpc5g_impl;

extern "C" {

int ldpc5g_crc(const int8_t* bits, int64_t ld, int64_t nbits, int32_t rows, int32_t poly,
               uint32_t* rem, void* stream) {
    clear_error();
    if (poly < 0 || poly > 5) return fail(LDPC5G_ESIZE, "bad CRC polynomial id %d", poly);
    if (rows < 0 || nbits < 0 || (rows > 1 && ld < nbits)) return fail(LDPC5G_ESIZE, "bad sizes");
    if (rows == 0) return LDPC5G_OK;
    if (!rem || (nbits > 0 && !bits)) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = check_hip(hipMemsetAsync(rem, 0, (size_t)rows * 4, st), "hipMemsetAsync")) return rc;
    if (nbits == 0) return LDPC5G_OK;
    hipLaunchKernelGGL(crc_rows_kernel, dim3(rows, (unsigned)crc_chunks(nbits)), dim3(kCrcNT), 0, st,
                       bits, ld, nbits, (int)poly, rem);
    return check_hip(hipGetLastError(), "crc_rows_kernel launch");
}

int ldpc5g_sch_config(int32_t A, int32_t Qm, double coderateby1024, int32_t NL, int32_t rv,
                      int64_t TBS_LBRM, int64_t G, ldpc5g_sch_cfg_t* c) {
    clear_error();
    if (!c) return fail(LDPC5G_ESIZE, "null cfg");
    memset(c, 0, sizeof *c);
    if (A < 1 || Qm < 1 || Qm > 10 || NL < 1 || G < 1 || TBS_LBRM < 0)
        return fail(LDPC5G_ESIZE, "bad SCH parameters A=%d Qm=%d NL=%d G=%lld", A, Qm, NL, (long long)G);
    if (rv < 0 || rv > 3) return fail(LDPC5G_ESIZE, "rv=%d not in [0,3] (nr_ldpc_ratematch.py:46)", rv);
    // TB CRC (nr_dlsch.py:34-40) and base graph selection (:44-49)
    c->A = A;
    c->B = A > 3824 ? A + 24 : A + 16;
    c->tb_crc_poly = A > 3824 ? LDPC5G_CRC24A : LDPC5G_CRC16;
    const double R = coderateby1024;
    c->bgn = (A <= 292 || (A <= 3824 && R <= 0.67 * 1024) || R <= 0.25 * 1024) ? 2 : 1;
    // get_cbs_info (ldpc_info.py:5-78)
    const int B = c->B, Kcb = c->bgn == 1 ? 8448 : 3840;
    int C, L, Bd;
    if (B <= Kcb) {
        L = 0, C = 1, Bd = B;
    } else {
        L = 24;
        C = (int)ceil((double)B / (double)(Kcb - L));
        Bd = B + C * L;
    }
    if (B % C || Bd % C) return fail(LDPC5G_ESIZE, "B=%d does not split into %d codeblocks", B, C);
    const int cbz = B / C, Kd = Bd / C;
    int Kb = 22;
    if (c->bgn == 2) Kb = B > 640 ? 10 : B > 560 ? 9 : B > 192 ? 8 : 6;
    int Zc = -1;
    for (int zi = 0; zi < LDPC5G_NUM_ZC; ++zi)   // ascending
        if (kLdpcZcList[zi] * Kb >= Kd) {
            Zc = kLdpcZcList[zi];
            break;
        }
    if (Zc < 0) return fail(LDPC5G_ESIZE, "no lifting size for K'=%d", Kd);
    c->C = C, c->cbz = cbz, c->Lcb = L, c->Zc = Zc;
    c->K = (c->bgn == 1 ? 22 : 10) * Zc;
    c->F = c->K - Kd;
    c->K_apo = cbz + L;
    c->N = (c->bgn == 1 ? 66 : 50) * Zc;
    // Ncb (nr_dlsch.py:63-65: I_LBRM = 1 with TBS_LBRM; nr_ulsch.py:55-58: Ncb = N when 0)
    int64_t Ncb = c->N;
    if (TBS_LBRM > 0) {
        const double nref = floor((double)TBS_LBRM / ((double)(C * 2) / 3.0));
        if (nref < Ncb) Ncb = (int64_t)nref;
    }
    c->Ncb = (int32_t)Ncb;
    // k0 (nr_ldpc_ratematch.py:29-61)
    static const int num1[4] = {0, 17, 33, 56}, num2[4] = {0, 13, 25, 43};
    const int num = c->bgn == 1 ? num1[rv] : num2[rv], den = c->bgn == 1 ? 66 : 50;
    c->k0 = (int32_t)floor((double)((int64_t)num * Ncb) / (double)(den * Zc)) * Zc;
    c->Qm = Qm, c->NL = NL, c->rv = rv, c->G = G;
    // Er (nr_ldpc_ratematch.py:5-27), float arithmetic as the reference
    const double gq = (double)G / (double)(NL * Qm);
    c->E_lo = NL * Qm * (int32_t)floor((double)G / (double)(NL * Qm * C));
    c->E_hi = NL * Qm * (int32_t)ceil((double)G / (double)(NL * Qm * C));
    const double thr = (double)C - fmod(gq, (double)C) - 1.0;
    int cs = 0;
    for (int j = 0; j < C; ++j) cs += (double)j <= thr;
    c->c_switch = cs;
    SchDev s;
    if (int rc = sch_dev(c, &s)) return rc;
    c->E_total = sch_total_E(s);
    return LDPC5G_OK;
}

int ldpc5g_sch_segment(const int8_t* trblk, int64_t lda, const ldpc5g_sch_cfg_t* cfg, int32_t T,
                       int8_t* ck, uint32_t* tb_crc, void* stream) {
    clear_error();
    SchDev s;
    if (int rc = sch_dev(cfg, &s)) return rc;
    if (T < 0 || (T > 1 && lda < s.A)) return fail(LDPC5G_ESIZE, "bad sizes T=%d lda=%lld", T, (long long)lda);
    if (T == 0) return LDPC5G_OK;
    if (!trblk || !ck || !tb_crc) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = check_hip(hipMemsetAsync(tb_crc, 0, (size_t)T * 4, st), "hipMemsetAsync")) return rc;
    hipLaunchKernelGGL(tb_crc_kernel, dim3(T, (unsigned)crc_chunks(s.A)), dim3(kCrcNT), 0, st, trblk,
                       lda, s, (const SchGeo*)nullptr, tb_crc);
    hipLaunchKernelGGL(cbseg_kernel, dim3(T * s.C), dim3(kCrcNT), 0, st, trblk, lda,
                       (const uint32_t*)tb_crc, s, (const SchGeo*)nullptr, (const RowRef*)nullptr, ck);
    return check_hip(hipGetLastError(), "segment launch");
}

int ldpc5g_sch_ratematch(const int8_t* ck, const ldpc5g_sch_cfg_t* cfg, int32_t T, int8_t* dn,
                         int8_t* g, int64_t ldg, void* stream) {
    clear_error();
    SchDev s;
    if (int rc = sch_dev(cfg, &s)) return rc;
    if (T < 0 || (T > 1 && ldg < sch_total_E(s))) return fail(LDPC5G_ESIZE, "bad sizes T=%d ldg=%lld", T, (long long)ldg);
    if (T == 0) return LDPC5G_OK;
    if (!ck || !dn || !g) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    const int rows = T * s.C;
    if (int rc = launch_encode(ck, dn, rows, s.bgn, s.Zc, zc_index(s.Zc), s.K, s.N, st)) return rc;
    if (s.E_hi > 0)
        hipLaunchKernelGGL(ratematch_kernel, dim3(rows, (s.E_hi / s.Qm + 255) / 256), dim3(256), 0, st, dn,
                           s, (const SchGeo*)nullptr, (const RowRef*)nullptr, g, ldg);
    return check_hip(hipGetLastError(), "ratematch launch");
}

int ldpc5g_sch_encode(const int8_t* trblk, int64_t lda, int8_t* g, int64_t ldg,
                      const ldpc5g_sch_cfg_t* cfg, int32_t T, int8_t* ck, int8_t* dn,
                      uint32_t* tb_crc, void* stream) {
    if (int rc = ldpc5g_sch_segment(trblk, lda, cfg, T, ck, tb_crc, stream)) return rc;
    return ldpc5g_sch_ratematch(ck, cfg, T, dn, g, ldg, stream);
}

int ldpc5g_sch_raterecover(const void* llr, int32_t llr_dtype, int64_t ldg,
                           const ldpc5g_sch_cfg_t* cfg, int32_t T, const void* harq_in,
                           void* llr_dn, int32_t dn_dtype, void* stream) {
    clear_error();
    SchDev s;
    if (int rc = sch_dev(cfg, &s)) return rc;
    if ((llr_dtype != LDPC5G_F32 && llr_dtype != LDPC5G_F64) || (dn_dtype != LDPC5G_F32 && dn_dtype != LDPC5G_F64))
        return fail(LDPC5G_ESIZE, "bad dtype");
    if (T < 0 || (T > 1 && ldg < sch_total_E(s))) return fail(LDPC5G_ESIZE, "bad sizes T=%d ldg=%lld", T, (long long)ldg);
    if (T == 0) return LDPC5G_OK;
    if (!llr || !llr_dn) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    return launch_raterecover(dim3(T * s.C), llr, llr_dtype, ldg, s, nullptr, nullptr, harq_in, llr_dn, dn_dtype,
                              std::max(s.E_lo, s.E_hi), st);
}

int ldpc5g_sch_tb_check(const int8_t* ck, int64_t ldc, const ldpc5g_sch_cfg_t* cfg, int32_t T,
                        int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok, uint32_t* tb_rem,
                        uint8_t* tb_ok, void* stream) {
    clear_error();
    SchDev s;
    if (int rc = sch_dev(cfg, &s)) return rc;
    if (T < 0 || ldc < s.K_apo || (T > 1 && ldb < s.B))
        return fail(LDPC5G_ESIZE, "bad sizes T=%d ldc=%lld ldb=%lld", T, (long long)ldc, (long long)ldb);
    if (T == 0) return LDPC5G_OK;
    if (!ck || !tbblk || !cb_crc_ok || !tb_rem || !tb_ok) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = check_hip(hipMemsetAsync(tb_rem, 0, (size_t)T * 4, st), "hipMemsetAsync")) return rc;
    hipLaunchKernelGGL(tb_check_kernel, dim3(T * s.C), dim3(kCrcNT), 0, st, ck, ldc, s,
                       (const SchGeo*)nullptr, (const RowRef*)nullptr, tbblk, ldb, cb_crc_ok, tb_rem);
    hipLaunchKernelGGL(tb_ok_kernel, dim3((T + 255) / 256), dim3(256), 0, st, (const uint32_t*)tb_rem,
                       tb_ok, (int)T);
    return check_hip(hipGetLastError(), "tb_check launch");
}

int ldpc5g_sch_decode(const void* llr, int32_t llr_dtype, int64_t ldg, const ldpc5g_sch_cfg_t* cfg,
                      int32_t T, const void* harq_in, void* llr_dn, int32_t dn_dtype, int8_t* ck,
                      uint8_t* status, int32_t* iters, int32_t L, double alpha, double beta,
                      int32_t schedule, int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok,
                      uint32_t* tb_rem, uint8_t* tb_ok, void* stream) {
    if (int rc = ldpc5g_sch_raterecover(llr, llr_dtype, ldg, cfg, T, harq_in, llr_dn, dn_dtype, stream)) return rc;
    if (T == 0) return LDPC5G_OK;
    const int Nf = (cfg->bgn == 1 ? 68 : 52) * cfg->Zc;
    if (int rc = ldpc5g_decode_ms(llr_dn, dn_dtype, ck, status, iters, T * cfg->C, cfg->bgn, cfg->Zc, L,
                                  alpha, beta, schedule, LDPC5G_RATE_MATCHED, cfg->N, Nf, stream))
        return rc;
    return ldpc5g_sch_tb_check(ck, Nf, cfg, T, tbblk, ldb, cb_crc_ok, tb_rem, tb_ok, stream);
}

int ldpc5g_sch_multi_sizes(const ldpc5g_sch_cfg_t* cfgs, int32_t T, int64_t* sizes) {
    clear_error();
    if (!sizes) return fail(LDPC5G_ESIZE, "null sizes");
    SchMulti m;
    if (int rc = m.build(cfgs, T)) return rc;
    sizes[0] = m.ck_elems, sizes[1] = m.dn_elems, sizes[2] = m.dck_elems, sizes[3] = (int64_t)m.rows.size();
    sizes[4] = m.max_A, sizes[5] = m.max_B, sizes[6] = m.max_E;
    return LDPC5G_OK;
}

int ldpc5g_sch_encode_multi(const int8_t* trblk, int64_t lda, int8_t* g, int64_t ldg,
                            const ldpc5g_sch_cfg_t* cfgs, int32_t T, int8_t* ck, int8_t* dn,
                            uint32_t* tb_crc, void* stream) {
    clear_error();
    SchMulti m;
    if (int rc = m.build(cfgs, T)) return rc;
    if (T > 1 && (lda < m.max_A || ldg < m.max_E))
        return fail(LDPC5G_ESIZE, "bad strides lda=%lld ldg=%lld (max A %d, max E %lld)", (long long)lda, (long long)ldg, m.max_A, (long long)m.max_E);
    if (T == 0) return LDPC5G_OK;
    if (!trblk || !g || !ck || !dn || !tb_crc) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = m.upload(st)) return rc;
    const SchDev s0{};
    const int rows = (int)m.rows.size();
    if (int rc = check_hip(hipMemsetAsync(tb_crc, 0, (size_t)T * 4, st), "hipMemsetAsync")) return rc;
    hipLaunchKernelGGL(tb_crc_kernel, dim3(T, (unsigned)crc_chunks(m.max_A)), dim3(kCrcNT), 0, st, trblk,
                       lda, s0, m.dgeo(), tb_crc);
    hipLaunchKernelGGL(cbseg_kernel, dim3(rows), dim3(kCrcNT), 0, st, trblk, lda, (const uint32_t*)tb_crc,
                       s0, m.dgeo(), m.drows(), ck);
    if (int rc = check_hip(hipGetLastError(), "segment launch")) return rc;
    // encoder: one launch per run of consecutive TBs with the same (bgn, Zc) (their rows are
    // contiguous with one stride)
    for (int t0 = 0; t0 < T;) {
        const SchDev& a = m.geo[t0].s;
        int t1 = t0 + 1, n = a.C;
        while (t1 < T && m.geo[t1].s.bgn == a.bgn && m.geo[t1].s.Zc == a.Zc) n += m.geo[t1++].s.C;
        if (int rc = launch_encode(ck + m.geo[t0].ck_off, dn + m.geo[t0].dn_off, n, a.bgn, a.Zc,
                                   zc_index(a.Zc), a.K, a.N, st))
            return rc;
        t0 = t1;
    }
    if (m.max_EQ > 0)
        hipLaunchKernelGGL(ratematch_kernel, dim3(rows, (m.max_EQ + 255) / 256), dim3(256), 0, st, dn, s0,
                           m.dgeo(), m.drows(), g, ldg);
    if (int rc = check_hip(hipGetLastError(), "ratematch launch")) return rc;
    return m.release();
}

}  // extern "C"

namespace ldpc5g_impl {
namespace {
// Reusable multi-configuration rate-recovery plan (host bytes, copied verbatim to the device):
//   SchPlanHdr | SchGeo[T] | RowRef[rows]
struct SchPlanHdr {
    int32_t magic, T, rows, max_cb_E;
    int64_t max_E, dn_elems;
};
constexpr int32_t kSchPlanMagic = 0x4c505253;   // "SRPL"
}  // namespace
}  // namespace ldpc5g_impl

extern "C" {

int64_t ldpc5g_sch_multi_plan(const ldpc5g_sch_cfg_t* cfgs, int32_t T, void* plan, int64_t plan_bytes) {
    clear_error();
    SchMulti m;
    if (int rc = m.build(cfgs, T)) return rc;
    const int64_t gb = (int64_t)m.geo.size() * (int64_t)sizeof(SchGeo), rb = (int64_t)m.rows.size() * (int64_t)sizeof(RowRef);
    const int64_t need = (int64_t)sizeof(SchPlanHdr) + gb + rb;
    if (!plan || plan_bytes < need) return need;
    SchPlanHdr h{kSchPlanMagic, T, (int32_t)m.rows.size(), 0, m.max_E, m.dn_elems};
    for (const SchGeo& g : m.geo) h.max_cb_E = std::max(h.max_cb_E, std::max(g.s.E_lo, g.s.E_hi));
    // rows largest first (E + N elements moved): a row is one workgroup, and a launch whose big rows
    // come last ends on a tail of a few busy CUs (row order does not change any output)
    std::stable_sort(m.rows.begin(), m.rows.end(), [&](const RowRef& a, const RowRef& b) {
        auto work = [&](const RowRef& r) {
            const SchDev& d = m.geo[r.t].s;
            return (int64_t)(r.c < d.c_switch ? d.E_lo : d.E_hi) + d.N;
        };
        return work(a) > work(b);
    });
    unsigned char* p = (unsigned char*)plan;
    memcpy(p, &h, sizeof h);
    memcpy(p + sizeof h, m.geo.data(), (size_t)gb);
    memcpy(p + sizeof h + gb, m.rows.data(), (size_t)rb);
    return need;
}

int ldpc5g_sch_raterecover_multi_plan(const void* plan_dev, const void* plan_host, const void* llr,
                                      int32_t llr_dtype, int64_t ldg, const void* harq_in, void* llr_dn,
                                      int32_t dn_dtype, void* stream) {
    clear_error();
    if (!plan_dev || !plan_host) return fail(LDPC5G_ESIZE, "null plan");
    SchPlanHdr h;
    memcpy(&h, plan_host, sizeof h);
    if (h.magic != kSchPlanMagic) return fail(LDPC5G_ESIZE, "not a rate-recovery plan (ldpc5g_sch_multi_plan)");
    if ((llr_dtype != LDPC5G_F32 && llr_dtype != LDPC5G_F64) || (dn_dtype != LDPC5G_F32 && dn_dtype != LDPC5G_F64))
        return fail(LDPC5G_ESIZE, "bad dtype");
    if (h.T > 1 && ldg < h.max_E) return fail(LDPC5G_ESIZE, "bad stride ldg=%lld (max E %lld)", (long long)ldg, (long long)h.max_E);
    if (h.rows == 0) return LDPC5G_OK;
    if (!llr || !llr_dn) return fail(LDPC5G_ESIZE, "null buffer");
    const SchGeo* g = (const SchGeo*)((const unsigned char*)plan_dev + sizeof(SchPlanHdr));
    const RowRef* r = (const RowRef*)(g + h.T);
    const SchDev s0{};
    return launch_raterecover(dim3((unsigned)h.rows), llr, llr_dtype, ldg, s0, g, r, harq_in, llr_dn, dn_dtype,
                              h.max_cb_E, (hipStream_t)stream);
}

int ldpc5g_sch_raterecover_multi(const void* llr, int32_t llr_dtype, int64_t ldg,
                                 const ldpc5g_sch_cfg_t* cfgs, int32_t T, const void* harq_in,
                                 void* llr_dn, int32_t dn_dtype, void* stream) {
    clear_error();
    SchMulti m;
    if (int rc = m.build(cfgs, T)) return rc;
    if ((llr_dtype != LDPC5G_F32 && llr_dtype != LDPC5G_F64) || (dn_dtype != LDPC5G_F32 && dn_dtype != LDPC5G_F64))
        return fail(LDPC5G_ESIZE, "bad dtype");
    if (T > 1 && ldg < m.max_E) return fail(LDPC5G_ESIZE, "bad stride ldg=%lld (max E %lld)", (long long)ldg, (long long)m.max_E);
    if (T == 0) return LDPC5G_OK;
    if (!llr || !llr_dn) return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = m.upload(st)) return rc;
    int max_cb_E = 0;
    for (const SchGeo& g : m.geo) max_cb_E = std::max(max_cb_E, std::max(g.s.E_lo, g.s.E_hi));
    const SchDev s0{};
    if (int rc = launch_raterecover(dim3((unsigned)m.rows.size()), llr, llr_dtype, ldg, s0, m.dgeo(), m.drows(),
                                    harq_in, llr_dn, dn_dtype, max_cb_E, st))
        return rc;
    return m.release();
}

int ldpc5g_sch_decode_multi(const void* llr, int32_t llr_dtype, int64_t ldg,
                            const ldpc5g_sch_cfg_t* cfgs, int32_t T, const void* harq_in,
                            void* llr_dn, int32_t dn_dtype, int8_t* ck, uint8_t* status,
                            int32_t* iters, int32_t L, double alpha, double beta, int32_t schedule,
                            int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok, uint32_t* tb_rem,
                            uint8_t* tb_ok, void* stream) {
    clear_error();
    SchMulti m;
    if (int rc = m.build(cfgs, T)) return rc;
    if ((llr_dtype != LDPC5G_F32 && llr_dtype != LDPC5G_F64) || (dn_dtype != LDPC5G_F32 && dn_dtype != LDPC5G_F64))
        return fail(LDPC5G_ESIZE, "bad dtype");
    if (T > 1 && (ldg < m.max_E || ldb < m.max_B))
        return fail(LDPC5G_ESIZE, "bad strides ldg=%lld ldb=%lld (max E %lld, max B %d)", (long long)ldg, (long long)ldb, (long long)m.max_E, m.max_B);
    if (T == 0) return LDPC5G_OK;
    if (!llr || !llr_dn || !ck || !status || !iters || !tbblk || !cb_crc_ok || !tb_rem || !tb_ok)
        return fail(LDPC5G_ESIZE, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = m.upload(st)) return rc;
    const SchDev s0{};
    const int rows = (int)m.rows.size();
    int max_cb_E = 0;
    for (const SchGeo& g : m.geo) max_cb_E = std::max(max_cb_E, std::max(g.s.E_lo, g.s.E_hi));
    if (int rc = launch_raterecover(dim3(rows), llr, llr_dtype, ldg, s0, m.dgeo(), m.drows(), harq_in, llr_dn,
                                    dn_dtype, max_cb_E, st))
        return rc;
    // every codeblock with its own (bgn, Zc): the mixed-Zc decoder (<= 2 launches)
    std::vector<ldpc5g_cb_desc_t> desc(rows);
    for (int r = 0; r < rows; ++r) {
        const SchGeo& G = m.geo[m.rows[r].t];
        const int c = m.rows[r].c;
        desc[r].bgn = G.s.bgn, desc[r].Zc = G.s.Zc;
        desc[r].llr_off = G.dn_off + (int64_t)c * G.s.N, desc[r].ck_off = G.dck_off + (int64_t)c * G.dck_ld;
    }
    if (int rc = ldpc5g_decode_ms_mixed(desc.data(), rows, llr_dn, dn_dtype, ck, status, iters, L, alpha, beta,
                                        schedule, LDPC5G_RATE_MATCHED, stream))
        return rc;
    if (int rc = check_hip(hipMemsetAsync(tb_rem, 0, (size_t)T * 4, st), "hipMemsetAsync")) return rc;
    hipLaunchKernelGGL(tb_check_kernel, dim3(rows), dim3(kCrcNT), 0, st, (const int8_t*)ck, (int64_t)0, s0,
                       m.dgeo(), m.drows(), tbblk, ldb, cb_crc_ok, tb_rem);
    hipLaunchKernelGGL(tb_ok_kernel, dim3((T + 255) / 256), dim3(256), 0, st, (const uint32_t*)tb_rem, tb_ok, (int)T);
    if (int rc = check_hip(hipGetLastError(), "tb_check launch")) return rc;
    return m.release();
}

}  // extern "C"
